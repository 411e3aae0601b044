#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${NN_VARIANTS:-0 6 7 8 9}; do for g in ${NN_GRIDS:-4 8}; do
  echo "variant $v grid $g"
  GBP_NN_VARIANT=$v GBP_NN_GRID=$g timeout -k 10 90 python3 -u tools/nn_micro.py --verts 5000,20000 2>&1 | grep verts || exit 1
done; done
