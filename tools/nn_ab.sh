#!/bin/bash
# A/B of libgbp.so builds on the planner's nearest-vertex search and the
# planner itself, separate processes, builds interleaved per round: each build
# is copied over the in-tree library in turn.  Usage: tools/nn_ab.sh ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
LIB=global_body_planner_amd/lib/libgbp.so
cp $LIB /tmp/libgbp_orig.so
for r in $(seq 1 $R); do
  for l in "$@"; do
    cp "$l" $LIB
    nn=$(timeout -k 10 60 python3 tools/nn_bench.py --verts ${NN_VERTS:-20000,40000} 2>/dev/null | grep "^nv" | tr '\n' ' ')
    pl=$(timeout -k 10 60 python3 tools/plan_run.py --max-time ${PLAN_TIME:-4} --batch 92749 2>/dev/null | tail -1 | python3 -c 'import json,sys; print(round(json.loads(sys.stdin.read())["extends_per_s"]/1e6,1))')
    echo "$(basename $l) | $nn| planner $pl M/s"
  done
done
cp /tmp/libgbp_orig.so $LIB
