#!/bin/bash
# Config-5 A/B of libgbp.so builds in separate processes (tools/config5.py,
# 10-s runs), builds interleaved per round; restores the in-tree library.
#   bash tools/c5_lib_ab.sh ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
LIB=global_body_planner_amd/lib/libgbp.so
cp $LIB /tmp/libgbp_orig.so
for r in $(seq 1 $R); do
  for l in "$@"; do
    cp "$l" $LIB
    out=$(timeout -k 10 120 python3 tools/config5.py --max-time ${C5_TIME:-10} --split 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["pair_checks_per_s"]/1e6,1), [round(v,1) for v in d["stage_split"]["us_per_half"].values()])')
    echo "$(basename $l) $out"
  done
done
cp /tmp/libgbp_orig.so $LIB
