#!/bin/bash
# Planner A/B of libgbp.so builds in separate processes: each build is copied
# over the in-tree library in turn (the planner library links it by rpath)
# and runs tools/plan_run.py; rounds alternate the builds.  Restores the
# original library at the end.  Usage: tools/plan_ab.sh ROUNDS lib1.so lib2.so ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$1; shift
LIB=global_body_planner_amd/lib/libgbp.so
cp $LIB /tmp/libgbp_orig.so
for r in $(seq 1 $R); do
  for l in "$@"; do
    cp "$l" $LIB
    out=$(timeout -k 10 120 python3 tools/plan_run.py --max-time ${PLAN_TIME:-5} ${PLAN_ARGS:---batch 87380} 2>/dev/null | tail -1)
    echo "$(basename $l) $out"
  done
done
cp /tmp/libgbp_orig.so $LIB
