#!/bin/bash
# Per-kernel breakdown of the device planner's half-iteration: a rocprofv3
# kernel trace of one 5-s planner run (tools/plan_run.py, config 3's pair)
# folded by tools/plan_breakdown.py; writes $OUT (default gpurun_out/plan_breakdown.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/plan_breakdown.txt}
d=gpurun_out/pbd
rm -rf $d
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $d -o run -- \
    python3 tools/plan_run.py --max-time ${PLAN_TIME:-5} ${PLAN_ARGS:-} > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
f=$(find $d -name "*kernel_trace.csv" | head -1)
{ cat $d.log; python3 tools/plan_breakdown.py "$f" --halves ${HALVES:-4000}; } > $OUT
find $d -name "*kernel_trace.csv" -delete
cat $OUT
