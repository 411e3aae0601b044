#!/bin/bash
# rocprofv3 passes for the validate kernel (run on the GPU box):
#   1. --kernel-trace --stats  (per-kernel durations)
#   2. --pmc FETCH_SIZE        (own pass: FETCH_SIZE takes 3 TCC slots)
#   3. --pmc WRITE_SIZE        (own pass)
#   4. --pmc TCC_HIT_sum TCC_MISS_sum (L2 hit rate)
# then tools/pmc_traffic.py folds them into gpurun_out/prof/summary.json.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
# --streams 1: every launch serial, so the per-dispatch durations are the
# kernel's own (overlapped launches on several streams stretch each other)
ARGS=${PROF_ARGS:---steps 20 --warmup 3 --cpu-seconds 0 --ttfs-runs 0 --streams 1 --lookup-micro 0 --config2 0 --fresh-batches 0 --config5-seconds 0}
TAG=${PROF_TAG:-run}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o $TAG -- \
    python3 bench.py $ARGS > $OUT/trace_bench.log 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o $TAG -- \
    python3 bench.py $ARGS > $OUT/fetch_bench.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o $TAG -- \
    python3 bench.py $ARGS > $OUT/write_bench.log 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l2 -o $TAG -- \
    python3 bench.py $ARGS > $OUT/l2_bench.log 2>&1 || { echo "l2 pass failed rc=$?"; exit 1; }
python3 tools/pmc_traffic.py $OUT > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
find $OUT -name "*.csv" | head -50
