#!/bin/bash
# One GPU session: parity tests, then a short bench.  Stops at the first
# GPU fault / abort / timeout (exit 124, 134, 137, 139); assertion failures
# (pytest exit 1) do not stop the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:--m gpu -q -x tests}
BENCH_ARGS=${BENCH_ARGS:---steps 10 --warmup 2 --cpu-seconds 10}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
case $rc in 0|1|5) ;; *) echo "stopping after pytest rc=$rc"; exit $rc;; esac
timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
