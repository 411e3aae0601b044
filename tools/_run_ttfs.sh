#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest -m gpu -q -x tests/test_gpu_parity.py > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1|5) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/diag.py --rounds 5 > gpurun_out/diag.txt 2>&1; cat gpurun_out/diag.txt
timeout -k 10 600 python tools/sweep.py --kernels persistent --waves 2,4 --grid 8 --block 256 --sched 1:0,3:0 --rounds 5 > gpurun_out/sweep.txt 2>&1; rc=$?
cat gpurun_out/sweep.txt
exit $rc
