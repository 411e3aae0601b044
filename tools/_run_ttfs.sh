#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest -m gpu -q -x tests/test_gpu_planner.py tests/test_gpu_parity.py > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
exit $rc
