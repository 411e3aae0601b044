#!/bin/bash
# ad-hoc GPU session: planner tests, rocprof passes, a 1024^2 TTFS run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest -m gpu -q -x tests/test_gpu_planner.py > gpurun_out/pytest_planner.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_planner.log
case $rc in 0|1) ;; *) exit $rc;; esac
PROF_TAG=r01b bash tools/profile.sh || exit $?
timeout -k 10 300 python tools/ttfs.py --terrain synth-rough-1024 --batches 43690 --seeds 1 --max-time 150 --out gpurun_out/ttfs1024b.jsonl > gpurun_out/ttfs1024b.log 2>&1 || exit $?
cat gpurun_out/ttfs1024b.log
