#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PROF_TAG=r01c bash tools/profile.sh || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --cpu-seconds 15 --ttfs-runs 1 --plan-max-time 20 > gpurun_out/bench_full.log 2>&1; rc=$?
tail -1 gpurun_out/bench_full.log
exit $rc
