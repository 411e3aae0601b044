#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ttfs.py --terrain synth-rough-1024 --batches 4096 --seeds 1 --max-time 60 > gpurun_out/ttfs_ext.log 2>&1; rc=$?
cat gpurun_out/ttfs_ext.log
exit $rc
