#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python tools/sweep.py --kernels persistent --waves 2 --grid 8 --block 256 --sched 1:0,3:8,3:16,3:32,3:64,3:128 --rounds 5 > gpurun_out/sweep.txt 2>&1; rc=$?
cat gpurun_out/sweep.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --kernels persistent --waves 2 --grid 8 --block 256 --sched 1:0,3:16,3:32 --rounds 3 --batch 65536 > gpurun_out/sweep64k.txt 2>&1; rc=$?
cat gpurun_out/sweep64k.txt
exit $rc
