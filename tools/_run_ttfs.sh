#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/config5.py --max-time 20 --batch 256 --out gpurun_out/config5.json > gpurun_out/config5.log 2>&1; rc=$?
tail -3 gpurun_out/config5.log
exit $rc
