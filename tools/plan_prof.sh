#!/bin/bash
# Kernel-trace profile of a device-loop planner run (tools/plan_run.py) and its
# top kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${PLAN_TIME:-8}
for nn in 0; do
  d=gpurun_out/pp_$nn
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 tools/plan_run.py --max-time $T > $d.log 2>&1 || { echo "run nn=$nn failed"; tail -5 $d.log; exit 1; }
  grep found $d.log
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: -float(x["TotalDurationNs"]))
for x in r[:18]:
    print(f'{int(x["Calls"]):8d} {float(x["AverageNs"]) / 1e3:9.2f}us {float(x["TotalDurationNs"]) / 1e9:7.3f}s {x["Name"][:90]}')
PY
  find $d -name "*kernel_trace.csv" -delete  # the stats are enough; traces of 8-s runs exceed gpurun's copy-back
done
