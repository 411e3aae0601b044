#!/bin/bash
# Config 5 (tools/config5.py, 10-s runs) against one environment knob:
#   KNOB=GBP_NS_GRID bash tools/c5_sweep.sh "32 64 128" ROUNDS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${2:-2}); do
  for v in $1; do
    out=$(env $KNOB=$v timeout -k 10 120 python3 tools/config5.py --max-time ${C5_TIME:-10} 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["pair_checks_per_s"]/1e6,1), round(d["extends_per_s"]/1e6,2), d["rank0"]["halves"])')
    echo "$KNOB $v: $out"
  done
done
