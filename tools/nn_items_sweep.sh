#!/bin/bash
# Planner (config-3 pair, 92,749 draws per half) against the matrix-core
# search's work items per launch (GBP_NN_ITEMS; default NH_ITEMS = 4096).
#   PLAN_TIME=20 bash tools/nn_items_sweep.sh "4096 2688 5376 8192" ROUNDS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${2:-2}); do
  for n in $1; do
    out=$(GBP_NN_ITEMS=$n timeout -k 10 120 python3 tools/plan_run.py --max-time ${PLAN_TIME:-20} --batch 92749 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["extends_per_s"]/1e6,1), d["vertices_a"], d["vertices_b"])')
    echo "nn_items $n: $out"
  done
done
