#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for r in 1 2; do
  for c in default 240 255; do
    if [ $c = default ]; then unset GBP_LA_CUS; else export GBP_LA_CUS=$c; fi
    out=$(timeout -k 10 90 python3 tools/plan_run.py --max-time 20 --batch 92749 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["extends_per_s"]/1e6,1), d["vertices_a"], d["vertices_b"])')
    echo "la_cus $c: $out"
  done
done
