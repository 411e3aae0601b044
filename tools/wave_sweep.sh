#!/bin/bash
# Headline protocol at each (waves, streams): bench.py's validate-only legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=${SWEEP_OUT:-gpurun_out/wave_sweep.jsonl}
: > $OUT
for w in ${WAVES:-2 3}; do
  for s in ${STREAMS:-1 2 4}; do
    timeout -k 10 120 python bench.py --steps 50 --warmup 5 --waves $w --streams $s --ttfs-runs 0 \
        --lookup-micro 0 --config2 0 --cpu-seconds 0 --out gpurun_out/ws.json > gpurun_out/ws.log 2>&1 \
      || { echo "bench w=$w s=$s failed"; tail -5 gpurun_out/ws.log; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ws.json'));print(json.dumps({'waves':$w,'streams':$s,'value':d['value'],'value_serial':d['value_serial'],'kernel_ms':d['kernel_ms_per_launch'],'frac':d['roofline']['frac']}))" | tee -a $OUT
  done
done
