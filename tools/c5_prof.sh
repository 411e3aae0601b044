#!/bin/bash
# Kernel-trace profile of config 5 (tools/config5.py: RRT*-Connect on
# synth-fractal-4096, the device loop) and its kernels, per call and per half.
#   C5_TIME=5 C5_TAG=r06c bash tools/c5_prof.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${C5_TIME:-5}
TAG=${C5_TAG:-c5}
d=gpurun_out/${TAG}_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 tools/config5.py --max-time $T --out $d.json > $d.log 2>&1 || { echo "config5 run failed"; tail -5 $d.log; exit 1; }
cat $d.json
f=$(find $d -name "*kernel_stats.csv" | head -1)
python3 - "$f" "$d.json" <<'PY' | tee gpurun_out/${TAG}_prof_summary.txt
import csv, json, sys
r = list(csv.DictReader(open(sys.argv[1])))
c5 = json.load(open(sys.argv[2]))
halves = c5["rank0"]["halves"]
r.sort(key=lambda x: -float(x["TotalDurationNs"]))
print(f"# config 5, {halves} halves; per-half = total / halves")
star = 0.0
for x in r[:24]:
    tot = float(x["TotalDurationNs"]) / 1e3
    if "k_star_" in x["Name"]:
        star += tot
    print(f'{int(x["Calls"]):8d} {float(x["AverageNs"]) / 1e3:9.2f}us {tot / halves:8.2f}us/half {x["Name"][:80]}')
print(f"k_star_* per half: {star / halves:.2f} us")
PY
if [ -n "$C5_KEEP" ]; then
  python3 tools/c5_trace.py $d | tee -a gpurun_out/${TAG}_prof_summary.txt
  python3 tools/c5_gaps.py $d | tee -a gpurun_out/${TAG}_prof_summary.txt
fi
find $d -name "*kernel_trace.csv" -delete
