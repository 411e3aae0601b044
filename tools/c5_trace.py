"""From a rocprofv3 kernel trace of config 5 (tools/c5_prof.sh with C5_KEEP=1):
durations of each half's two pair-check launches (the extends' candidates after
k_la_commit / k_targets, and the insertions' connect checks, k_star_check),
and what ran on the GPU meanwhile.
    python3 tools/c5_trace.py gpurun_out/<tag>_prof"""
import csv
import glob
import sys

import numpy as np

rows = []
for path in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(path, newline="") as f:
        rows.extend(csv.DictReader(f))
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", ""),
              r.get("Grid_Size", ""), r.get("Workgroup_Size", "")) for r in rows))
cand, star = [], []
for s, e, n, q, g, wg in ev:
    if "k_star_check" in n:
        star.append(e - s)
    elif "k_validate_persistent" in n:
        cand.append(e - s)
print("candidate checks: n %d median %.1f us" % (len(cand), np.median(cand) / 1e3 if cand else 0))
print("insertion checks: n %d median %.1f us, p90 %.1f" % (
    len(star), np.median(star) / 1e3 if star else 0, np.percentile(star, 90) / 1e3 if star else 0))
qs = {}
for s, e, n, q, g, wg in ev:
    qs.setdefault(q, 0)
    qs[q] += 1
print("queues:", qs)
print("grid/wg of validate:", {(g, wg) for s, e, n, q, g, wg in ev if "k_validate" in n})
