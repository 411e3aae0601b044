"""Gaps between consecutive kernels on each queue of a rocprofv3 kernel trace
of config 5 (tools/c5_prof.sh with C5_KEEP=1 keeps the trace): per (kernel ->
next kernel) transition on the same queue, the median idle time between the
first one's end and the next one's start.
    python3 tools/c5_gaps.py gpurun_out/<tag>_prof"""
import collections
import csv
import glob
import sys

import numpy as np

rows = []
for path in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(path, newline="") as f:
        rows.extend(csv.DictReader(f))


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    if n.startswith("_ZN12_GLOBAL__N_1"):  # mangled: _ZN12_GLOBAL__N_1<len><name>...
        i = len("_ZN12_GLOBAL__N_1")
        j = i
        while j < len(n) and n[j].isdigit():
            j += 1
        n = n[j:j + int(n[i:j])] if j > i else n
    return n.split("(")[0].split("<")[0][:28]


byq = collections.defaultdict(list)
for r in rows:
    byq[r.get("Queue_Id", "")].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
for q, ev in sorted(byq.items(), key=lambda kv: -len(kv[1])):
    ev.sort()
    gaps = collections.defaultdict(list)
    busy = sum(e - s for s, e, _ in ev)
    span = ev[-1][1] - ev[0][0]
    for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
        gaps[(n0, n1)].append(s1 - e0)
    print(f"queue {q}: {len(ev)} kernels, busy {busy / span:.2f} of its span")
    top = sorted(gaps.items(), key=lambda kv: -len(kv[1]) * np.mean(kv[1]))[:16]
    for (a, b), g in top:
        print(f"  {a:28s} -> {b:28s} n {len(g):6d} median gap {np.median(g) / 1e3:7.2f} us, "
              f"mean {np.mean(g) / 1e3:7.2f} us")
