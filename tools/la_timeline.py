"""Timeline of the device planner's two streams from a rocprofv3 results
database (tools/plan_run.py under rocprofv3 --kernel-trace): per stream the
busy time, the kernels' mean durations, and how much of the side stream's
work overlaps the caller's stream.  python3 tools/la_timeline.py run_results.db"""
import re
import sqlite3
import sys

import numpy as np


def load(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, stream_id, queue_id, start, end from kernels order by start").fetchall()
    out = []
    for name, sid, qid, s, e in rows:
        m = re.search(r"(k_[a-z0-9_]+|__amd_rocclr_\w+)", name)
        out.append((m.group(1) if m else name[:24], sid, qid, s, e))
    return out


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    merged = []
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                merged.append((cs, ce))
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        merged.append((cs, ce))
    return merged


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s = max(a[i][0], b[j][0])
        e = min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path):
    ks = load(path)
    # the steady state: the middle 80 % of the run
    t0, t1 = ks[0][3], ks[-1][4]
    lo, hi = t0 + 0.1 * (t1 - t0), t0 + 0.9 * (t1 - t0)
    ks = [k for k in ks if k[3] >= lo and k[4] <= hi]
    span = hi - lo
    streams = {}
    for k in ks:
        streams.setdefault(k[2], []).append(k)
    nval = sum(1 for k in ks if k[0] == "k_validate_persistent")
    print(f"window {span / 1e6:.1f} ms, {nval} validate launches (halves): "
          f"{span / 1e3 / max(nval, 1):.1f} us per half")
    busy = {}
    for q, lst in sorted(streams.items(), key=lambda x: -len(x[1])):
        u = union([(k[3], k[4]) for k in lst])
        busy[q] = u
        b = sum(e - s for s, e in u)
        print(f"queue {q}: {len(lst)} launches, busy {b / span:.3f} of the window "
              f"({b / 1e3 / max(nval, 1):.1f} us per half)")
        by = {}
        for k in lst:
            by.setdefault(k[0], []).append((k[4] - k[3]) / 1e3)
        for name, v in sorted(by.items(), key=lambda x: -sum(x[1])):
            print(f"    {name:26s} {len(v):7d} x {np.mean(v):7.1f} us  ({sum(v) / 1e3 / max(nval, 1) * 1e3:6.1f} us per half)")
    qs = list(busy)
    if len(qs) >= 2:
        ov = overlap(busy[qs[0]], busy[qs[1]])
        allu = union([iv for q in qs for iv in busy[q]])
        idle = span - sum(e - s for s, e in allu)
        print(f"overlap of the two busiest queues: {ov / 1e3 / max(nval, 1):.1f} us per half; "
              f"GPU idle (no kernel on any queue): {idle / 1e3 / max(nval, 1):.1f} us per half")


if __name__ == "__main__":
    main(sys.argv[1])
