"""Per-kernel summary (calls, total, mean, median) of a rocprofv3 results
database (rocpd sqlite, rocprofv3's default output): python3 tools/prof_db.py run_results.db"""
import re
import sqlite3
import sys

import numpy as np


def summary(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels").fetchall()
    by = {}
    for name, s, e in rows:
        m = re.search(r"(k_[a-z0-9_]+|__amd_rocclr_\w+)", name)
        key = m.group(1) if m else name[:28]
        if "nn_mfma" in key:  # the template arguments tell the searches apart
            key += "<%s>" % ",".join(re.findall(r"Li(\d+)E|(true|false)", name)[0][:1])
        by.setdefault(key, []).append(e - s)
    out = []
    for k, v in by.items():
        v = np.array(v, np.float64) / 1e3
        out.append((v.sum(), k, len(v), v.mean(), np.median(v)))
    return sorted(out, reverse=True)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(p)
        print("%-28s %8s %12s %10s %10s" % ("kernel", "calls", "total ms", "mean us", "median us"))
        for tot, k, n, m, med in summary(p):
            print("%-28s %8d %12.1f %10.1f %10.1f" % (k[:28], n, tot / 1e3, m, med))
