"""Fold rocprofv3 CSV output (tools/profile.sh) into per-kernel figures.

HBM traffic per launch of the validate kernel, corrected as
MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts 128-B requests at 64 B, i.e. it reads HALF the
fetched bytes, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
(Infinity-Cache hits are counted in FETCH_SIZE, not excluded.)
Writes <dir>/summary.json and prints a table.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def rows(pattern):
    out = []
    for path in glob.glob(pattern, recursive=True):
        with open(path, newline="") as f:
            out.extend(csv.DictReader(f))
    return out


def main(d):
    summary = {"kernels": {}, "counters": {}}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        name = r.get("Name") or r.get("KERNEL_NAME") or r.get("Kernel_Name")
        summary["kernels"][name] = {
            "calls": int(float(r.get("Calls", 0))),
            "avg_ns": float(r.get("AverageNs", 0)),
            "total_ns": float(r.get("TotalDurationNs", 0)),
            "pct": float(r.get("Percentage", 0)),
        }
    acc = defaultdict(lambda: defaultdict(list))
    for sub in ("fetch", "write", "l2"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        summary["counters"][k] = {c: sum(v) / len(v) for c, v in cs.items()}
    # the headline's launch: the k_validate variant with the longest average
    # dispatch in the trace (the planner's own, if any ran, are shorter)
    kv = sorted((n for n in summary["kernels"] if "k_validate" in n),
                key=lambda n: -summary["kernels"][n]["avg_ns"])
    val = [k for k in kv if k in summary["counters"]] or \
        [k for k in summary["counters"] if "k_validate" in k]
    if val:
        c = summary["counters"][val[0]]
        summary["validate_kernel"] = val[0]
        fetch = c.get("FETCH_SIZE")
        write = c.get("WRITE_SIZE")
        if fetch is not None and write is not None:
            summary["validate_hbm_bytes_per_launch"] = (2.0 * fetch + write) * 1024.0
            summary["validate_fetch_kib_raw"] = fetch
            summary["validate_write_kib_raw"] = write
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            summary["validate_l2_hit_rate"] = hit / (hit + miss)
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if "validate_hbm_bytes_per_launch" in summary:  # what bench.py reads (profiles/pmc_traffic.json)
        k = [summary["validate_kernel"]] if summary.get("validate_kernel") in summary["kernels"] else \
            [n for n in summary["kernels"] if "k_validate" in n]
        with open(os.path.join(d, "pmc_traffic.json"), "w") as f:
            json.dump({"terrain": os.environ.get("PMC_TERRAIN", "synth-rough-1024"),
                       "batch": int(os.environ.get("PMC_BATCH", "262144")),
                       "kernel": k[0][k[0].index("k_validate"):k[0].index("(gbp::")] if k else None,
                       "avg_ns_trace": summary["kernels"][k[0]]["avg_ns"] if k else None,
                       "hbm_bytes_per_launch": summary["validate_hbm_bytes_per_launch"],
                       "fetch_kib_raw": summary.get("validate_fetch_kib_raw"),
                       "write_kib_raw": summary.get("validate_write_kib_raw"),
                       "l2_hit_rate": summary.get("validate_l2_hit_rate"),
                       "correction": "(2*FETCH_SIZE + WRITE_SIZE)*1024, MI355X_MICROARCH.md §HBM",
                       "source": "tools/profile.sh: rocprofv3 --kernel-trace --stats, then separate "
                                 "--pmc FETCH_SIZE / WRITE_SIZE / TCC_HIT,TCC_MISS runs"}, f, indent=1)
    for k, v in sorted(summary["kernels"].items(), key=lambda kv: -kv[1]["total_ns"]):
        print(f"{v['calls']:6d} calls  avg {v['avg_ns'] / 1e3:10.2f} us  {v['pct']:6.2f}%  {k[:90]}")
    for k in ("validate_hbm_bytes_per_launch", "validate_fetch_kib_raw", "validate_write_kib_raw",
              "validate_l2_hit_rate"):
        if k in summary:
            print(k, summary[k])


if __name__ == "__main__":
    main(sys.argv[1])
