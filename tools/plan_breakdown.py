"""Mean duration per position in the device planner's half-iteration, from a
rocprofv3 --kernel-trace CSV of tools/plan_run.py (halves start at k_targets, or
after the previous half's second k_append when their targets were drawn ahead);
the last --halves halves."""
import argparse
import csv
import collections
import re


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--halves", type=int, default=4000)
    p.add_argument("--min-kernels", type=int, default=7,
                   help="a half-iteration's kernels from k_targets on (fewer: a cut-off half)")
    a = p.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    halves, cur, appends = [], None, 0
    for r in rows:
        n = r["Kernel_Name"]
        # a half starts at k_targets, or (its targets drawn ahead in the previous
        # half's search) at the first planner kernel after the previous half's
        # second k_append
        if "k_targets" in n or (cur is not None and appends >= 2 and "k_" in n
                                and "copyBuffer" not in n):
            cur = []
            appends = 0
            halves.append(cur)
        if "k_append" in n:
            appends += 1
        if cur is not None:
            short = re.sub(r"^.*?(k_[a-z0-9_]+).*$", r"\1", n.replace("_ZN12_GLOBAL__N_1", ""))
            short = re.sub(r"^\d+", "", short)
            cur.append((short, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    halves = [h for h in halves if len(h) >= a.min_kernels][-a.halves:]
    pos = collections.defaultdict(list)
    span = []
    for h in halves:
        for i, (n, s, e) in enumerate(h):
            pos[(i, n)].append((e - s) / 1e3)
        span.append((h[-1][2] - h[0][1]) / 1e3)
    tot = 0.0
    print(f"{'pos':>3} {'kernel':28s} {'calls':>6} {'mean':>8}    {'median':>8} {'p90':>8}")
    for (i, n), v in sorted(pos.items()):
        m = sum(v) / len(v)
        tot += m
        vs = sorted(v)
        med, p90 = vs[len(vs) // 2], vs[min(len(vs) - 1, int(0.9 * len(vs)))]
        print(f"{i:3d} {n:28s} {len(v):6d} {m:8.1f} us {med:8.1f} {p90:8.1f}")
    print(f"sum of kernel means per half {tot:.1f} us; first-start to last-end per half "
          f"{sum(span) / len(span):.1f} us over {len(halves)} halves")


if __name__ == "__main__":
    main()
