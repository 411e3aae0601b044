"""Interleaved A/B sweep of validate-kernel variants in ONE process
(cdna_hip_programming.md §5.4 rule 24): every variant is timed in each of R
rounds, rounds interleaved; prints median/min ms per launch and checks that
every variant returns bit-identical outputs."""
import argparse
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--batch", type=int, default=262144)
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--launches", type=int, default=10)
    p.add_argument("--kernels", default="direct,persistent")
    p.add_argument("--waves", default="2,3,4")
    p.add_argument("--block", default="256")
    p.add_argument("--lds", default="1", help="coordinates: 0 global, 1 LDS, 2 computed (affine)")
    p.add_argument("--set", action="append", default=[],
                   help="extra option axis KEY=v1,v2 (KEY: an OPT_* name such as PREFETCH, or its id)")
    p.add_argument("--order", default="batch",
                   help="attempt order: batch (as generated), x (sorted by s_near x), xy "
                        "(x-stripes, then y), binsXxY (X x-stripes x Y y-bands, random within)")
    p.add_argument("--adaptive", action="store_true")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    data = td.by_name(a.terrain)
    T = gbp.Terrain.from_data(data, device=0)
    s, act, d, _, _ = W.make_attempts(T, a.batch, W.CONFIG_SEEDS[3])
    if a.order != "batch":  # diagnostic: a position-ordered batch (L2 locality per XCD)
        ext = [float(data.x[0]), float(data.x[-1]), float(data.y[0]), float(data.y[-1])]
        if a.order == "rand":  # a random permutation (scattered rows and outputs)
            g = torch.Generator(device="cpu").manual_seed(7)
            key = torch.randperm(s.shape[0], generator=g).to(s.device).double()
        elif a.order == "x":
            key = s[:, 0]
        elif a.order == "xy":
            key = torch.floor(s[:, 0] / 2.56) * 64 + s[:, 1]
        else:
            bx, by = map(int, a.order[4:].split("x"))
            ix = ((s[:, 0] - ext[0]) / (ext[1] - ext[0]) * bx).floor().clamp(0, bx - 1)
            iy = ((s[:, 1] - ext[2]) / (ext[3] - ext[2]) * by).floor().clamp(0, by - 1)
            key = ix * by + iy
        perm = torch.argsort(key, stable=True)
        s, act = s[perm].contiguous(), act[perm].contiguous()
        d = d[perm].contiguous() if d is not None else d
    variants = []
    for k in a.kernels.split(","):
        for w in (map(int, a.waves.split(",")) if k == "persistent" else [1]):
            for b in map(int, a.block.split(",")):
                for lds in map(int, a.lds.split(",")):
                    variants.append((k, w, b, lds))
    extra_keys, extra_vals = [], []
    for spec in a.set:
        k, vals = spec.split("=")
        extra_keys.append((k, int(k) if k.isdigit() else getattr(L, "OPT_" + k.upper())))
        extra_vals.append([int(x) for x in vals.split(",")])
    variants = [v + (ex,) for v in variants for ex in itertools.product(*extra_vals)]
    times = {v: [] for v in variants}
    ref = None
    ref_chk = None
    st = torch.cuda.current_stream()
    for r in range(a.rounds):
        for v in variants:
            k, w, b, lds, ex = v
            for (_, key), val in zip(extra_keys, ex):
                T.set_option(key, val)
            T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT if k == "persistent" else L.KERNEL_DIRECT)
            T.set_option(L.OPT_WAVES, w)
            T.set_option(L.OPT_LDS_COORDS, 1 if lds == 1 else 0)
            T.set_option(L.OPT_AFFINE_COORDS, 1 if lds == 2 else 0)
            T.set_option(L.OPT_BLOCK, b)
            out = T.validate_pairs(s, act, d, adaptive=a.adaptive)
            if r == 0:
                print(f"variant {v}: coordinate mode {T.get_option(L.OPT_COORD_MODE)}", flush=True)
                sig = (out.valid.cpu().numpy().tobytes(), out.flags.cpu().numpy().tobytes(),
                       out.counts.cpu().numpy().tobytes(), out.s_new.cpu().numpy().tobytes())
                if ref is None:
                    ref = sig
                elif sig != ref:
                    print(f"MISMATCH in variant {v}", flush=True)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(a.launches)]
            for e0, e1 in ev:
                e0.record(st)
                T.validate_pairs(s, act, d, adaptive=a.adaptive, out=out)
                e1.record(st)
            torch.cuda.synchronize()
            # every round's last launch against the first round's outputs
            chk = (int(out.flags.to(torch.int64).sum()), int(out.counts.to(torch.int64).sum()),
                   int((out.s_new.nan_to_num(0.0) * 1e3).to(torch.int64).sum()))
            if ref_chk is None:
                ref_chk = chk
            elif chk != ref_chk:
                print(f"MISMATCH (round {r}) in variant {v}: {chk} vs {ref_chk}", flush=True)
            times[v].extend(e0.elapsed_time(e1) for e0, e1 in ev)
    rows = []
    for v in variants:
        t = np.array(times[v])
        rows.append({"kernel": v[0], "waves": v[1], "block": v[2], "lds": v[3],
                     "set": {name: val for (name, _), val in zip(extra_keys, v[4])},
                     "median_ms": float(np.median(t)), "min_ms": float(t.min()),
                     "attempts_per_s": a.batch / (np.median(t) * 1e-3)})
    rows.sort(key=lambda r: r["median_ms"])
    for r in rows:
        print(f"{r['kernel']:10s} w={r['waves']} b={r['block']} lds={r['lds']} {r['set']} "
              f"median {r['median_ms']:.4f} ms  min {r['min_ms']:.4f} ms  "
              f"{r['attempts_per_s'] / 1e6:.1f} M attempts/s")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"terrain": a.terrain, "batch": a.batch, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
