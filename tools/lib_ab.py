"""Interleaved A/B of libgbp.so builds in ONE process (cdna_hip_programming.md
§5.4 rule 24): each build gets its own handle on the same terrain and the same
resident attempt batch; every build is timed in each of R rounds (HIP events
on the launch stream, validate kernel only), rounds interleaved; decisions,
counts and s_new must agree across builds.

    python tools/lib_ab.py ab_libs/libgbp_old.so ab_libs/libgbp_new.so --waves 3
    python tools/lib_ab.py global_body_planner_amd/lib/libgbp.so --opts "lds:LDS_COORDS=1;cm2:LDS_COORDS=0"

--opts: named option sets (GBP_OPT_* names without the prefix) applied to
every library's handle in turn, as further variants of the same interleaving.
"""
import argparse
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
    p.add_argument("libs", nargs="+")
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--coarse", type=int, default=0,
                   help="subsample the terrain to every k-th grid line (same extent, "
                        "k-times coarser cells): a map small enough for the LDS-terrain variant")
    p.add_argument("--batch", type=int, default=262144)
    p.add_argument("--seed", type=int, default=W.CONFIG_SEEDS[3])
    p.add_argument("--waves", default="3")
    p.add_argument("--rounds", type=int, default=7)
    p.add_argument("--launches", type=int, default=10)
    p.add_argument("--out", default=None)
    p.add_argument("--opts", default="", help="'name:OPT=v,OPT=v;name2:...' option variants")
    a = p.parse_args()
    data = td.by_name(a.terrain)
    if a.coarse > 1:
        k = a.coarse
        h = float(data.x[1] - data.x[0]) * k
        sub = lambda g: None if g is None else np.ascontiguousarray(g[::k, ::k])  # noqa: E731
        nx, ny = data.z[::k, ::k].shape
        data = td.TerrainData(np.arange(nx, dtype=np.float64) * h, np.arange(ny, dtype=np.float64) * h,
                              sub(data.z), sub(data.dx), sub(data.dy), sub(data.dz),
                              name=f"{data.name}/coarse{k}")
        print(f"terrain {data.name}: {nx} x {ny}, spacing {h}", flush=True)
    base = gbp.Terrain.from_data(data, device=0)
    s, act, d, _, _ = W.make_attempts(base, a.batch, a.seed)
    Ts = [(os.path.basename(path), gbp.Terrain.from_data(data, device=0, lib=L.load(path)))
          for path in a.libs]
    waves = [int(w) for w in a.waves.split(",")]
    variants = [("", {})]
    if a.opts:
        variants = []
        for part in a.opts.split(";"):
            nm, _, kv = part.partition(":")
            variants.append((nm, {k: int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}))
    Ts = [(f"{name}{'/' + vn if vn else ''}", T, vo) for name, T in Ts for vn, vo in variants]
    keys = [(name, w) for name, _, _ in Ts for w in waves]
    times = {k: [] for k in keys}
    ref = None
    st = torch.cuda.current_stream()
    for r in range(a.rounds):
        for (name, T, vo) in Ts:
            for k, v in vo.items():
                T.set_option(getattr(L, "OPT_" + k), v)
            for w in waves:
                T.set_option(L.OPT_WAVES, w)
                out = T.validate_pairs(s, act, d)
                if r == 0:
                    sig = (out.valid.cpu().numpy().tobytes(), out.counts.cpu().numpy().tobytes(),
                           out.s_new.cpu().numpy().tobytes())
                    if ref is None:
                        ref = sig
                    elif sig != ref:
                        print(f"MISMATCH: {name} w={w}", flush=True)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(a.launches)]
                for e0, e1 in ev:
                    e0.record(st)
                    T.validate_pairs(s, act, d, out=out)
                    e1.record(st)
                torch.cuda.synchronize()
                times[(name, w)].extend(e0.elapsed_time(e1) for e0, e1 in ev)
    rows = []
    for k in keys:
        t = np.array(times[k])
        rows.append({"lib": k[0], "waves": k[1], "median_ms": round(float(np.median(t)), 4),
                     "min_ms": round(float(t.min()), 4)})
    for r in rows:
        print(f"{r['lib']:24s} w={r['waves']} median {r['median_ms']:.4f} ms min {r['min_ms']:.4f} ms",
              flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"terrain": a.terrain, "batch": a.batch, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
