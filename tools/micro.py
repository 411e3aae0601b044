"""Microbenchmarks of the engine's building blocks on synth-rough-1024.

  K1 terrain lookup (BASELINE target: >= 40% of HBM roofline): 2^24 uniform
     in-domain points, algorithmic bytes 56 per lookup (16 B xy in, 32 B of fp64
     z cells, 8 B height out).
  isValidState throughput on sampled states (one state per lane).
Prints one JSON object.
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

HBM_PEAK = 8000.0


def timeit(fn, launches=20, rounds=3):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(launches)]
        for e0, e1 in ev:
            e0.record(st)
            fn()
            e1.record(st)
        torch.cuda.synchronize()
        ts += [e0.elapsed_time(e1) for e0, e1 in ev]
    return float(np.median(ts)), float(np.min(ts))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--points", type=int, default=1 << 24)
    p.add_argument("--states", type=int, default=1 << 20)
    a = p.parse_args()
    data = td.synth_rough(1024)
    T = gbp.Terrain.from_data(data, device=0)
    out = {}
    g = torch.Generator(device="cuda").manual_seed(5)
    x0, xN, y0, yN = data.bounds
    xy = torch.empty((a.points, 2), dtype=torch.float64, device="cuda")
    xy[:, 0].uniform_(x0, xN, generator=g)
    xy[:, 1].uniform_(y0, yN, generator=g)
    h = torch.empty(a.points, dtype=torch.float64, device="cuda")
    import ctypes
    VP = ctypes.c_void_p
    lib = L.load()
    sp = VP(torch.cuda.current_stream().cuda_stream)

    def k1():
        lib.gbp_height_batch_dev(T._h, a.points, VP(xy.data_ptr()), VP(h.data_ptr()), None, None, sp)

    med, mn = timeit(k1)
    alg = 56.0 * a.points
    out["k1_height"] = {"points": a.points, "median_ms": med, "min_ms": mn,
                        "lookups_per_s": a.points / (med * 1e-3),
                        "achieved_GBps_alg": alg / (med * 1e-3) / 1e9,
                        "frac_alg": alg / (med * 1e-3) / 1e9 / HBM_PEAK,
                        "hbm_bytes_min": 24.0 * a.points,
                        "achieved_GBps_min_bytes": 24.0 * a.points / (med * 1e-3) / 1e9}
    st, _ = T.sample_states(a.states, 3, 11, 0)
    v = torch.empty(a.states, dtype=torch.uint8, device="cuda")
    f = torch.empty(a.states, dtype=torch.int32, device="cuda")
    c = torch.empty(a.states, dtype=torch.int32, device="cuda")

    def vs():
        lib.gbp_valid_states_dev(T._h, a.states, VP(st.data_ptr()), None, 1, VP(v.data_ptr()),
                                 VP(f.data_ptr()), VP(c.data_ptr()), sp)

    med, mn = timeit(vs)
    vs_res = T.valid_states(st, 1)
    cc = vs_res[2].to(torch.int64) & 0xFFFFFFFF
    out["valid_states"] = {"states": a.states, "median_ms": med, "min_ms": mn,
                           "states_per_s": a.states / (med * 1e-3),
                           "valid_fraction": float(vs_res[0].float().mean()),
                           "G_per_state": float((cc & 0xFFFF).sum()) / a.states}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
