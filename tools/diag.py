"""Time diagnostic builds of the validate kernel against the real one in one
process (interleaved rounds).  Diagnostic builds compute wrong answers on
purpose (no trig / no bracket fix-up) and exist only to price those parts."""
import argparse
import glob
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", type=int, default=3)
p.add_argument("--launches", type=int, default=10)
p.add_argument("--waves", type=int, default=2)
a = p.parse_args()
data = td.synth_rough(1024)
libs = {"real": L.load()}
for path in sorted(glob.glob(os.path.join(ROOT, "global_body_planner_amd", "lib", "diag", "*.so"))):
    libs[os.path.basename(path)[7:-3]] = L.load(path)
Ts = {k: gbp.Terrain.from_data(data, device=0, lib=v) for k, v in libs.items()}
for T in Ts.values():
    T.set_option(L.OPT_WAVES, a.waves)
s, act, d, _, _ = W.make_attempts(Ts["real"], 262144, W.CONFIG_SEEDS[3])
st_states, _ = Ts["real"].sample_states(1 << 20, 3, 11, 0)
times = {k: [] for k in Ts}
vtimes = {k: [] for k in Ts}
htimes = {k: [] for k in Ts}
g = torch.Generator(device="cuda").manual_seed(5)
npts = 1 << 24
xy = torch.empty((npts, 2), dtype=torch.float64, device="cuda")
xy[:, 0].uniform_(data.bounds[0], data.bounds[1], generator=g)
xy[:, 1].uniform_(data.bounds[2], data.bounds[3], generator=g)
st = torch.cuda.current_stream()
for r in range(a.rounds):
    for k, T in Ts.items():
        out = T.validate_pairs(s, act, d)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        for e0, e1 in ev:
            e0.record(st)
            T.validate_pairs(s, act, d, out=out)
            e1.record(st)
        torch.cuda.synchronize()
        times[k] += [e0.elapsed_time(e1) for e0, e1 in ev]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        for e0, e1 in ev:
            e0.record(st)
            T.valid_states(st_states, 1)
            e1.record(st)
        torch.cuda.synchronize()
        vtimes[k] += [e0.elapsed_time(e1) for e0, e1 in ev]
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        for e0, e1 in ev:
            e0.record(st)
            T.height(xy)
            e1.record(st)
        torch.cuda.synchronize()
        htimes[k] += [e0.elapsed_time(e1) for e0, e1 in ev]
        if r == 0:
            c = out.counts.to(torch.int64) & 0xFFFFFFFF
            print(f"{k:16s} valid={int(out.valid.sum())} V={int((c >> 16).sum())}", flush=True)
for k, t in times.items():
    print(f"{k:16s} pairs median {np.median(t):.4f} ms  min {np.min(t):.4f} ms   "
          f"valid_states(1M) median {np.median(vtimes[k]):.4f} ms   "
          f"height(16M) median {np.median(htimes[k]):.4f} ms")
