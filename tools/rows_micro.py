"""Time the persistent validate kernel on a saved set of pair checks
(e.g. config 5's insertion connect actions: python3 tools/rows_micro.py rows.npz)."""
import sys
import os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402

z = np.load(sys.argv[1])
data = td.by_name(sys.argv[2] if len(sys.argv) > 2 else "synth-fractal-4096")
T = gbp.Terrain.from_data(data, device=0)
S = torch.from_numpy(z["S"]).cuda()
A = torch.from_numpy(z["A"]).cuda()
d = torch.zeros(S.shape[0], dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for n in (64, 390, S.shape[0]):
    for opts in ({}, {"HELPERS": 0}):
        for k, v in opts.items():
            T.set_option(getattr(L, "OPT_" + k), v)
        out = T.validate_pairs(S[:n], A[:n], d[:n])
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            T.validate_pairs(S[:n], A[:n], d[:n], out=out)
            e1.record(st)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(n, opts, "median %.4f ms" % np.median(ts), flush=True)
        for k in opts:
            T.set_option(getattr(L, "OPT_" + k), 1)
