"""Which attempts two builds of libgbp.so decide differently (A/B debugging):
per-field comparison of validate_pairs on the same resident batch, and the
first differing attempts checked against the CPU restatement (oracle)."""
import argparse
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
    p.add_argument("lib_a")
    p.add_argument("lib_b")
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--batch", type=int, default=262144)
    p.add_argument("--seed", type=int, default=W.CONFIG_SEEDS[3])
    p.add_argument("--waves", type=int, default=2)
    a = p.parse_args()
    data = td.by_name(a.terrain)
    base = gbp.Terrain.from_data(data, device=0)
    s, act, d, _, _ = W.make_attempts(base, a.batch, a.seed)
    outs = []
    for path in (a.lib_a, a.lib_b):
        T = gbp.Terrain.from_data(data, device=0, lib=L.load(path))
        T.set_option(L.OPT_WAVES, a.waves)
        o = T.validate_pairs(s, act, d)
        torch.cuda.synchronize()
        outs.append({k: getattr(o, k).cpu().numpy() for k in ("valid", "flags", "counts", "s_new", "t_new")})
    A, B = outs
    snew_a = (A["flags"] & L.F_SNEW_SET) != 0 if hasattr(L, "F_SNEW_SET") else None
    bad = np.zeros(a.batch, bool)
    for k in ("valid", "flags", "counts"):
        m = A[k] != B[k]
        print(k, "differs at", int(m.sum()), "attempts")
        bad |= m
    sn = ~np.all((A["s_new"] == B["s_new"]) | (np.isnan(A["s_new"]) & np.isnan(B["s_new"])), axis=1)
    print("s_new differs at", int(sn.sum()), "(all rows, set or not)")
    idx = np.flatnonzero(bad)[:10]
    for i in idx:
        print(i, "dir", int(d[i]), "A", A["valid"][i], hex(A["flags"][i]), A["counts"][i] & 0xFFFF, A["counts"][i] >> 16,
              "B", B["valid"][i], hex(B["flags"][i]), B["counts"][i] & 0xFFFF, B["counts"][i] >> 16)
    if idx.size:
        import oracle
        O = oracle.OracleTerrain.from_data(data)
        sv = s.cpu().numpy()[idx]
        av = act.cpu().numpy()[idx]
        dv = d.cpu().numpy()[idx]
        v, _, _, f, c = O.validate_pairs(sv, av, dv)
        for j, i in enumerate(idx):
            print("oracle", i, v[j], hex(f[j]), c[j] & 0xFFFF, c[j] >> 16)


if __name__ == "__main__":
    main()
