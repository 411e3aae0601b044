"""The planner's nearest-vertex search on a planner tree (bench_data/trees5.npz:
the trees of a 5-s config-3 run, tools/dump_trees.py) against 43,690 targets:
gbp_tree_nearest_dev timed with HIP events per tree size, result checked
against the fp64 scan.  Run under rocprofv3 --kernel-trace for the split
between k_nn_mfma and k_nn_hreduce."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--verts", default="10000,20000,40000")
    p.add_argument("--launches", type=int, default=20)
    a = p.parse_args()
    z = np.load(os.path.join(ROOT, "bench_data", "trees5.npz"))
    V = np.concatenate([z["a"], z["b"]])
    q = torch.from_numpy(np.load(os.path.join(ROOT, "bench_data", "targets43k.npy"))).cuda()
    T = gbp.Terrain.from_data(td.synth_rough(1024), device=0)
    ws = gbp.PlanWorkspace(T, q.shape[0])
    for nv in [int(v) for v in a.verts.split(",")]:
        vs = np.ascontiguousarray(V[:nv])
        tree = gbp.DeviceTree(vs[0], device=0, capacity=nv + 16)
        tree.append(vs[1:], np.zeros((nv - 1, 10)), np.zeros(nv - 1, np.int32))
        T.set_option(gbp._lib.OPT_NN_STATS, 1)
        ws = gbp.PlanWorkspace(T, q.shape[0])
        ws.reset()
        idx = ws.nearest(tree, q)
        nst = ws.status()
        T.set_option(gbp._lib.OPT_NN_STATS, 0)
        ws = gbp.PlanWorkspace(T, q.shape[0])
        ref, _ = gbp.nearest(q, torch.from_numpy(vs).cuda())
        ok = bool(torch.equal(idx, ref))
        st = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.launches)]
        for e0, e1 in ev:
            e0.record(st)
            ws.nearest(tree, q)
            e1.record(st)
        torch.cuda.synchronize()
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
        print(f"nv {nv}: {ms * 1e3:.1f} us per search (k_nn_mfma + k_nn_hreduce), exact {ok}; re-checked half-chunks {nst['stat_nn_rechecks']}, segment scans {nst['stat_nn_scans']}", flush=True)


if __name__ == "__main__":
    main()
