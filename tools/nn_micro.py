"""Nearest neighbour in a device tree (gbp_tree_nearest_dev, the device
loop's k_nn_partial + k_nn_reduce) for the planner's shapes: Q queries against
a tree of V vertices; HIP events on the launch stream; checks the result
against gbp_nearest_batch_dev (the engine's original NN) bit for bit."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--queries", type=int, default=20480)
    p.add_argument("--verts", default="5000,20000")
    p.add_argument("--launches", type=int, default=10)
    a = p.parse_args()
    data = td.synth_rough(1024)
    T = gbp.Terrain.from_data(data, device=0)
    q = T.sample_states(a.queries, seed=3, stream_id=2)[0]
    rows = []
    for nv in [int(v) for v in a.verts.split(",")]:
        T.set_option(gbp._lib.OPT_NN_STATS, 1)
        ws = gbp.PlanWorkspace(T, a.queries)
        vs, _ = T.sample_states(nv, seed=4, stream_id=1)
        vh = vs.cpu().numpy()
        tree = gbp.DeviceTree(vh[0], device=0, capacity=nv + 16)
        tree.append(vh[1:], np.zeros((nv - 1, 10)), np.zeros(nv - 1, np.int32))
        ws.reset()
        idx = ws.nearest(tree, q)
        nst = ws.status()
        T.set_option(gbp._lib.OPT_NN_STATS, 0)
        ws = gbp.PlanWorkspace(T, a.queries)
        ref, _ = gbp.nearest(q, vs)
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
        ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(a.launches)]
        for e0, e1 in ev2:
            e0.record(st)
            gbp.nearest(q, vs)
            e1.record(st)
        torch.cuda.synchronize()
        ms_old = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev2]))
        pairs = a.queries * nv
        rows.append({"queries": a.queries,
                     "verts": nv, "ms": round(ms, 4), "pairs_per_s": round(pairs / (ms * 1e-3), 1),
                     "ms_nearest_batch": round(ms_old, 4), "match": ok,
                     "rechecks_per_query": nst["stat_nn_rechecks"] / a.queries,
                     "scans_per_query": nst["stat_nn_scans"] / a.queries})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
