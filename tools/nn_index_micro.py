"""The planner's targets' nearest-neighbour search on dumped planner trees
(tools/tree_dump.py): gbp_tree_nearest_dev through the tree's index
(k_nnq_bucket + k_nn_pruned + k_nn_reduce_idx) against the full filtered scan
(k_nn_filter + k_nn_reduce), HIP events on the launch stream, results
compared bit for bit.  --tail: the fraction of the tree appended after the
index was built (scanned in full)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


def timed(fn, launches):
    st = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(launches)]
    for e0, e1 in ev:
        e0.record(st)
        fn()
        e1.record(st)
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--trees", default="gpurun_out/trees.npz")
    p.add_argument("--names", default="a_5000,a_15000,b_15000")
    p.add_argument("--tail", type=float, default=0.05)
    p.add_argument("--launches", type=int, default=20)
    a = p.parse_args()
    d = np.load(a.trees)
    data = td.synth_rough(1024)
    T = gbp.Terrain.from_data(data, device=0)
    qh = d["queries"]
    q = torch.from_numpy(np.ascontiguousarray(qh)).cuda()
    ws = gbp.PlanWorkspace(T, q.shape[0])
    for name in a.names.split(","):
        V = d[name]
        n = V.shape[0]
        k = n - int(round(a.tail * n))
        plain = gbp.DeviceTree(V[0], device=0, capacity=n + 16)
        plain.append(V[1:], np.zeros((n - 1, 10)), np.zeros(n - 1, np.int32))
        idx_t = gbp.DeviceTree(V[0], device=0, capacity=n + 16)
        idx_t.append(V[1:k], np.zeros((k - 1, 10)), np.zeros(k - 1, np.int32))
        nidx = idx_t.build_index(data.bounds)
        idx_t.append(V[k:], np.zeros((n - k, 10)), np.zeros(n - k, np.int32))
        r0 = ws.nearest(plain, q)
        r1 = ws.nearest(idx_t, q)
        torch.cuda.synchronize()
        ms0 = timed(lambda: ws.nearest(plain, q), a.launches)
        ms1 = timed(lambda: ws.nearest(idx_t, q), a.launches)
        print(json.dumps({"tree": name, "vertices": n, "indexed": nidx, "queries": int(q.shape[0]),

                          "ms_filter": round(ms0, 4), "ms_index": round(ms1, 4),
                          "match": bool(torch.equal(r0, r1))}), flush=True)


if __name__ == "__main__":
    main()
