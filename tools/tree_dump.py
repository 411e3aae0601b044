"""Grow the device planner loop's trees (gbp_plan_half_dev, the sequence
buildRRTConnectDevice enqueues) on the config-3 pair and save them with a set
of planner-distributed queries, for offline nearest-neighbour analysis
(tools/nn_prune_eval.py): how much of the O(queries x vertices) scan a
bounding-box pruning could skip on the planner's real trees.

    python tools/tree_dump.py --halves 600 --out gpurun_out/trees.npz
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


class PlanStatus(ctypes.Structure):
    """gbp_plan_status (include/gbp.h)."""
    _fields_ = [("halt", ctypes.c_uint32), ("done", ctypes.c_uint32), ("error", ctypes.c_uint32),
                ("halt_half", ctypes.c_int32), ("n_targets", ctypes.c_int32),
                ("n_validate", ctypes.c_int32), ("n_added", ctypes.c_int32),
                ("added_base", ctypes.c_int32), ("n_conn_added", ctypes.c_int32),
                ("meet_half", ctypes.c_int32), ("meet", ctypes.c_uint64),
                ("ext_base", ctypes.c_int64), ("ext_counter", ctypes.c_int64),
                ("stat_targets", ctypes.c_int64), ("stat_attempts", ctypes.c_int64),
                ("stat_added", ctypes.c_int64), ("stat_conn_added", ctypes.c_int64),
                ("stat_fragile_resolved", ctypes.c_int64), ("stat_depth_capped", ctypes.c_int64),
                ("gate_seq", ctypes.c_uint64)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--halves", type=int, default=600)
    p.add_argument("--batch", type=int, default=43690)
    p.add_argument("--seed", type=int, default=20251018)
    p.add_argument("--snapshots", default="5000,15000,50000", help="tree sizes to save")
    p.add_argument("--queries", type=int, default=30000)
    p.add_argument("--out", default="gpurun_out/trees.npz")
    a = p.parse_args()
    lib = L.load()
    data = td.by_name(a.terrain)
    T = gbp.Terrain.from_data(data, device=0)
    h = T.height_host([[1.0, 10.23], [19.42, 10.23]])[0]
    start = planner.start_goal_state(h[0], 1.0, 10.23)
    goal = planner.start_goal_state(h[1], 19.42, 10.23)
    ws = gbp.PlanWorkspace(T, a.batch)
    cap = 1 << 20
    trees = [gbp.DeviceTree(start, capacity=cap), gbp.DeviceTree(goal, capacity=cap)]
    L.check(lib.gbp_plan_reset(ws._h, 0, None), "plan_reset")
    st = PlanStatus()
    snaps = sorted(int(v) for v in a.snapshots.split(","))
    out = {}
    for hh in range(a.halves):
        k = hh & 1
        rc = lib.gbp_plan_half_dev(T._h, ws._h, trees[k]._h, trees[k ^ 1]._h, hh,
                                   L.FORWARD if k == 0 else L.REVERSE, a.batch, a.seed, 101 + k,
                                   (hh >> 1) * a.batch, 0, 0, None)
        L.check(rc, "plan_half")
        L.check(lib.gbp_plan_status_read(ws._h, ctypes.byref(st), None), "status")
        while st.halt:
            kk = st.halt_half & 1
            resume = ctypes.c_int(-1)
            L.check(lib.gbp_plan_resolve_host(T._h, ws._h, trees[kk]._h, trees[kk ^ 1]._h,
                                              L.FORWARD if kk == 0 else L.REVERSE, a.batch, 0,
                                              ctypes.byref(resume), None, None), "resolve")
            L.check(lib.gbp_plan_half_dev(T._h, ws._h, trees[kk]._h, trees[kk ^ 1]._h, st.halt_half,
                                          L.FORWARD if kk == 0 else L.REVERSE, a.batch, a.seed,
                                          101 + kk, (st.halt_half >> 1) * a.batch, 0, resume.value,
                                          None), "resume")
            L.check(lib.gbp_plan_status_read(ws._h, ctypes.byref(st), None), "status")
        if st.done:
            print("solved at half", hh)
            break
        na, nb = len(trees[0]), len(trees[1])
        while snaps and max(na, nb) >= snaps[0]:
            s = snaps.pop(0)
            out[f"a_{s}"] = trees[0].read()[0]
            out[f"b_{s}"] = trees[1].read()[0]
            print(f"half {hh}: snapshot {s}: {na} + {nb} vertices", flush=True)
        if not snaps:
            break
    # queries: the planner's targets (randomState draws, STANCE-valid) of a later index range
    q, _ = T.sample_states(a.queries, a.seed, 101, 10 ** 9)
    v, _, _ = T.valid_states(q, L.STANCE)
    out["queries"] = q[v.bool()].cpu().numpy()
    np.savez_compressed(a.out, **out)
    print("saved", a.out, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
