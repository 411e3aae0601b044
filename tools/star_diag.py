"""Diagnostics for the device RRT*-Connect (algorithm 5) against the oracle:
the first half count at which trees / counters differ, per variant."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td

data = td.synth_rough(256)
O = oracle.OracleTerrain.from_data(data)
oracle.set_scan_mode(1)
hs, _ = O.ground_height(1.0, 2.55)
hg, _ = O.ground_height(4.02, 2.55)
start = planner.start_goal_state(hs, 1.0, 2.55)
goal = planner.start_goal_state(hg, 4.02, 2.55)


def same(dev, ref):
    for t in "ab":
        if dev[t]["v"].shape[0] != ref[t]["v"].shape[0]:
            return f"{t} size {dev[t]['v'].shape[0]} vs {ref[t]['v'].shape[0]}"
        for k in ("parent",):
            bad = np.flatnonzero(dev[t][k] != ref[t][k])
            if bad.size:
                return f"{t} {k} first {bad[:5]} dev {dev[t][k][bad[:5]]} ref {ref[t][k][bad[:5]]}"
        bad = np.flatnonzero(dev[t]["g"].view(np.int64) != ref[t]["g"].view(np.int64))
        if bad.size:
            return f"{t} g first {bad[:5]}"
        bad = np.flatnonzero(np.any(dev[t]["act"] != ref[t]["act"], axis=1))
        if bad.size:
            return f"{t} act first {bad[:5]}"
    return None


for halves in [int(h) for h in sys.argv[1:]] or [40, 80, 120, 160, 200, 240, 300]:
    ref = O.plan(start, goal, batch=1024, seed=3, max_halves=halves, star=True, stream_a=401,
                 stream_b=402, nthreads=8)
    for alg, eps in ((1, 1e-5), (5, 1e-5), (5, None)):
        dev = planner.plan_rrt_star_connect(data, start, goal, batch=1024, max_time=600.0, seed=3,
                                            max_halves=halves, trees=True, device_loop=alg == 5,
                                            fragile_eps=eps)
        d = same(dev, ref)
        print(f"halves {halves} alg {alg} eps {eps}: rewires {dev['rewires']} vs {ref['rewires']}, "
              f"attempts {dev['attempts_checked']} vs {ref['attempts']}, connects {dev['connects']} "
              f"vs {ref['connects']}, resolved {dev['fragile_resolved']} halts {dev['halts']}: "
              f"{d or 'same'}", flush=True)
