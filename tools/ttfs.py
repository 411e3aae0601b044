"""Time-to-first-solution sweep of the batched RRT-Connect planner.

  python tools/ttfs.py --terrain synth-rough-256 --batches 1,16,256 --seeds 3 --max-time 30
Prints one JSON line per run (terrain, batch, seed, found, ttfs, iterations,
extends, vertices) and a summary per batch size.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402

PAIRS = {  # first STANCE-valid goal scanning down from L-1 along y = L/2
    "synth-rough-256": ((1.0, 2.55), (4.02, 2.55)),
    "synth-rough-1024": ((1.0, 10.23), (19.42, 10.23)),
    "slope-gridmap": ((1.0, 0.0), (8.0, 0.0)),
    "rough_terrain-gridmap": ((0.0, 0.0), (10.0, 0.0)),  # the launch defaults (BASELINE §2)
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--batches", default="1,64,256,1024")
    p.add_argument("--seeds", type=int, default=3)
    p.add_argument("--seed0", type=int, default=20251018)
    p.add_argument("--max-time", type=float, default=30.0)
    p.add_argument("--out", default=None)
    p.add_argument("--algorithm", type=int, default=3, help="3: the device loop (bench.py's)")
    a = p.parse_args()
    data = td.by_name(a.terrain)
    T = gbp.Terrain.from_data(data, device=0)
    (xs, ys), (xg, yg) = PAIRS[a.terrain]
    h = T.height_host(np.array([[xs, ys], [xg, yg]]))[0]
    start = planner.start_goal_state(h[0], xs, ys)
    goal = planner.start_goal_state(h[1], xg, yg)
    f = open(a.out, "w") if a.out else None
    for b in [int(v) for v in a.batches.split(",")]:
        times = []
        for k in range(a.seeds):
            out = planner.plan_rrt_connect(data, start, goal, batch=b, max_time=a.max_time,
                                           seed=a.seed0 + 7919 * k, algorithm=a.algorithm)
            row = {"terrain": a.terrain, "batch": b, "seed": a.seed0 + 7919 * k,
                   "found": out["found"], "ttfs": out["time_to_first"],
                   "total": out["total_time"], "iterations": out["iterations"],
                   "targets": out["targets"], "extends": out["extends"],
                   "attempts": out["attempts_checked"], "connects": out["connects"],
                   "va": out["vertices_a"], "vb": out["vertices_b"],
                   "n_states": out["n_states"], "path_length": out["path_length"],
                   "extent_a": [round(v, 3) for v in out["extent_a"]],
                   "extent_b": [round(v, 3) for v in out["extent_b"]]}
            print(json.dumps(row), flush=True)
            if f:
                f.write(json.dumps(row) + "\n")
                f.flush()
            times.append(out["time_to_first"] if out["found"] else float("inf"))
        t = np.array(times)
        print(f"# batch {b}: solved {np.isfinite(t).sum()}/{len(t)} median "
              f"{np.median(t):.3f}s times {np.round(t, 3).tolist()}", flush=True)


if __name__ == "__main__":
    main()
