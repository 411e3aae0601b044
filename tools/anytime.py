"""Anytime restarts of the batched RRT-Connect (algorithm 2, the reference's
buildRRTConnect loop, rrt_connect.cpp:323-467): solutions found and the best
post-processed path cost after max_time_opt, next to the first solution's.

  python tools/anytime.py --terrain synth-rough-256 --opt 2 --seeds 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (start/goal heights only)
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402

PAIRS = {"synth-rough-256": ((1.0, 2.55), (4.02, 2.55)), "slope-gridmap": ((1.0, 0.0), (8.0, 0.0))}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-rough-256")
    p.add_argument("--opt", type=float, default=2.0, help="max_time_opt seconds")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--seeds", type=int, default=3)
    a = p.parse_args()
    data = td.by_name(a.terrain)
    O = oracle.OracleTerrain.from_data(data)
    (xs, ys), (xg, yg) = PAIRS[a.terrain]
    start = planner.start_goal_state(O.ground_height(xs, ys)[0], xs, ys)
    goal = planner.start_goal_state(O.ground_height(xg, yg)[0], xg, yg)
    for k in range(a.seeds):
        seed = 100 + k
        first = planner.plan_rrt_connect_anytime(data, start, goal, max_time_opt=0.0, batch=a.batch,
                                                 max_time=60.0, seed=seed)
        best = planner.plan_rrt_connect_anytime(data, start, goal, max_time_opt=a.opt, batch=a.batch,
                                                max_time=60.0, seed=seed)
        print(json.dumps({"terrain": a.terrain, "seed": seed, "batch": a.batch, "max_time_opt": a.opt,
                          "first_cost": first["path_cost"], "first_ttfs": first["time_to_first"],
                          "best_cost": best["path_cost"], "solutions": best["solutions"],
                          "total_time": round(best["total_time"], 3),
                          "best_states": best["n_states"]}), flush=True)


if __name__ == "__main__":
    main()
