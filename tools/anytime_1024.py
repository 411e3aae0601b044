"""SURVEY's config-3 pair on synth-rough-1024 ((1.0, 10.23) -> (19.42, 10.23))
through the reference's own levers, once: buildRRTConnect's
anytime restarts (rrt_connect.cpp:323-467: fresh trees every restart, horizon
poseDistance / 16 s growing x1.2) with every restart's search resident on the
device (algorithm 4), state_direction_sampling on at params.yaml:21-24's
threshold p = 0.05, 60 s per seed, stopping at the first solution.

  python tools/anytime_1024.py --seeds 3 --max-time 60 > profiles/r04_anytime_1024.jsonl
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seeds", type=int, default=3)
    p.add_argument("--max-time", type=float, default=60.0)
    p.add_argument("--batch", type=int, default=43690)
    p.add_argument("--state-p", type=float, default=0.05)
    a = p.parse_args()
    data = td.synth_rough(1024)
    T = gbp.Terrain.from_data(data, device=0)
    h = T.height_host([[1.0, 10.23], [19.42, 10.23]])[0]
    start = planner.start_goal_state(h[0], 1.0, 10.23)
    goal = planner.start_goal_state(h[1], 19.42, 10.23)
    cfg = L.sampling(state_flag=True, state_p=a.state_p)
    for k in range(a.seeds):
        seed = 20251018 + k
        out = planner.plan_rrt_connect_anytime(data, start, goal, max_time_opt=0.0, device_loop=True,
                                               batch=a.batch, max_time=a.max_time, seed=seed,
                                               sampling=cfg)
        print(json.dumps({"pair": "synth-rough-1024 (1.0, 10.23) -> (19.42, 10.23)", "seed": seed,
                          "algorithm": "buildRRTConnect anytime restarts, device-resident search",
                          "state_direction_sampling": {"flag": True, "p": a.state_p},
                          "batch": a.batch, "max_time_s": a.max_time,
                          "solved": bool(out["found"]),
                          "time_to_first": out["time_to_first"] if out["found"] else None,
                          "total_time": round(out["total_time"], 3),
                          "extends": out["extends"], "iterations": out["iterations"],
                          "last_restart_vertices": [out["vertices_a"], out["vertices_b"]],
                          "last_restart_tree_x_extent": [round(v, 3) for v in
                                                         (out["extent_a"][:2] + out["extent_b"][:2])],
                          "path_cost": out["path_cost"] if out["found"] else None}), flush=True)


if __name__ == "__main__":
    main()
