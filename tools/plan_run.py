"""One device-loop planner run (buildRRTConnectDevice, algorithm 3) on a bench
terrain, for profiling (rocprofv3 --kernel-trace --stats -- python3 tools/plan_run.py)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402

PAIRS = {"synth-rough-1024": ((1.0, 10.23), (19.42, 10.23), 43690),
         "synth-rough-256": ((1.0, 2.55), (4.02, 2.55), 10922),
         "slope-gridmap": ((1.0, 0.0), (8.0, 0.0), 10922)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--batch", type=int, default=0)
    p.add_argument("--max-time", type=float, default=5.0)
    p.add_argument("--seed", type=int, default=20251018)
    p.add_argument("--algorithm", type=int, default=3)
    p.add_argument("--runs", type=int, default=1)
    p.add_argument("--nn-stats", type=int, default=0, help="GBP_OPT_NN_STATS (re-check counters)")
    a = p.parse_args()
    data = td.by_name(a.terrain)
    (xs, ys), (xg, yg), b = PAIRS[a.terrain]
    T = gbp.Terrain.from_data(data, device=0)
    h = T.height_host([[xs, ys], [xg, yg]])[0]
    start = planner.start_goal_state(h[0], xs, ys)
    goal = planner.start_goal_state(h[1], xg, yg)
    for k in range(a.runs):
        out = planner.plan_rrt_connect(data, start, goal, batch=a.batch or b, max_time=a.max_time,
                                       seed=a.seed + k, algorithm=a.algorithm,
                                       nn_stats=a.nn_stats)
        run_t = out["time_to_first"] if out["found"] else out["total_time"]
        print(json.dumps({k2: out[k2] for k2 in ("found", "time_to_first", "total_time", "iterations",
                                                   "extends", "vertices_a", "vertices_b", "targets", "nn_rechecks", "nn_scans",
                                                   "fragile_resolved", "status_reads")}
                         | {"extends_per_s": out["extends"] / max(run_t, 1e-9)}), flush=True)


if __name__ == "__main__":
    main()
