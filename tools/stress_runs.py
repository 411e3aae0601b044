"""Device-loop planners on configurations beyond the bench's, checked only for
running to completion with consistent counters (no oracle at this scale):
RRT-Connect (algorithm 3) at 92,749 draws per half on synth-fractal-4096,
the anytime restarts on the device (algorithm 4) on synth-rough-1024, and
RRT* (algorithm 5) at 16,384 draws per half on synth-fractal-4096, and
RRT* with the adaptive step size on synth-rough-1024.
    python3 tools/stress_runs.py [--seconds 8]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from config5 import first_valid  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=8.0)
    a = p.parse_args()
    runs = [("synth-fractal-4096", 3, 92749, False), ("synth-rough-1024", 4, 43690, False),
            ("synth-fractal-4096", 5, 16384, False), ("synth-rough-1024", 5, 8192, True)]
    for name, alg, batch, adaptive in runs:
        data = td.by_name(name)
        T = gbp.Terrain.from_data(data, device=0)
        L = data.x[-1]
        start = first_valid(T, 1.0, L / 2, 0.02)
        goal = first_valid(T, 9.0, L / 2, -0.02)
        kw = dict(batch=batch, max_time=a.seconds, seed=7, adaptive=adaptive)
        if alg == 5:
            out = planner.plan_rrt_star_connect(data, start, goal, device_loop=True, **kw)
        elif alg == 4:
            out = planner.plan_rrt_connect(data, start, goal, algorithm=4, max_time_opt=a.seconds, **kw)
        else:
            out = planner.plan_rrt_connect(data, start, goal, algorithm=alg, **kw)
        keep = {k: out[k] for k in ("found", "halves", "extends", "attempts_checked", "connects",
                                    "vertices_a", "vertices_b", "fragile_resolved", "total_time")
                if k in out}
        print(json.dumps({"terrain": name, "algorithm": alg, "batch": batch, "adaptive": adaptive, **{
            k: (float(v) if isinstance(v, (np.floating, float)) else int(v)) for k, v in keep.items()}}),
            flush=True)


if __name__ == "__main__":
    main()
