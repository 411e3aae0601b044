"""Grow config 5's RRT* trees on the device (algorithm 5, synth-fractal-4096,
4096 draws per half) and save them for offline analysis:
    python tools/star_grow_dump.py --halves 15000 --out gpurun_out/c5_trees.npz"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from global_body_planner_amd import planner  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
import oracle  # noqa: E402  (start / goal only: the oracle's isValidState)
from tests.test_gpu_oracle_scale import _first_valid  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--halves", type=int, default=15000)
p.add_argument("--out", default="gpurun_out/c5_trees.npz")
a = p.parse_args()
data = td.by_name("synth-fractal-4096")
O = oracle.OracleTerrain.from_data(data)
oracle.set_scan_mode(1)
L = data.x[-1]
start = _first_valid(O, 1.0, L / 2, 0.02)
goal = _first_valid(O, 9.0, L / 2, -0.02)
g = planner.plan_rrt_star_connect(data, start, goal, batch=4096, max_time=300.0, seed=20251020,
                                  max_halves=a.halves, trees=True, tree_capacity=1 << 17,
                                  device_loop=True)
np.savez_compressed(a.out, start=start, goal=goal, extends=g["extends"], halves=g["halves"],
                    **{f"{t}_{k}": g[t][k] for t in "ab" for k in ("v", "act", "parent", "g")})
print("saved", a.out, len(g["a"]["v"]), len(g["b"]["v"]), g["rewires"])
