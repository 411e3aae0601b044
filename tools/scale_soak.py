"""Parity soak of the device planner (algorithm 3, the look-ahead search
active) against orc_plan at the bench's batch: several seeds and pairs on
synth-rough-1024, 92,749 draws per half, a fixed number of halves each;
every vertex, action, parent, g and counter compared bit for bit.

    python3 tools/scale_soak.py --seeds 6 --halves 8
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from global_body_planner_amd import planner  # noqa: E402
from tests.test_gpu_oracle_scale import DRAWS, NTHREADS, _compare, _terrain  # noqa: E402
from tests.test_gpu_planner import _start_goal  # noqa: E402

PAIRS = [(1.0, 10.23, 6.8, 10.23), (1.0, 10.23, 19.42, 10.23), (3.0, 4.0, 9.0, 15.0)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seeds", type=int, default=6)
    p.add_argument("--halves", type=int, default=8)
    a = p.parse_args()
    data, O = _terrain()
    bad = 0
    for k in range(a.seeds):
        xy = PAIRS[k % len(PAIRS)]
        seed = 20251018 + 7919 * k
        start, goal = _start_goal(O, *xy)
        t0 = time.time()
        dev = planner.plan_rrt_connect(data, start, goal, algorithm=3, batch=DRAWS, max_time=300.0,
                                       seed=seed, trees=True, tree_capacity=1 << 18,
                                       max_halves=a.halves, nn_stats=True)
        t1 = time.time()
        ref = O.plan(start, goal, batch=DRAWS, seed=seed, max_halves=a.halves, nthreads=NTHREADS)
        t2 = time.time()
        try:
            _compare(dev, ref)
            ok = True
        except AssertionError as e:
            ok = False
            bad += 1
            print("MISMATCH", repr(e)[:500], flush=True)
        print(json.dumps({"seed": seed, "pair": xy, "halves": dev["halves"], "found": dev["found"],
                          "vertices": [len(ref["a"]["v"]), len(ref["b"]["v"])],
                          "targets": ref["targets"], "pair_checks": ref["attempts"],
                          "nn_scans": dev["nn_scans"], "fragile_resolved": dev["fragile_resolved"],
                          "device_s": round(t1 - t0, 2), "oracle_s": round(t2 - t1, 2),
                          "equal": ok}), flush=True)
    print(f"# {a.seeds - bad}/{a.seeds} runs bit-identical", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
