"""BASELINE config 5: RRT*-Connect on synth-fractal-4096 (one tree pair per GPU).

  python tools/config5.py --max-time 20 [--algorithm 5] [--batch 4096] [--out f.json]
  torchrun --nproc-per-node N tools/config5.py ...   (N independent restarts, best path
                                                       shared by one all_gather)

Start (1.0, L/2) and goal 8 m further along +x (the first STANCE-valid points
scanning outward / inward in 0.02 m steps; z = 0.375 + ground, v = (1,0,0)).
Reports time to first solution, the best connection's cost, rewires, and the
engine work rates (pair checks / s, extends / s) of the anytime RRT*-Connect.
algorithm 5 (default): the search resident on the device (buildRRTStarConnectDevice:
neighbourhoods, insertion connect checks and the ordered choose-parent / rewire
replay in HBM); algorithm 1: the host-driven batched loop (round 1's figure).
bench.py's config5 sub-record calls run_config5().
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import planner, sharding  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


def first_valid(T, x, y, step, n=400):
    xs = x + step * np.arange(n)
    xy = np.stack([xs, np.full(n, y)], 1)
    h = T.height_host(xy)[0]
    st = np.zeros((n, 8))
    st[:, 0], st[:, 1], st[:, 2], st[:, 3] = xs, y, 0.375 + h, 1.0
    v, _, _ = T.valid_states(torch.from_numpy(st), gbp.STANCE)
    k = int(np.argmax(v.cpu().numpy() > 0))
    return st[k]


STAGES = ("half", "stages 0-3: targets, extends' search, pair checks, select, append",
          "stage 6: neighbourhoods (k_star_count with its scan, k_star_fill), the connect "
          "checks and their pair checks (k_star_check)",
          "stage 7 on its own stream: k_star_replay (+ k_star_rank after Tb's halves)",
          "stages 4-5: connects' search, k_connect, append (with the shared list)",
          "stage 6 up to its pair checks: k_star_count, k_star_fill",
          "stage 6's connect checks (actions and pair checks, k_star_check)")


def stage_split(data, start, goal, batch, max_time, seed, device):
    """The same run again with per-half timing events (gbp_plan_stage_timing):
    microseconds per half-iteration of each stage group; stage 7 runs beside
    stages 4-5 and the next half, so the groups do not add up to the half
    (and stage 6's two parts are inside stage 6)."""
    out = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=max_time,
                                        seed=seed, device=device, device_loop=True,
                                        stage_timing=True)
    nh = max(1, int(out["stage_halves"]))
    split = {name: round(us / nh, 2) for name, us in zip(STAGES, out["stage_us"])}
    return {"us_per_half": split, "timed_halves": int(out["stage_halves"]),
            "halves": int(out["halves"]),
            # stage 6 less its pair checks: k_star_count, k_star_fill
            "k_star_on_caller_stream_us_per_half": round(split[STAGES[2]] - split[STAGES[6]], 2),
            "k_star_replay_side_stream_us_per_half": split[STAGES[3]],
            "source": "hipEvents per half on the streams the stages run on (a second run of "
                      "the same length with timing on)"}


def run_config5(terrain="synth-fractal-4096", batch=4096, max_time=20.0, seed=20251020, span=8.0,
                algorithm=5, rank=0, world=1, device=0, data=None, split=False):
    """One RRT*-Connect run per rank (seed + rank), best path all_gathered;
    returns the record (rank 0's view) for every rank.  split: add the
    per-stage time split (a second timed run).  (bench.py adds the CPU
    baseline: the oracle's RRT* loop.)"""
    dev = torch.device("cuda", device)
    t0 = time.perf_counter()
    if data is None:
        data = td.by_name(terrain)
    t_gen = time.perf_counter() - t0
    T = gbp.Terrain.from_data(data, device=device)
    L = data.x[-1]
    start = first_valid(T, 1.0, L / 2, 0.02)
    goal = first_valid(T, 1.0 + span, L / 2, -0.02)
    out = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=max_time,
                                        seed=seed + rank, device=device,
                                        device_loop=algorithm == 5)
    found = bool(out["found"])
    cost = out["path_cost"] if found else float("nan")
    who, best = sharding.gather_best_path(cost, out["path_length"], 0.0,
                                          out["states"] if found else None,
                                          out["actions"] if found else None, device=dev)
    ttf = torch.tensor([out["time_to_first"] if found else float("inf")], dtype=torch.float64,
                       device=dev)
    work = torch.tensor([float(out["attempts_checked"]), float(out["rewires"]),
                         float(out["connects"]), float(out["extends"]), float(out["total_time"])],
                        dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ttf, op=dist.ReduceOp.MIN)
        t_max = work[4:].clone()
        dist.all_reduce(work, op=dist.ReduceOp.SUM)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        work[4] = t_max[0]
    b = sharding.unpack_path(best)
    wall = float(work[4].item())
    extra = {}
    if split and algorithm == 5:
        extra["stage_split"] = stage_split(data, start, goal, batch, max_time, seed + rank, device)
    return {**extra,
        "config": "5: RRT*-Connect, %s, %d GPU(s), %d draws per half, %.1f s anytime" % (
            terrain, world, batch, max_time),
        "planner": "buildRRTStarConnectDevice (search resident on the device)" if algorithm == 5
                   else "buildRRTStarConnectBatched (host-driven insertion replay)",
        "terrain_gen_s": round(t_gen, 2),
        "start": start[:3].tolist(), "goal": goal[:3].tolist(),
        "start_state": start.tolist(), "goal_state": goal.tolist(), "seed": seed, "batch": batch,
        "time_to_first_solution_s": float(ttf.item()),
        "best_cost": b["cost"], "best_rank": who, "best_path_states": int(b["states"].shape[0]),
        "pair_checks_per_s": round(float(work[0].item()) / wall, 1),
        "extends_per_s": round(float(work[3].item()) / wall, 1),
        "rewires": int(work[1].item()), "connect_checks": int(work[2].item()),
        "extends": int(work[3].item()),
        "rank0": {k: out[k] for k in ("iterations", "halves", "targets", "extends",
                                      "attempts_checked", "connects", "vertices_a", "vertices_b",
                                      "rewires", "solutions", "total_time", "time_to_first",
                                      "fragile_resolved", "status_reads")},
    }


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrain", default="synth-fractal-4096")
    p.add_argument("--batch", type=int, default=4096)
    p.add_argument("--max-time", type=float, default=20.0)
    p.add_argument("--seed", type=int, default=20251020)
    p.add_argument("--span", type=float, default=8.0)
    p.add_argument("--algorithm", type=int, default=5, choices=(1, 5))
    p.add_argument("--out", default=None)
    p.add_argument("--split", action="store_true", help="add the per-stage time split")
    a = p.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    res = run_config5(a.terrain, a.batch, a.max_time, a.seed, a.span, a.algorithm, rank, world, local,
                      split=a.split)
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.out:
            with open(a.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
