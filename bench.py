"""Benchmark: batched extend attempts/s on synth-rough-1024 (BASELINE config 3).

A step = one pass of the hot path (gbp_validate_pairs: isValidStateActionPair /
...Reverse for every attempt) over one resident batch of 262,144 attempts per
GPU (s_near ~ randomState | STANCE-valid, action =
getRandomAction(normal at a random target), FORWARD/REVERSE alternating,
seed 20251018).  Inputs are generated on the GPU before timing (Philox-keyed,
so rank r's shard [r*B, (r+1)*B) is the same data wherever it is generated).

Multi-GPU: one process per GPU (torchrun), each rank its own contiguous shard,
no data-path collective ("scaling": "weak"); only the timing max and the
counter sums cross ranks.

The timed region is K back-to-back launches (no events inside), issued
round-robin on `--streams` HIP streams (default 2; the steps are independent
passes, each with its own output buffers, so one launch's ragged end overlaps
the next one's start); the serial single-stream loop is timed too and
reported as `value_serial`.  Step k runs on resident batch k mod
`--fresh-batches` (8 distinct batches of the same distribution, all resident
before timing), so no launch replays the previous one's Infinity-Cache-warm
rows; the one-batch replay rates are reported under `replay`.  A further pass
of K launches bracketed by HIP events on one stream gives the kernel's own
duration for the roofline.

Extra fields: `roofline` for the validate kernel (algorithmic bytes per
SURVEY §8(d): 144 B in + 76 B out + 32 B x (G + V) per attempt, G/V = the
executed getGroundHeight / isValidState calls reported by the kernel itself,
over the HIP-event-timed kernel duration), `cpu_baseline` (the CPU
restatement with the reference's O(N) scans, one host thread, rank 0, N=1),
`cpu_baseline_all_cores` (same, OpenMP over the job's host threads),
`terrain_lookup` (the K1 lookup microbenchmark with its own roofline).
"""
import argparse
import json
import re
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import sharding  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E (MI355X_MICROARCH.md chip table)
BYTES_IN, BYTES_OUT, BYTES_PER_LOOKUP = 144, 76, 32
METRIC = "valid extend-attempts/sec + time-to-first-solution, 1024×1024 rough_terrain"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--batch", type=int, default=262144, help="attempts per GPU per step")
    p.add_argument("--terrain", default="synth-rough-1024")
    p.add_argument("--seed", type=int, default=W.CONFIG_SEEDS[3])
    p.add_argument("--kernel", choices=["persistent", "direct"], default="persistent")
    p.add_argument("--waves", type=int, default=2,
                   help="waves per SIMD of the headline's validate launches (2: best alone and "
                        "overlapped on --streams since the kernel holds one bracket form, "
                        "profiles/r03f_wave_sweep.jsonl)")
    p.add_argument("--streams", type=int, default=2,
                   help="HIP streams the K independent steps are issued on round-robin (1: serial)")
    p.add_argument("--adaptive", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="bounded CPU-baseline sample (0 disables)")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    p.add_argument("--out", default=None, help="also write the JSON line here")
    p.add_argument("--lookup-micro", type=int, default=1,
                   help="also run the K1 terrain-lookup microbenchmark (rank 0)")
    p.add_argument("--ttfs-runs", type=int, default=3,
                   help="batched RRT-Connect runs for time-to-first-solution (0 disables)")
    p.add_argument("--plan-batch", type=int, default=0,
                   help="targets per half-iteration (0: SURVEY §8(d), the config's attempt batch / 6 "
                        "candidates: 43,690 at 1024^2 (256k), 10,923 at 256^2 (64k))")
    p.add_argument("--plan-max-time", type=float, default=20.0, help="seconds per planner run")
    p.add_argument("--plan-algorithm", type=int, default=3,
                   help="3: the search resident on the device (buildRRTConnectDevice), "
                        "0: the host-driven batched loop (buildRRTConnectBatched)")
    p.add_argument("--config5-seconds", type=float, default=10.0,
                   help="config 5 (RRT*-Connect, synth-fractal-4096, the device loop) run "
                        "length per rank; 0 = skip")
    p.add_argument("--config5-batch", type=int, default=4096,
                   help="config 5: randomState draws per half-iteration")
    p.add_argument("--config2", type=int, default=1,
                   help="also measure config 2 (synth-rough-256, 65,536 attempts) (rank 0)")
    p.add_argument("--config2-waves", type=int, default=2,
                   help="waves per SIMD for config 2's 65,536-attempt launches (2: their fill and "
                        "drain dominate; 3 measured slower)")
    p.add_argument("--config2-streams", type=int, default=4,
                   help="HIP streams for config 2's launches (small launches: more overlap pays)")
    p.add_argument("--fresh-batches", type=int, default=8,
                   help="distinct resident batches the timed steps cycle through (1: replay one)")
    return p.parse_args()


def cpu_baseline(data, s, a, d, seconds, threads=1):
    """The oracle (reference algorithm, O(N) scans) on this host: 1 thread (the
    reference's execution model) or `threads` OpenMP threads over attempts."""
    try:
        import oracle
    except Exception as e:  # pragma: no cover
        return {"value": None, "error": f"oracle unavailable: {e}"}
    O = oracle.OracleTerrain.from_data(data)
    oracle.set_scan_mode(0)
    n_total, done, chunk = s.shape[0], 0, 256 * threads
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds and done < n_total:
        hi = min(n_total, done + chunk)
        O.validate_pairs(s[done:hi], a[done:hi], d[done:hi], nthreads=threads)
        done = hi
    dt = time.perf_counter() - t0
    return {"value": round(done / dt, 1), "unit": "extend-attempts/s", "cores": threads,
            "kind": "port",
            "sample": f"first {done} attempts of the same batch on the host CPU "
                      f"({dt:.1f} s, {threads} thread(s), oracle/gbp_oracle.c linear-scan brackets)",
            "host_cpu": _cpu_model(), "host_threads_available": os.cpu_count()}


def terrain_lookup_micro(T, data, dev, points=1 << 24, launches=10):
    """K1 (SURVEY §8(d) 'terrain-lookup microbenchmark', target >= 40 % of HBM
    roofline): 2^24 uniform in-domain points on the bench terrain, 56 algorithmic
    bytes per lookup (16 B xy in, 32 B of z cells, 8 B height out), HIP events
    on the launch stream."""
    import ctypes
    g = torch.Generator(device=dev).manual_seed(5)
    x0, xN, y0, yN = data.bounds
    xy = torch.empty((points, 2), dtype=torch.float64, device=dev)
    xy[:, 0].uniform_(x0, xN, generator=g)
    xy[:, 1].uniform_(y0, yN, generator=g)
    h = torch.empty(points, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    VP = ctypes.c_void_p

    def k1():
        rc = T._lib.gbp_height_batch_dev(T._h, points, VP(xy.data_ptr()), VP(h.data_ptr()), None,
                                         None, VP(st.cuda_stream))
        if rc != 0:
            raise gbp.GbpError(rc, "height_batch")

    k1()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(launches)]
    for e0, e1 in ev:
        e0.record(st)
        k1()
        e1.record(st)
    torch.cuda.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    achieved = 56.0 * points / (ms * 1e-3) / 1e9
    return {"kernel": "k_height", "points": points, "ms_per_launch": round(ms, 4),
            "lookups_per_s": round(points / (ms * 1e-3), 1), "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "bytes_per_lookup": 56, "z_storage": ["auto", "f32", "f64"][T.info()["storage"]]}


# start (1.0, L/2), goal = the first STANCE-valid point scanning
# down from L - 1 along y = L/2; reference wall times (its own
# CPU build, 3 seeds) where it solved
TTFS_PAIRS = {
    "synth-rough-1024": {"start": (1.0, 10.23), "goal": (19.42, 10.23), "reference_s": None,
                         "reference_note": "no solution within 1700 s (BASELINE §2.1)",
                         "batch": 262144 // 6},
    # the same start, the goal on the start side of the 0.55-m step up at x = 7.0
    # (the first STANCE-valid point scanning x down from 6.8 along y = 10.23, as
    # §8(d) scans for the SURVEY goal; tools/wall_check.py)
    "synth-rough-1024-near": {"terrain": "synth-rough-1024", "start": (1.0, 10.23),
                              "goal": (6.8, 10.23), "reference_s": None,
                              "reference_note": "not measured by the survey", "batch": 262144 // 6},
    "synth-rough-256": {"start": (1.0, 2.55), "goal": (4.02, 2.55),
                        "reference_s": [0.05, 1.19, 2.64], "batch": 65536 // 6},
    # config 1: the slope CSV through the grid_map geometry; the
    # reference's own CPU build took 12.0 / 27.0 / 28.8 s (BASELINE §2)
    "slope-gridmap": {"start": (1.0, 0.0), "goal": (8.0, 0.0),
                      "reference_s": [12.0, 27.0, 28.8], "batch": 65536 // 6},
}


def time_to_first_solution(data, name, runs, max_time, args, rank, world, dev, pair_key=None):
    """Batch-synchronous RRT-Connect (include/gbp_planner.h) from the pair's
    start to its goal, z = 0.375 + ground, v = (1, 0, 0).  With N ranks each run
    is config 4: one independent tree pair per GPU (seed + rank), first solution
    = min over ranks, best path shared by one all_gather of the fixed-size record."""
    from global_body_planner_amd import planner
    T = gbp.Terrain.from_data(data, device=dev.index)
    pair = TTFS_PAIRS[pair_key or name]
    xy = torch.tensor([pair["start"], pair["goal"]], dtype=torch.float64, device=dev)
    h = T.height(xy)[0].cpu().numpy()
    xy = xy.cpu().numpy()
    start = planner.start_goal_state(h[0], xy[0, 0], xy[0, 1])
    goal = planner.start_goal_state(h[1], xy[1, 0], xy[1, 1])
    out_runs = []
    best = None
    # each half-iteration "draws enough targets to issue about
    # 256k attempts" (config 3; 64k for configs 1-2): pair["batch"] valid
    # targets x 6 candidates; the draws per half are that many over the
    # terrain's STANCE-valid fraction of randomState draws (isValidState
    # filter, rrt_connect.cpp:254), measured here on 65,536 draws
    q, _ = T.sample_states(65536, seed=args.seed, stream_id=7)
    pv = float(T.valid_states(q, L.STANCE)[0].float().mean().item())
    batch = args.plan_batch or int(round(pair["batch"] / max(pv, 0.05)))
    ext_total, time_total = 0, 0.0
    for k in range(runs):
        # config 4: the ranks' searches stop together at the first solution of
        # any of them (one all_reduce(MAX) per group of half-iterations)
        poll = sharding.stop_together(dev) if world > 1 and args.plan_algorithm == 3 else None
        out = planner.plan_rrt_connect(data, start, goal, batch=batch,
                                       max_time=max_time, algorithm=args.plan_algorithm,
                                       seed=args.seed + 7919 * k + rank, device=dev.index,
                                       stop_poll=poll)
        ttf = out["time_to_first"] if out["found"] else float("inf")
        ext_total += out["extends"]
        time_total += out["time_to_first"] if out["found"] else out["total_time"]
        t = torch.tensor([ttf], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
        out_runs.append({"ttfs_s": float(t.item()), "rank0_iterations": out["iterations"],
                         "rank0_extends": out["extends"],
                         "rank0_extends_per_s": round(out["extends"] / max(
                             out["time_to_first"] if out["found"] else out["total_time"], 1e-9), 1),
                         "rank0_fragile_resolved": out["fragile_resolved"],
                         "rank0_status_reads": out["status_reads"],
                         "rank0_attempts": out["attempts_checked"],
                         "rank0_vertices": out["vertices_a"] + out["vertices_b"],
                         "rank0_tree_x_extent": [round(out["extent_a"][0], 2),
                                                 round(out["extent_a"][1], 2),
                                                 round(out["extent_b"][0], 2),
                                                 round(out["extent_b"][1], 2)]})
        if k == runs - 1:
            # ranked by the reference's path_cost_ (rrt_connect.cpp:304-313, :401)
            cost = out["path_cost"] if out["found"] else float("nan")
            who, rec = sharding.gather_best_path(cost, out["path_length"], 0.0,
                                                 out["states"] if out["found"] else None,
                                                 out["actions"] if out["found"] else None,
                                                 device=dev)
            u = sharding.unpack_path(rec)
            best = {"rank": who, "cost": u["cost"], "n_states": int(u["states"].shape[0])}
    solved = [r["ttfs_s"] for r in out_runs if np.isfinite(r["ttfs_s"])]
    res = {"terrain": name, "pair": pair_key or name,
           "value": float(np.median(solved)) if solved else None, "unit": "s",
           "solved": f"{len(solved)}/{len(out_runs)}", "runs": out_runs, "best_path": best,
           "batch": batch, "stance_valid_fraction": round(pv, 4),
           "targets_per_half": int(round(batch * pv)), "max_time_s": max_time,
           "planner": "buildRRTConnectDevice (search resident on the device)"
                      if args.plan_algorithm == 3 else "buildRRTConnectBatched (host loop)",
           "planner_extends_per_s": round(ext_total / max(time_total, 1e-9), 1),
           "start": [float(v) for v in start[:3]], "goal": [float(v) for v in goal[:3]],
           "reference_s": pair["reference_s"],
           "definition": "wall seconds from the build call's start to the first REACHED "
                         "connect (min over ranks), median over solved runs"}
    if pair.get("reference_note"):
        res["reference_note"] = pair["reference_note"]
    return res


def extend_micro(T, s, tgt, d, seed, launches=10):
    """RRTClass::newConfig + extend acceptance (rrt.cpp:20-102) for B/6 extends
    per launch (config 3: 256k attempts = 43,690 extends of up to 6 candidates):
    candidate actions drawn at the target's surface normal, checked, the closest
    valid one selected (gbp_extend_batch_dev, HIP events on the launch stream)."""
    import ctypes
    n = s.shape[0] // 6
    dev = s.device
    VP = ctypes.c_void_p
    res = torch.empty(n, dtype=torch.int32, device=dev)
    cho = torch.empty(n, dtype=torch.int32, device=dev)
    sn = torch.empty((n, 8), dtype=torch.float64, device=dev)
    an = torch.empty((n, 10), dtype=torch.float64, device=dev)
    cnt = torch.empty(n, dtype=torch.int32, device=dev)
    efl = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    sv, tv, dv = s[:n].contiguous(), tgt[:n].contiguous(), d[:n].contiguous()

    def ext():
        rc = T._lib.gbp_extend_batch_dev(T._h, n, VP(sv.data_ptr()), VP(tv.data_ptr()),
                                         VP(dv.data_ptr()), 0, 0, seed, 0, VP(res.data_ptr()),
                                         VP(cho.data_ptr()), VP(sn.data_ptr()), VP(an.data_ptr()),
                                         VP(cnt.data_ptr()), VP(efl.data_ptr()), VP(st.cuda_stream))
        if rc != 0:
            raise gbp.GbpError(rc, "extend_batch")

    ext()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(launches)]
    for e0, e1 in ev:
        e0.record(st)
        ext()
        e1.record(st)
    torch.cuda.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    adv = int((res != 0).sum().item())
    return {"extends_per_launch": n, "ms_per_launch": round(ms, 4),
            "extends_per_s": round(n / (ms * 1e-3), 1),
            "non_trapped_fraction": round(adv / n, 5),
            "definition": "newConfig (<= 6 candidates, first valid in index order) + the "
                          "closer-than-s_near acceptance, per extend"}



def measure(T, s, a, d, B, res, args, dev, world, streams=None, batches=None):
    """The timed region of the contract: K launches back to back between a
    barrier + synchronize on both sides, issued round-robin on S HIP streams
    (each with its own outputs), then the same K serially on one stream, then K
    launches bracketed by HIP events on the launch stream (the kernel's own
    duration for the roofline).  `batches` (a list of (s, a, d) resident
    batches) makes the serial pass cycle through distinct inputs instead.
    Returns (elapsed_streams, elapsed_serial, kernel_ms)."""
    import ctypes
    VP = ctypes.c_void_p
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    ins = [(VP(x.data_ptr()), VP(y.data_ptr()), VP(z.data_ptr())) for x, y, z in (batches or [(s, a, d)])]
    optr0 = [VP(t.data_ptr()) for t in (res.valid, res.s_new, res.t_new, res.flags, res.counts)]

    def launch(inp, p, st):
        rc = T.validate_pairs_raw(B, inp[0], inp[1], inp[2], 0, int(args.adaptive), p[0], p[1], p[2],
                                  p[3], p[4], VP(st))
        if rc != 0:
            raise gbp.GbpError(rc, "validate_pairs")

    S = max(1, args.streams if streams is None else streams)
    strs = [torch.cuda.Stream(device=dev) for _ in range(S)]
    outs = [res] + [T.validate_pairs(s, a, d, adaptive=args.adaptive) for _ in range(S - 1)]
    optr = [[VP(t.data_ptr()) for t in (o.valid, o.s_new, o.t_new, o.flags, o.counts)] for o in outs]

    def timed(fn):
        for k in range(args.warmup):
            fn(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(args.steps):  # the timed region: K launches back to back
            fn(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    elapsed_serial = timed(lambda k: launch(ins[k % len(ins)], optr0, sp))
    elapsed = timed(lambda k: launch(ins[k % len(ins)], optr[k % S], strs[k % S].cuda_stream)) \
        if S > 1 else elapsed_serial
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    for e0, e1 in ev:
        e0.record(stream)
        launch(ins[0], optr0, sp)
        e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
    return elapsed, elapsed_serial, kern_ms


def config2_line(args, dev):
    """Config 2 (north_star 'extend-attempts/sec on synthetic
    256x256'): synth-rough-256, 65,536 attempts per launch, seed 20251017, the
    same protocol as the headline (streams, serial, HIP-event kernel time,
    roofline, bounded single-thread CPU baseline)."""
    data2 = td.by_name("synth-rough-256")
    T2 = gbp.Terrain.from_data(data2, device=dev.index)
    T2.set_option(L.OPT_WAVES, args.config2_waves)
    B2 = 65536
    s2, a2, d2, _, _ = W.make_attempts(T2, B2, W.CONFIG_SEEDS[2])
    r2 = T2.validate_pairs(s2, a2, d2, adaptive=args.adaptive)
    torch.cuda.synchronize()
    c = r2.counts.to(torch.int64) & 0xFFFFFFFF
    gv = int(((c & 0xFFFF) + (c >> 16)).sum().item())
    batches2 = None  # fresh inputs per step, as the headline
    if args.fresh_batches > 1:
        batches2 = [(s2, a2, d2)] + [W.make_attempts(T2, B2, W.CONFIG_SEEDS[2], index_base=k * B2)[:3]
                                     for k in range(1, args.fresh_batches)]
    el, el_serial, kms = measure(T2, s2, a2, d2, B2, r2, args, dev, 1, streams=args.config2_streams,
                                 batches=batches2)
    byts = B2 * (BYTES_IN + BYTES_OUT) + BYTES_PER_LOOKUP * gv
    ach = byts / (kms * 1e-3) / 1e9
    out = {"workload": "config 2: synth-rough-256, 65,536-attempt batch, isValidStateActionPair"
                       "[Reverse] 50/50, seed 20251017",
           "value": round(B2 * args.steps / el, 1), "unit": "extend-attempts/s",
           "value_serial": round(B2 * args.steps / el_serial, 1),
           "kernel_ms_per_launch": round(kms, 4), "waves": args.config2_waves,
           "streams": args.config2_streams,
           "inputs": f"fresh: step k runs on resident batch k mod {max(1, args.fresh_batches)}",
           "valid_fraction": float(r2.valid.to(torch.int64).sum().item()) / B2,
           "lookups_per_attempt": gv / B2,
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBPS, 4),
                        "algorithmic_bytes_per_launch": byts}}
    if args.cpu_seconds > 0:
        out["cpu_baseline"] = cpu_baseline(data2, s2.cpu().numpy(), a2.cpu().numpy(),
                                           d2.cpu().numpy(), min(args.cpu_seconds, 5.0))
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def config5_cpu_baseline(c5, halves=8):
    """Config 5's CPU baseline: the oracle's RRT*-Connect loop (orc_plan with
    star; the reference's O(N) bracket scans), 1 thread, on the same terrain
    with the same start / goal, seed, streams and draws as the device run,
    from the roots for `halves` half-iterations (~12 s on the GPU box's EPYC)."""
    import oracle
    data = td.by_name("synth-fractal-4096")
    O = oracle.OracleTerrain.from_data(data)
    oracle.set_scan_mode(0)
    b = int(c5["batch"])
    t0 = time.perf_counter()
    r = O.plan(np.array(c5["start_state"]), np.array(c5["goal_state"]), batch=b,
               seed=int(c5["seed"]), max_halves=halves, star=True, stream_a=401, stream_b=402,
               capacity=1 << 16, nthreads=1)
    dt = time.perf_counter() - t0
    return {"value": round(r["attempts"] / dt, 1), "unit": "pair checks/s", "cores": 1,
            "kind": "port", "extends_per_s": round(r["extends"] / dt, 1),
            "sample": f"orc_plan(star) from the roots, {halves} half-iterations x {b} draws "
                      f"({r['attempts']} pair checks, {r['extends']} extends, linear bracket "
                      f"scans) in {dt:.1f} s on {_cpu_model() or 'the host'}"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        # what the process group itself reports (torchrun's WORLD_SIZE is only
        # what the launcher asked for): a SCALE line shows RCCL saw N ranks
        world, backend = dist.get_world_size(), dist.get_backend()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    data = td.by_name(args.terrain)
    T = gbp.Terrain.from_data(data, device=local)
    T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT if args.kernel == "persistent" else L.KERNEL_DIRECT)
    T.set_option(L.OPT_WAVES, args.waves)
    B = args.batch
    base, _ = sharding.weak_shard(rank, B)   # rank r: attempts [r*B, (r+1)*B) of one global stream
    s, a, d, tgt, tries = W.make_attempts(T, B, args.seed, index_base=base)
    res = T.validate_pairs(s, a, d, adaptive=args.adaptive)
    torch.cuda.synchronize()
    # per-launch algorithmic bytes from the kernel's own G/V counters
    c = res.counts.to(torch.int64) & 0xFFFFFFFF
    gv = int(((c & 0xFFFF) + (c >> 16)).sum().item())
    # the kernel fetches all ten probes of every evaluated sample (straight-line
    # isValidState): 10 V probes issued by the charged samples, beside G + V
    probes = 10 * int((c >> 16).sum().item())
    n_valid = int(res.valid.to(torch.int64).sum().item())
    flags = res.flags.to(torch.int64) & 0xFFFFFFFF
    n_ood = int(((flags & L.F_OOD) != 0).sum().item())
    n_frag = int(((flags & L.F_FRAGILE) != 0).sum().item())
    bytes_per_launch = B * (BYTES_IN + BYTES_OUT) + BYTES_PER_LOOKUP * gv

    # every timed step runs on a NEW resident batch (8 distinct batches of the
    # same distribution cycled): no replay of Infinity-Cache-warm rows, as in a
    # planner whose iterations never repeat their inputs
    batches = None
    if args.fresh_batches > 1:
        batches = [(s, a, d)] + [W.make_attempts(T, B, args.seed, index_base=base + k * world * B)[:3]
                                 for k in range(1, args.fresh_batches)]
    replay = None
    if batches is not None:  # (measured first: it also brings the GPU to its clocks)
        el_rp, el_rps, _ = measure(T, s, a, d, B, res, args, dev, world)
        el_rp = sharding.reduce_run(el_rp, [0], dev)[0]
        el_rps = sharding.reduce_run(el_rps, [0], dev)[0]
        replay = {"value": round(B * world * args.steps / el_rp, 1),
                  "value_serial": round(B * world * args.steps / el_rps, 1),
                  "definition": "every step on the same resident batch (round 1's protocol)"}
    elapsed, elapsed_serial, kern_ms = measure(T, s, a, d, B, res, args, dev, world, batches=batches)
    elapsed_serial = sharding.reduce_run(elapsed_serial, [0], dev)[0]
    del batches

    elapsed, sums = sharding.reduce_run(elapsed, [B, n_valid, n_ood, n_frag, gv, probes], dev)
    sums = torch.tensor(sums, dtype=torch.float64)
    tot_attempts = float(sums[0].item()) * args.steps
    value = tot_attempts / elapsed

    ttfs = ttfs2 = ttfs1 = ttfs_near = None
    if args.ttfs_runs > 0:
        ttfs = time_to_first_solution(data, args.terrain, args.ttfs_runs, args.plan_max_time, args,
                                      rank, world, dev) if args.terrain in TTFS_PAIRS else None
        if args.terrain == "synth-rough-1024":
            ttfs_near = time_to_first_solution(data, args.terrain, args.ttfs_runs,
                                               args.plan_max_time, args, rank, world, dev,
                                               pair_key="synth-rough-1024-near")
        # config 2 (synth-rough-256), where the reference has wall times to compare with
        ttfs2 = time_to_first_solution(td.by_name("synth-rough-256"), "synth-rough-256", 3, 20.0,
                                       args, rank, world, dev)
        ttfs1 = time_to_first_solution(td.by_name("slope-gridmap"), "slope-gridmap", 3, 20.0,
                                       args, rank, world, dev)

    config5 = None
    if args.config5_seconds > 0:  # every rank runs one tree pair (config 4/5 style restarts)
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools"))
        from config5 import run_config5
        config5 = run_config5(batch=args.config5_batch, max_time=args.config5_seconds,
                              rank=rank, world=world, device=local, split=world == 1)
        if world == 1 and args.cpu_seconds > 0:
            config5["cpu_baseline"] = config5_cpu_baseline(config5)

    if rank == 0:
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic = None
        if args.traffic_json and os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as f:
                    tj = json.load(f)
                km = re.search(r"<[^,]+, (true|false), (\d+),", tj.get("kernel", ""))
                if (tj.get("terrain") == args.terrain and tj.get("batch") == B and km
                        and int(km.group(2)) == args.waves
                        and (km.group(1) == "true") == bool(args.adaptive)):
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "extend-attempts/s",
            "n_gpus": world,
            "dist_backend": backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "streams": max(1, args.streams),
            "value_serial": round(tot_attempts / elapsed_serial, 1),
            "ms_per_step_serial": round(elapsed_serial / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY §8(d) synth-rough-1024, Philox-keyed attempts)",
            "config": {
                "workload": "config 3: synth-rough-1024, 262,144-attempt batch per GPU, "
                            "isValidStateActionPair[Reverse] 50/50",
                "terrain": args.terrain, "batch_per_gpu": B, "global_batch": int(sums[0].item()),
                "seed": args.seed, "kernel": args.kernel, "waves": args.waves,
                "adaptive": args.adaptive, "terrain_storage": ["auto", "f32", "f64"][T.info()["storage"]],
                "parallelism": f"shard{world} (no collective on the data path)",
            },
            "valid_true_per_s": round(float(sums[1].item()) * args.steps / elapsed, 1),
            "valid_fraction": float(sums[1].item()) / float(sums[0].item()),
            "ood_fraction": float(sums[2].item()) / float(sums[0].item()),
            "fragile": int(sums[3].item()),
            "lookups_per_attempt": float(sums[4].item()) / float(sums[0].item()),
            "probes_issued_per_attempt": float(sums[5].item()) / float(sums[0].item()),
            "kernel_ms_per_launch": round(kern_ms, 4),
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "achieved_per_step_overlapped": round(
                    bytes_per_launch / (elapsed / args.steps) / 1e9, 1),
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                "kernel": "k_validate_persistent" if args.kernel == "persistent" else "k_validate_direct",
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "inputs": (f"fresh: step k runs on resident batch k mod {args.fresh_batches} "
                       "(distinct batches of the same distribution)" if replay else "one resident batch"),
            "replay": replay,
            "time_to_first_solution": ttfs,
            "time_to_first_solution_before_wall": ttfs_near,
            "time_to_first_solution_config2": ttfs2,
            "time_to_first_solution_config1": ttfs1,
            "config5": config5,
        }
        if args.lookup_micro:
            out["terrain_lookup"] = terrain_lookup_micro(T, data, dev)
            out["extend_batch"] = extend_micro(T, s, tgt, d, args.seed)
            if ttfs and ttfs.get("planner_extends_per_s"):
                out["planner_vs_extend_batch"] = round(
                    ttfs["planner_extends_per_s"] / out["extend_batch"]["extends_per_s"], 4)
        if args.config2 and world == 1:
            out["config2"] = config2_line(args, dev)
        if world == 1 and args.cpu_seconds > 0:
            s_h, a_h, d_h = s.cpu().numpy(), a.cpu().numpy(), d.cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(data, s_h, a_h, d_h, args.cpu_seconds)
            # all host cores the box gives this job (OMP_NUM_THREADS there), OpenMP
            # over attempts (SURVEY §8(d) CPU baseline (ii))
            nt = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
            out["cpu_baseline_all_cores"] = cpu_baseline(data, s_h, a_h, d_h,
                                                         min(args.cpu_seconds, 5.0), nt)
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
