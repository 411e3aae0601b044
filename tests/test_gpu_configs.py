"""BASELINE configs 4 and 5 on the HIP path (GPU).

Config 4 — "1024x1024 rough_terrain, 8 independent restart trees sharded
1-per-GPU, RCCL best-path allgather" (rrt_connect.cpp:350-425):
world-size-2 processes (gloo here; bench.py runs the same code over RCCL), both
on cuda:0, each running one independent tree pair of the device-resident
planner (seed + rank), then the sized best-path exchange
(sharding.gather_best_path: all_reduce(MAX) of the path lengths, one
all_gather, argmin of path_cost).  Every rank must hold the same argmin record
(ties to the lowest rank), and the record's path must pass the oracle's edge
checks.  Two pairs: config 2's (synth-rough-256) and config 4's own terrain
with the goal on the start side of the 0.55-m step at x = 7.0 (the SURVEY
pair's goal lies past it and past a 0.65-m drop at x = 11.2:
tools/wall_check.py).

Config 5 — "4096x4096 synthetic fractal terrain, RRT*-Connect rewire with
k-nearest wavefront scan" (rrt_star_connect.cpp:12-75): pair-check and
neighbourhood parity against the oracle on synth-fractal-4096 (whose
coordinate vectors leave no LDS for the attempt rows, so the kernels compute
coordinates from the verified affine form), then a short RRT*-Connect run
whose path passes the edge checks.
"""
import os
import socket

import numpy as np
import pytest

import oracle
from global_body_planner_amd import _lib as L
from global_body_planner_amd import terrain_data as td
from tests.helpers import same_f64, assert_pairs_equal, attempts_oracle, resolver, u32

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _config4_worker(rank, world, port, q, name, xy, batch):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import global_body_planner_amd as gbp
        from global_body_planner_amd import planner, sharding
        data = td.by_name(name)
        T = gbp.Terrain.from_data(data, device=0)
        h = T.height_host([[xy[0], xy[1]], [xy[2], xy[3]]])[0]
        start = planner.start_goal_state(h[0], xy[0], xy[1])
        goal = planner.start_goal_state(h[1], xy[2], xy[3])
        out = planner.plan_rrt_connect_device(data, start, goal, batch=batch, max_time=60.0,
                                              seed=20251019 + rank, post_process=True)
        cost = out["path_cost"] if out["found"] else float("nan")
        best, brec = sharding.gather_best_path(cost, out["path_length"], 0.0,
                                               out["states"] if out["found"] else None,
                                               out["actions"] if out["found"] else None)
        u = sharding.unpack_path(brec)
        q.put((rank, bool(out["found"]), cost, best, u["cost"], u["states"].numpy(),
               u["actions"].numpy(), start, goal))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,xy,batch", [
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1024),
    # config 4's own terrain, the goal on the start side of the 0.55-m step at
    # x = 7.0 (bench.py TTFS_PAIRS "synth-rough-1024-near", tools/wall_check.py)
    ("synth-rough-1024", (1.0, 10.23, 6.8, 10.23), 8192),
    # ... and at config 3's own per-half draws (SURVEY's 43,690 targets after
    # the STANCE filter: bench.py's planner batch, tests/test_gpu_oracle_scale.py)
    ("synth-rough-1024", (1.0, 10.23, 6.8, 10.23), 92749),
])
def test_config4_restart_trees_best_path_allgather(gpu, name, xy, batch):
    import torch.multiprocessing as mp
    from tests.test_gpu_planner import check_path
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, 2, port, q, name, xy, batch))
             for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] for r in res), "every restart tree pair found a path"
    costs = [r[2] for r in res]
    want = int(np.argmin(costs))  # ties -> lowest rank
    for r in res:
        assert r[3] == want and r[4] == costs[want]
        assert np.array_equal(r[5], res[0][5]) and np.array_equal(r[6], res[0][6])
    data = td.by_name(name)
    O = oracle.OracleTerrain.from_data(data)
    S, A = res[0][5], res[0][6]
    out = {"found": 1, "states": S, "actions": A,
           "path_duration": float(np.sum(A[:, 6] + A[:, 7]))}
    check_path(O, out, res[0][7], res[0][8])
    print(f"config 4 (2 ranks, {name}): costs {costs}, best rank {want}, {len(S)} states")


def _early_stop_worker(rank, world, port, q, batch):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import global_body_planner_amd as gbp
        from global_body_planner_amd import planner, sharding
        data = td.synth_rough(1024)
        T = gbp.Terrain.from_data(data, device=0)
        # rank 0: the pair before the wall (solved in milliseconds); rank 1:
        # SURVEY's pair across the walls (unsolved in 20 s)
        gx = 6.8 if rank == 0 else 19.42
        h = T.height_host([[1.0, 10.23], [gx, 10.23]])[0]
        start = planner.start_goal_state(h[0], 1.0, 10.23)
        goal = planner.start_goal_state(h[1], gx, 10.23)
        out = planner.plan_rrt_connect_device(data, start, goal, batch=batch, max_time=30.0,
                                              seed=20251019 + rank,
                                              stop_poll=sharding.stop_together("cpu"))
        q.put((rank, out["found"], out["polls"], out["stopped_by_peer"], out["status_reads"],
               out["total_time"], out["halves"]))
    finally:
        dist.destroy_process_group()


def test_config4_early_stop(gpu):
    """Config 4's optional early termination: after each group
    of half-iterations every rank posts its found flag with one
    all_reduce(MAX); a rank whose own search is far from a solution stops
    within one group of the other rank's first solution (same number of
    polls), instead of running out its 30-s budget."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_early_stop_worker, args=(r, 2, port, q, 8192)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, f0, p0, s0, _, t0, h0), (r1, f1, p1, s1, _, t1, h1) = res
    assert f0 == 1 and f1 == 0
    assert p0 == p1 >= 1               # the same polls: stopped in the same group
    assert s0 == 0 and s1 == 1         # rank 1 was stopped by rank 0's solution
    assert t1 < 10.0                   # not its 30-s budget
    print(f"early stop: rank 0 solved after {h0} halves ({t0:.3f} s), rank 1 stopped after "
          f"{h1} halves ({t1:.3f} s), {p0} polls each")


def _throughput_worker(rank, world, port, q, per_rank, seed):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import global_body_planner_amd as gbp
        from global_body_planner_amd import sharding
        from global_body_planner_amd import workload as W
        T = gbp.Terrain.from_data(td.synth_rough(256), device=0)
        base, n = sharding.weak_shard(rank, per_rank)
        s, a, d, _, _ = W.make_attempts(T, n, seed, index_base=base)
        r = T.validate_pairs(s, a, d)
        torch.cuda.synchronize()
        c = u32(r.counts).astype(np.int64)
        gv = int(((c & 0xFFFF) + (c >> 16)).sum())
        el, sums = sharding.reduce_run(0.5 + rank, [n, int(r.valid.sum().item()), gv], "cpu")
        q.put((rank, el, sums, r.valid.cpu().numpy(), r.s_new.cpu().numpy(), r.t_new.cpu().numpy(),
               u32(r.flags), u32(r.counts)))
    finally:
        dist.destroy_process_group()


def test_engine_weak_sharding_world2(gpu):
    """The throughput configs' multi-GPU path on the engine: two
    ranks (gloo, both on cuda:0) each generate their weak shard
    [r B, (r + 1) B) of the Philox stream on the device and validate it; the
    only cross-rank traffic is reduce_run (MAX time, SUM counters).  The summed
    counters equal the single-process 2B batch, and each rank's outputs are
    bit-identical to the matching half of that batch."""
    import global_body_planner_amd as gbp
    import torch.multiprocessing as mp
    from global_body_planner_amd import workload as W
    per, seed = 16384, W.CONFIG_SEEDS[2]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_throughput_worker, args=(r, 2, port, q, per, seed)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    T = gbp.Terrain.from_data(td.synth_rough(256), device=0)
    s, a, d, _, _ = W.make_attempts(T, 2 * per, seed)
    ref = T.validate_pairs(s, a, d)
    torch.cuda.synchronize()
    rv, rsn, rtn = ref.valid.cpu().numpy(), ref.s_new.cpu().numpy(), ref.t_new.cpu().numpy()
    rf, rc = u32(ref.flags), u32(ref.counts)
    c = rc.astype(np.int64)
    want = [2.0 * per, float(rv.sum()), float(((c & 0xFFFF) + (c >> 16)).sum())]
    for r in res:
        assert r[1] == 1.5 and r[2] == want   # MAX of the elapsed times, SUM of the counters
        sl = slice(r[0] * per, (r[0] + 1) * per)
        assert np.array_equal(r[3], rv[sl]) and np.array_equal(r[6], rf[sl])
        assert np.array_equal(r[7], rc[sl])
        sn_set = (rf[sl] & L.F_SNEW_SET) != 0
        tn_set = (rf[sl] & L.F_TNEW_SET) != 0
        assert np.array_equal(r[4][sn_set].view(np.uint64), rsn[sl][sn_set].view(np.uint64))
        assert np.array_equal(r[5][tn_set].view(np.uint64), rtn[sl][tn_set].view(np.uint64))
    print(f"weak shards: 2 x {per} attempts, {int(want[1])} valid, {int(want[2])} lookups")


_fractal = {}


def fractal_pair():
    import global_body_planner_amd as gbp
    if not _fractal:
        data = td.synth_fractal(4096)
        _fractal["v"] = (data, gbp.Terrain.from_data(data, device=0),
                         oracle.OracleTerrain.from_data(data))
    return _fractal["v"]


@pytest.mark.parametrize("adaptive", [False, True])
def test_config5_fractal4096_pair_parity(gpu, adaptive):
    data, T, O = fractal_pair()
    assert T.get_option(L.OPT_COORD_MODE) == 2   # computed (affine) coordinates
    oracle.set_scan_mode(1)
    try:
        n = 24000
        s, a, d, _, _ = attempts_oracle(O, n, seed=4096 + int(adaptive), nthreads=16)
        res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d),
                               adaptive=adaptive)
        gpu_t = (res.valid.cpu().numpy(), res.s_new.cpu().numpy(), res.t_new.cpu().numpy(),
                 u32(res.flags), u32(res.counts))
        ref = O.validate_pairs(s, a, d, adaptive=adaptive, nthreads=16)
        nres = assert_pairs_equal(gpu_t, ref, f"fractal ad{adaptive}",
                                  resolve=resolver(T, s, a, d, adaptive))
        assert ref[0].sum() > 0
        print(f"config 5 parity: {n} attempts bit-exact ({int(ref[0].sum())} valid, {nres} "
              f"re-decided), adaptive {adaptive}")
    finally:
        oracle.set_scan_mode(0)


def test_config5_fractal4096_neighbourhoods(gpu):
    """PlannerClass::neighborhoodDist (planner_class.cpp:173-182, RRT*'s rewire
    set, delta = 3.0) on fractal-4096 states: the k_neighbors wavefront scan
    against the oracle, ascending index, truncation counted."""
    import global_body_planner_amd as gbp
    data, T, O = fractal_pair()
    verts, _ = O.sample_states(4000, 77, 1, 0, L.STANCE, 256, nthreads=16)
    q, _ = O.sample_states(700, 78, 2, 0, L.STANCE, 256, nthreads=16)
    vt, qt = torch.from_numpy(verts).cuda(), torch.from_numpy(q).cuda()
    for radius in (3.0, 8.0):
        out, cnt = gbp.neighbors(qt, vt, radius, max_out=64)
        ro, rc = oracle.neighbors_batch(q, verts, radius, max_out=64, nthreads=16)
        assert np.array_equal(cnt.cpu().numpy(), rc)
        got = out.cpu().numpy()
        for i in range(q.shape[0]):
            k = min(int(rc[i]), 64)
            assert np.array_equal(got[i, :k], ro[i, :k]), i
    assert rc.max() > 0


@pytest.mark.parametrize("n_nearest", [1, 8, 64])
def test_config5_fractal4096_knn(gpu, n_nearest):
    """PlannerClass::neighborhoodN (planner_class.cpp:151-171) — config 5's
    "k-nearest wavefront scan" (k_knn, gbp_knn_batch_dev) — on fractal-4096
    states against the oracle: the heap's pop order (ascending distance,
    ties by ascending index), indices and distances bit for bit; exact
    duplicate vertices (ties), a tree smaller than N, NaN components."""
    import global_body_planner_amd as gbp
    data, T, O = fractal_pair()
    verts, _ = O.sample_states(30000, 77, 1, 0, L.STANCE, 256, nthreads=16)
    q, _ = O.sample_states(1500, 78, 2, 0, L.STANCE, 256, nthreads=16)
    verts[1000:1200] = verts[5000:5200]        # exact duplicates: ties
    verts[20000:20100] = q[:100]               # queries' own states (distance 0)
    verts[::997, 3] = np.nan                   # NaN distances order last
    q = np.concatenate([q, verts[[5000, 5001, 7]], np.full((1, 8), np.nan)])
    for nv in (verts.shape[0], 40, 1):
        vt, qt = torch.from_numpy(np.ascontiguousarray(verts[:nv])).cuda(), torch.from_numpy(q).cuda()
        idx, dist = gbp.knn(qt, vt, n_nearest)
        ri, rd = oracle.knn_batch(q, verts[:nv], n_nearest, nthreads=16)
        assert np.array_equal(idx.cpu().numpy(), ri), (nv, n_nearest)
        assert np.all(same_f64(dist.cpu().numpy(), rd)), (nv, n_nearest)
    # a query equal to the duplicated vertex 5000 (== vertex 1000): the lower index first
    idx, _ = gbp.knn(torch.from_numpy(q[-4:-3]).cuda(), torch.from_numpy(verts).cuda(), n_nearest)
    assert idx.cpu().numpy()[0, 0] == 1000
    print(f"k-nearest N={n_nearest}: {q.shape[0]} queries x {verts.shape[0]} vertices bit-exact")


def test_config5_rrt_star_fractal4096(gpu):
    from global_body_planner_amd import planner
    from tests.test_gpu_planner import check_path
    data, T, O = fractal_pair()
    y = float(data.y[-1]) / 2
    xy = np.array([[1.0 + 0.02 * k, y] for k in range(200)])
    st = np.zeros((200, 8))
    st[:, :2] = xy
    st[:, 2] = 0.375 + T.height_host(xy)[0]
    st[:, 3] = 1.0
    v, _, _ = T.valid_states_host(st, L.STANCE)
    start = st[int(np.argmax(v))]
    xy2 = np.array([[9.0 - 0.02 * k, y] for k in range(200)])
    st2 = st.copy()
    st2[:, :2] = xy2
    st2[:, 2] = 0.375 + T.height_host(xy2)[0]
    v2, _, _ = T.valid_states_host(st2, L.STANCE)
    goal = st2[int(np.argmax(v2))]
    out = planner.plan_rrt_star_connect(data, start, goal, batch=256, max_time=4.0, seed=20251020)
    check_path(O, out, start, goal)
    assert out["solutions"] >= 1 and out["rewires"] > 0
    print(f"config 5 RRT*: first solution {out['time_to_first']:.3f} s, cost {out['path_cost']:.3f}, "
          f"{out['rewires']} rewires, {out['vertices_a'] + out['vertices_b']} vertices")


@pytest.mark.parametrize("n_nearest", [1, 8, 64])
def test_knn_cost_add_yaw(gpu, n_nearest):
    """neighborhoodN with cost_add_yaw set (planner_class.cpp:157-158): the
    yaw-weighted key poseDistance * lw + stateYawDistance * yw scanned on the
    device (k_knn<true>, gbp_knn_yaw_batch_host: yaws with glibc on the host)
    against the oracle, indices and keys bit for bit; ties, NaN, a tree
    smaller than N, two weightings (params.yaml:17-20 defaults 1 / 1)."""
    import global_body_planner_amd as gbp
    data, T, O = fractal_pair()
    verts, _ = O.sample_states(20000, 81, 1, 0, L.STANCE, 256, nthreads=16)
    q, _ = O.sample_states(600, 82, 2, 0, L.STANCE, 256, nthreads=16)
    verts[1000:1200] = verts[5000:5200]        # exact duplicates: ties
    verts[::997, 4] = np.nan                   # NaN keys order last
    verts[7, 3:5] = 0.0                        # atan2(0, 0)
    q = np.concatenate([q, verts[[5000, 7]], np.full((1, 8), np.nan)])
    for lw, yw in ((1.0, 1.0), (0.7, 3.0)):
        for nv in (verts.shape[0], 40, 1):
            idx, dist = gbp.knn_yaw(q, verts[:nv], n_nearest, lw, yw)
            ri, rd = oracle.knn_yaw_batch(q, verts[:nv], n_nearest, lw, yw, nthreads=16)
            assert np.array_equal(idx, ri), (nv, n_nearest, lw)
            assert np.all(same_f64(dist, rd)), (nv, n_nearest, lw)
    print(f"yaw-weighted k-nearest N={n_nearest}: {q.shape[0]} queries x {verts.shape[0]} bit-exact")
