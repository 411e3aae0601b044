"""BASELINE configs 4 and 5 on the HIP path (GPU).

Config 4 — "1024x1024 rough_terrain, 8 independent restart trees sharded
1-per-GPU, RCCL best-path allgather" (rrt_connect.cpp:350-425):
world-size-2 processes (gloo here; bench.py runs the same code over RCCL), both
on cuda:0, each running one independent tree pair of the device-resident
planner (seed + rank), then one all_gather of the fixed-size best-path record
(sharding.allgather_best_path).  Every rank must hold the same argmin record
(ties to the lowest rank), and the record's path must pass the oracle's edge
checks.  The config-2 start/goal pair is used: synth-rough-1024's goal sits
beyond the nearest-neighbour-upsampled walls no planner has crossed
(DESIGN.md §8), so a solvable pair is needed to compare paths.

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
from tests.helpers import assert_pairs_equal, attempts_oracle, resolver, u32

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _config4_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import global_body_planner_amd as gbp
        from global_body_planner_amd import planner, sharding
        data = td.synth_rough(256)
        T = gbp.Terrain.from_data(data, device=0)
        h = T.height_host([[1.0, 2.55], [4.02, 2.55]])[0]
        start = planner.start_goal_state(h[0], 1.0, 2.55)
        goal = planner.start_goal_state(h[1], 4.02, 2.55)
        out = planner.plan_rrt_connect_device(data, start, goal, batch=1024, max_time=60.0,
                                              seed=20251019 + rank, post_process=True)
        cost = out["path_cost"] if out["found"] else float("nan")
        rec = sharding.pack_path(cost, out["path_length"], 0.0,
                                 out["states"] if out["found"] else None,
                                 out["actions"] if out["found"] else None)
        best, brec = sharding.allgather_best_path(rec)
        u = sharding.unpack_path(brec)
        q.put((rank, bool(out["found"]), cost, best, u["cost"], u["states"].numpy(),
               u["actions"].numpy(), start, goal))
    finally:
        dist.destroy_process_group()


def test_config4_restart_trees_best_path_allgather(gpu):
    import torch.multiprocessing as mp
    from tests.test_gpu_planner import check_path
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config4_worker, args=(r, 2, port, q)) for r in range(2)]
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
    data = td.synth_rough(256)
    O = oracle.OracleTerrain.from_data(data)
    S, A = res[0][5], res[0][6]
    out = {"found": 1, "states": S, "actions": A,
           "path_duration": float(np.sum(A[:, 6] + A[:, 7]))}
    check_path(O, out, res[0][7], res[0][8])
    print(f"config 4 (2 ranks): costs {costs}, best rank {want}, {len(S)} states")


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
