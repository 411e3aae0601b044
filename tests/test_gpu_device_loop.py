"""The search resident on the device (include/gbp.h "device trees and the
device planner loop"; csrc/gbp_plan.hip) against the host-driven batched
planner it replaces (csrc/host/gbp_planner.cpp buildRRTConnectBatched), and
the device tree / extend-into-tree primitives (SURVEY §8(b) items 4-5,
§8(f) row 1) against the engine's batched primitives and the oracle.

Bar: for the same (seed, batch) the device loop builds the same trees and
returns the same path, bit for bit (same RNG streams, same insertion order,
same FRAGILE re-decisions); every path edge passes the oracle's pair check.
Reference: rrt_connect.cpp:230-314 (runRRTConnect), rrt.cpp:77-102 (extend),
graph_class.cpp:28-42 (addVertex / addEdge), planner_class.cpp:185-200
(getNearestNeighbor).
"""
import numpy as np
import pytest

import oracle
from global_body_planner_amd import _lib as L
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td
from tests.helpers import attempts_oracle, same_f64
from tests.test_gpu_planner import _start_goal, check_path

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.mark.parametrize("name,xy,batch,seed", [
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 64, 11),
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 4096, 3),
    ("slope-gridmap", (1.0, 0.0, 8.0, 0.0), 512, 3),
])
def test_device_loop_equals_host_batched(gpu, name, xy, batch, seed):
    data = td.by_name(name)
    O = oracle.OracleTerrain.from_data(data)
    start, goal = _start_goal(O, *xy)
    host = planner.plan_rrt_connect(data, start, goal, batch=batch, max_time=120.0, seed=seed)
    dev = planner.plan_rrt_connect_device(data, start, goal, batch=batch, max_time=120.0, seed=seed)
    assert host["found"] == 1 and dev["found"] == 1
    check_path(O, dev, start, goal)
    assert np.array_equal(dev["states"], host["states"])
    assert np.array_equal(dev["actions"], host["actions"])
    for k in ("vertices_a", "vertices_b", "targets", "extends", "attempts_checked", "connects",
              "fragile_resolved", "depth_capped"):
        assert dev[k] == host[k], (k, dev[k], host[k])
    assert dev["path_length"] == host["path_length"] and dev["path_cost"] == host["path_cost"]
    assert dev["status_reads"] >= 1
    print(f"{name} batch {batch}: {dev['vertices_a']}+{dev['vertices_b']} vertices, "
          f"{dev['extends']} extends, host {host['time_to_first']:.4f} s, device "
          f"{dev['time_to_first']:.4f} s in {dev['status_reads']} status reads")


@pytest.mark.parametrize("batch,seed", [(4096, 3), (1024, 8)])
def test_device_loop_forced_halts_equal_host_batched(gpu, batch, seed):
    """Halt -> gbp_plan_resolve_host -> resume in every stage.  A FRAGILE
    margin of 1e-5 (GBP_OPT_FRAGILE_EPS; any margin >= 1e-12 leaves results
    unchanged, only more of them are re-decided with glibc) flags about 2 % of
    the state checks, so the targets, extend and connect stages all halt many
    times; k_connect's 1024-workgroup grid (batch 4096) exceeds what is
    resident at once, so workgroups start after the halt was raised in their
    own launch and must still compute their items (gate_seq).  The device
    loop must still equal the host batched planner bit for bit."""
    data = td.synth_rough(256)
    O = oracle.OracleTerrain.from_data(data)
    start, goal = _start_goal(O, 1.0, 2.55, 4.02, 2.55)
    kw = dict(batch=batch, max_time=120.0, seed=seed, fragile_eps=1e-5)
    host = planner.plan_rrt_connect(data, start, goal, **kw)
    dev = planner.plan_rrt_connect_device(data, start, goal, **kw)
    assert host["found"] == 1 and dev["found"] == 1
    check_path(O, dev, start, goal)
    assert np.array_equal(dev["states"], host["states"])
    assert np.array_equal(dev["actions"], host["actions"])
    for k in ("vertices_a", "vertices_b", "targets", "extends", "attempts_checked", "connects",
              "fragile_resolved", "depth_capped"):
        assert dev[k] == host[k], (k, dev[k], host[k])
    assert all(h > 0 for h in dev["halts"][:3]), dev["halts"]   # targets, extend, connect
    print(f"batch {batch}: halts {dev['halts']}, {dev['fragile_resolved']} re-decided, "
          f"{dev['status_reads']} status reads")


def test_device_loop_stance_invalid_start(gpu):
    """SURVEY H12 on the device loop: the STANCE-invalid slope start never grows."""
    data = td.csv_gridmap("slope")
    O = oracle.OracleTerrain.from_data(data)
    start, goal = _start_goal(O, 0.0, 0.0, 8.0, 0.0)
    out = planner.plan_rrt_connect_device(data, start, goal, batch=256, max_time=2.0, seed=1)
    assert out["found"] == 0 and out["vertices_a"] == 1 and out["vertices_b"] > 1


@pytest.mark.parametrize("direction", [0, 1])
def test_extend_into_device_tree(gpu, direction):
    """gbp_extend_tree_host (nearest neighbour, newConfig, acceptance and the
    ordered append on the device) equals the engine's primitives composed on
    the host: gbp_nearest_batch + gbp_extend_batch_host + appends in order; the
    appended vertices' g is g[parent] + poseDistance (graph_class.cpp:36-42)."""
    import global_body_planner_amd as gbp
    data = td.synth_rough(256)
    T = gbp.Terrain.from_data(data, device=0)
    O = oracle.OracleTerrain.from_data(data)
    n_tree, n = 700, 9000
    verts = attempts_oracle(O, n_tree, seed=71)[0]
    # targets near the tree (a perturbed vertex each), so that some extends get
    # closer than their nearest vertex and are appended (rrt.cpp:52-68)
    rng = np.random.default_rng(direction)
    targets = verts[rng.integers(0, n_tree, n)].copy()
    targets[:, :2] += rng.normal(scale=0.4, size=(n, 2))
    targets[:, 3:6] += rng.normal(scale=0.5, size=(n, 3))
    tree = gbp.DeviceTree(verts[0], device=0)
    tree.append(verts[1:], np.zeros((n_tree - 1, 10)), np.arange(n_tree - 1, dtype=np.int32))
    ws = gbp.PlanWorkspace(T, n)
    res, vtx, nres = ws.extend_tree_host(T, tree, targets, direction, seed=5, extend_base=300)
    # the same through the batched primitives
    idx, _ = gbp.nearest(torch.from_numpy(targets).cuda(), torch.from_numpy(verts).cuda())
    idx = idx.cpu().numpy()
    r2, ch2, sn2, an2, c2, f2 = T.extend_host(verts[idx], targets, direction, seed=5,
                                              extend_base=300)
    assert np.array_equal(res, r2)
    keep = np.flatnonzero(r2 != L.TRAPPED)
    assert keep.size > 0
    assert np.array_equal(vtx[keep], n_tree + np.arange(keep.size))
    assert np.all(vtx[r2 == L.TRAPPED] == -1)
    s, a, p, g = tree.read()
    assert s.shape[0] == n_tree + keep.size
    assert np.all(same_f64(s[n_tree:], sn2[keep])) and np.all(same_f64(a[n_tree:], an2[keep]))
    assert np.array_equal(p[n_tree:], idx[keep])
    for j, i in enumerate(keep):
        gp = g[idx[i]] + oracle.pose_distance(verts[idx[i]], sn2[i])
        assert g[n_tree + j] == gp
    print(f"direction {direction}: {keep.size} of {n} extends appended, {nres} re-decided")


def test_device_tree_api(gpu):
    import global_body_planner_amd as gbp
    rng = np.random.default_rng(0)
    root = rng.normal(size=8)
    t = gbp.DeviceTree(root, device=0, capacity=4)
    assert len(t) == 1
    s = rng.normal(size=(20, 8))
    a = rng.normal(size=(20, 10))
    p = np.array([0] + list(range(19)), np.int32)   # a chain: parents appended in the same call
    t.append(s, a, p)                                # grows past the initial capacity
    S, A, P, G = t.read()
    assert len(t) == 21 and np.array_equal(S[0], root) and np.array_equal(S[1:], s)
    assert np.array_equal(A[1:], a) and P[0] == -1 and np.array_equal(P[1:], p)
    acc = 0.0
    for i in range(1, 21):
        acc = acc + oracle.pose_distance(S[P[i]], S[i])
        assert G[i] == G[P[i]] + oracle.pose_distance(S[P[i]], S[i])
    with pytest.raises(L.GbpError):
        t.append(s[:1], a[:1], np.array([99], np.int32))  # parent out of range


def test_tree_nearest_exact(gpu):
    """gbp_tree_nearest_dev (k_nn_mfma + k_nn_hreduce: fp16-split scores on the
    matrix cores, a rigorous threshold and fp64 re-checks)
    returns exactly the fp64 scan's index (gbp_nearest_batch_dev,
    planner_class.cpp:185-200: lowest index among equal distances) on random
    states and on the cases that stress the filter: exact duplicates (ties),
    vertices equal in fp16 / fp32 but distinct in fp64, near-equal distances
    on 1e-8 shells, magnitudes past the fp16 rows' range (|v| >= 128: the
    tree is searched in fp64) and NaN queries (index 0)."""
    import global_body_planner_amd as gbp
    data = td.synth_rough(256)
    T = gbp.Terrain.from_data(data, device=0)
    rng = np.random.default_rng(5)
    nq = 4096
    ws = gbp.PlanWorkspace(T, nq)

    def check(verts, q, label):
        tree = gbp.DeviceTree(verts[0], device=0, capacity=verts.shape[0] + 1)
        n = verts.shape[0]
        tree.append(verts[1:], np.zeros((n - 1, 10)), np.zeros(n - 1, np.int32))
        qt = torch.from_numpy(np.ascontiguousarray(q)).cuda()
        got = ws.nearest(tree, qt).cpu().numpy()
        ref, _ = gbp.nearest(qt, torch.from_numpy(verts).cuda())
        ref = ref.cpu().numpy()
        bad = np.flatnonzero(got != ref)
        assert bad.size == 0, (label, bad[:5], got[bad[:5]], ref[bad[:5]])

    # random states, a tree spanning many chunks
    verts = T.sample_states(20000, seed=41, stream_id=1)[0].cpu().numpy()
    q = T.sample_states(nq, seed=42, stream_id=2)[0].cpu().numpy()
    check(verts, q, "random")
    # odd vertex counts (a chunk ending inside a unit) and a single vertex
    for nv in (4097, 20000 - 63, 1):
        check(np.ascontiguousarray(verts[:nv]), q, f"odd {nv}")
    # far from the origin (|v| near the fp16 rows' bound, and past it: fp64)
    for off in (40.0, 120.0, 300.0, 5000.0):
        sh = np.zeros(8)
        sh[:2] = off
        check(verts + sh, q + sh, f"offset {off}")
    # near-equal distances: 5 vertices on a unit shell around each query, radii
    # 1 + O(1e-8): the scores order them almost at random, only the threshold
    # keeps the fp64 minimiser (tests/test_nn_mfma_bound.py)
    for off in (0.0, 100.0):
        sh = np.zeros(8)
        sh[:2] = off
        dirs = rng.normal(size=(nq, 5, 8))
        dirs /= np.linalg.norm(dirs, axis=2, keepdims=True)
        rad = 1.0 + rng.normal(scale=1e-8, size=(nq, 5, 1))
        shell = np.ascontiguousarray(((q + sh)[:, None, :] + dirs * rad).reshape(-1, 8))
        check(shell, q + sh, f"shell {off}")
    # clusters: 64 centres, 300 vertices each within 1e-9, exact duplicates
    # among them; queries at and near the centres
    base = verts[:64]
    cl = np.repeat(base, 300, axis=0) + rng.normal(scale=1e-9, size=(64 * 300, 8))
    cl[::7] = np.repeat(base, 300, axis=0)[::7]          # exact copies of a centre
    perm = rng.permutation(cl.shape[0])
    cl = np.ascontiguousarray(cl[perm])
    qc = np.repeat(base, nq // 64, axis=0) + rng.normal(scale=1e-10, size=(nq, 8))
    qc[::3] = np.repeat(base, nq // 64, axis=0)[::3]
    check(cl, qc, "clusters")
    # magnitudes beyond the fp16 rows' range, and NaN queries
    big = verts.copy()
    big[::1000, 2] = 3e16
    qn = q.copy()
    qn[::97, 4] = np.nan
    qn[5::101, 0] = 2e16
    check(big, qn, "big/nan")
    # a few queries (the connect stage's): the direct fp64 search k_nn_small
    # takes up to 32, the matrix-core pair the rest; both on the clusters
    # (ties, exact duplicates), NaN and huge queries and a 1-vertex tree
    for nqs in (1, 2, 3, 5, 31, 32, 33):
        check(cl, np.ascontiguousarray(qc[:nqs]), f"few {nqs} clusters")
        check(big, np.ascontiguousarray(qn[:nqs * 97 + 6:97][:nqs]), f"few {nqs} big/nan")
    check(np.ascontiguousarray(verts[:1]), np.ascontiguousarray(q[:3]), "few 3 one vertex")


def test_append_past_capacity_is_reported_not_faulted(gpu):
    """A device-loop append beyond a tree's reserved capacity (the caller's
    job, gbp_tree_reserve) is dropped: status.error bit 1 is set, the gate
    stops every later launch of the sequence (no search reads rows past the
    capacity) and the tree's count stays at its capacity."""
    import global_body_planner_amd as gbp
    data = td.synth_rough(256)
    T = gbp.Terrain.from_data(data, device=0)
    O = oracle.OracleTerrain.from_data(data)
    start, goal = _start_goal(O, 1.0, 2.55, 4.02, 2.55)
    ws = gbp.PlanWorkspace(T, 4096)
    ta = gbp.DeviceTree(start, device=0, capacity=2)
    tb = gbp.DeviceTree(goal, device=0, capacity=2)
    ws.reset(0)
    st = None
    for h in range(40):   # until an extend appends more than one vertex to a 2-row tree
        ws.halves(T, ta, tb, h, 1, 4096, seed=3)
        st = ws.status()
        if st["error"] or st["done"] or st["halt"]:
            break
    assert st["error"] & 2, (st["error"], st["done"], st["halt"])
    assert len(ta) <= 2 and len(tb) <= 2
    torch.cuda.synchronize()
