"""GPU parity: the HIP engine (through the C ABI) against the CPU restatement.

Bar: bit-exact for decisions, flags, lookup counts, s_new and t_new on EVERY
attempt (all FP64 arithmetic is restated in the reference's order without
FMA).  Attempts whose trig-dependent margin is within 1e-12 (GBP_F_FRAGILE)
are re-decided on the host with glibc first (gbp_resolve_fragile_host), as
the product does; none is excluded.  Samplers use device log/sin/cos/acos and
are compared with an explicit relative tolerance (1e-12).
"""
import numpy as np
import pytest

import oracle
from global_body_planner_amd import _lib as L
from global_body_planner_amd import terrain_data as td
from tests.helpers import assert_pairs_equal, attempts_oracle, bits, resolver, same_f64, u32

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TERRAINS = ["synth-rough-256", "slope-gridmap", "rough_terrain-gridmap", "rough_terrain-direct"]
_cache = {}


def terrain_pair(name, **kw):
    import global_body_planner_amd as gbp
    key = (name, tuple(sorted(kw.items())))
    if key not in _cache:
        data = td.by_name(name)
        _cache[key] = (data, gbp.Terrain.from_data(data, device=0, **kw),
                       oracle.OracleTerrain.from_data(data))
    return _cache[key]


@pytest.fixture(autouse=True)
def _bisect():
    oracle.set_scan_mode(1)  # same brackets as the linear scan, faster
    yield
    oracle.set_scan_mode(0)


def np_(t):
    return t.cpu().numpy()


# ---- K1 ----------------------------------------------------------------------
@pytest.mark.parametrize("coords", [1, 2, 0])
@pytest.mark.parametrize("name", TERRAINS)
def test_height_and_normal_parity(gpu, name, coords):
    data, T, O = terrain_pair(name)
    T.set_option(L.OPT_LDS_COORDS, 1 if coords == 1 else 0)
    T.set_option(L.OPT_AFFINE_COORDS, 1 if coords == 2 else 0)
    rng = np.random.default_rng(1)
    x0, xN, y0, yN = data.bounds
    n = 20000
    xy = np.stack([rng.uniform(x0 - 0.3, xN + 0.3, n), rng.uniform(y0 - 0.3, yN + 0.3, n)], 1)
    # grid lines, +-1 ulp around them, and the exact upper edges (reference UB)
    gx = data.x[rng.integers(0, data.x.size, 500)]
    gy = data.y[rng.integers(0, data.y.size, 500)]
    extra = [np.stack([gx, gy], 1), np.stack([np.nextafter(gx, -np.inf), gy], 1),
             np.stack([np.nextafter(gx, np.inf), np.nextafter(gy, np.inf)], 1),
             np.array([[xN, y0], [x0, yN], [xN, yN], [x0, y0]])]
    xy = np.concatenate([xy] + extra)
    h, nan, ood = T.height(torch.from_numpy(xy))
    rh, rnan, rood = O.height_batch(xy, nthreads=8)
    assert np.array_equal(np_(ood), rood)
    assert np.array_equal(np_(nan), rnan)
    assert np.array_equal(bits(np_(h)), bits(rh)) or np.array_equal(
        np.isnan(np_(h)), np.isnan(rh)) and np.array_equal(bits(np_(h)[~np.isnan(rh)]),
                                                           bits(rh[~np.isnan(rh)]))
    nrm, nood = T.normal(torch.from_numpy(xy))
    rn, rnood = O.normal_batch(xy, nthreads=8)
    assert np.array_equal(np_(nood), rnood)
    ok = rnood == 0
    assert np.array_equal(bits(np_(nrm)[ok]), bits(rn[ok]))
    T.set_option(L.OPT_LDS_COORDS, 1)
    T.set_option(L.OPT_AFFINE_COORDS, 1)


def test_height_nan_cells(gpu):
    import global_body_planner_amd as gbp
    data = td.synth_rough(64)
    z = data.z.copy()
    z[10:13, 20:22] = np.nan
    z[40, 5] = np.nan
    T = gbp.Terrain(data.x, data.y, z, data.dx, data.dy, data.dz, device=0)
    O = oracle.OracleTerrain(data.x, data.y, z, data.dx, data.dy, data.dz)
    rng = np.random.default_rng(2)
    xy = np.stack([rng.uniform(0, data.x[-1], 20000), rng.uniform(0, data.y[-1], 20000)], 1)
    h, nan, ood = T.height(torch.from_numpy(xy))
    rh, rnan, rood = O.height_batch(xy)
    assert rnan.sum() > 0
    assert np.array_equal(np_(nan), rnan) and np.array_equal(np_(ood), rood)
    assert np.array_equal(np.isnan(np_(h)), np.isnan(rh))
    ok = ~np.isnan(rh)
    assert np.array_equal(bits(np_(h)[ok]), bits(rh[ok]))
    # validity on the NaN map
    st, _ = O.sample_states(20000, 5, 9, 0, -1, 1, nthreads=8)
    for phase in (L.STANCE, L.FLIGHT):
        v, f, c = T.valid_states(torch.from_numpy(st), phase)
        rv, rf, rc = O.valid_states(st, phase, nthreads=8)
        assert np.array_equal(np_(v), rv)
        assert np.array_equal(u32(f), rf)
        assert np.array_equal(u32(c), rc)
    assert ((rf & L.F_NAN) != 0).sum() > 0


# ---- isValidState ------------------------------------------------------------
@pytest.mark.parametrize("name", TERRAINS)
def test_valid_states_parity(gpu, name):
    data, T, O = terrain_pair(name)
    st, _ = O.sample_states(30000, 11, 7, 0, -1, 1, nthreads=8)
    for phase in (L.STANCE, L.FLIGHT):
        v, f, c = T.valid_states(torch.from_numpy(st), phase)
        rv, rf, rc = O.valid_states(st, phase, nthreads=8)
        m = np.uint32(~(L.F_FRAGILE | L.F_RESOLVED) & 0xFFFFFFFF)
        frag = (u32(f) & L.F_FRAGILE) != 0
        # the host entry re-decides FRAGILE states with glibc: every state matches
        hv, hf, hc = T.valid_states_host(st, phase)
        assert np.array_equal(hv, rv) and np.array_equal(hf & m, rf & m) and np.array_equal(hc, rc)
        assert np.array_equal(np_(v)[~frag], rv[~frag])
        assert np.array_equal(u32(f)[~frag] & m, rf[~frag] & m)
        assert np.array_equal(u32(c)[~frag], rc[~frag])


# ---- K2: the hot path ------------------------------------------------------------
@pytest.mark.parametrize("kernel", [L.KERNEL_DIRECT, L.KERNEL_PERSISTENT])
@pytest.mark.parametrize("adaptive", [False, True])
@pytest.mark.parametrize("name", TERRAINS)
def test_validate_pairs_parity(gpu, name, kernel, adaptive):
    data, T, O = terrain_pair(name)
    T.set_option(L.OPT_KERNEL, kernel)
    n = 20000
    s, a, d, _, _ = attempts_oracle(O, n, seed=123 + len(name))
    res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d),
                           adaptive=adaptive)
    gpu_t = (np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags), u32(res.counts))
    ref = O.validate_pairs(s, a, d, adaptive=adaptive, nthreads=8)
    nfrag = assert_pairs_equal(gpu_t, ref, f"{name}/k{kernel}/ad{adaptive}",
                               resolve=resolver(T, s, a, d, adaptive))
    assert nfrag <= n * 1e-3
    assert ref[0].sum() > 0 or name.startswith("slope")  # some valid pairs are exercised


@pytest.mark.parametrize("kernel", [L.KERNEL_DIRECT, L.KERNEL_PERSISTENT])
@pytest.mark.parametrize("waves", [1, 2, 3, 4])
def test_validate_pairs_register_variants(gpu, kernel, waves):
    data, T, O = terrain_pair("synth-rough-256")
    T.set_option(L.OPT_KERNEL, kernel)
    T.set_option(L.OPT_WAVES, waves)
    try:
        s, a, d, _, _ = attempts_oracle(O, 8192, seed=77)
        res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d))
        gpu_t = (np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags), u32(res.counts))
        assert_pairs_equal(gpu_t, O.validate_pairs(s, a, d, nthreads=8), f"w{waves}",
                           resolve=resolver(T, s, a, d))
    finally:
        T.set_option(L.OPT_WAVES, 2)


@pytest.mark.parametrize("kernel", [L.KERNEL_DIRECT, L.KERNEL_PERSISTENT])
def test_validate_pairs_edge_cases(gpu, kernel):
    """Empty batch, untouched outputs, degenerate stance/flight times, edges."""
    data, T, O = terrain_pair("synth-rough-256")
    T.set_option(L.OPT_KERNEL, kernel)
    empty = T.validate_pairs(torch.empty((0, 8), dtype=torch.float64),
                             torch.empty((0, 10), dtype=torch.float64), L.FORWARD)
    assert empty.valid.numel() == 0
    s, a, d, _, _ = attempts_oracle(O, 4000, seed=5)
    a = a.copy()
    s = s.copy()
    k = np.arange(4000)
    a[k % 7 == 0, 7] = 0.0          # no flight phase
    a[k % 7 == 1, 6] = -0.1         # stance loop never runs (t_s < 0)
    a[k % 7 == 2, 6] = np.nan       # NaN stance time
    a[k % 7 == 3, 7] = 0.05         # exactly one flight sample boundary
    a[k % 7 == 4, 7] = 1e-300       # denormal-ish flight time
    a[k % 13 == 5, 6] = np.inf      # the reference never terminates: engine sample cap
    a[k % 13 == 6, 7] = np.inf
    xN, yN = data.x[-1], data.y[-1]
    s[k % 11 == 0, 0] = xN          # centre exactly at the map edge (UB lookup)
    s[k % 11 == 1, 1] = yN
    s[k % 11 == 2, 0] = data.x[10]  # centre exactly on a grid line
    sentinel = np.full((4000, 8), 12345.0)
    tsent = np.full(4000, -7.0)
    for adaptive in (False, True):
        res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d),
                               adaptive=adaptive, s_new=torch.from_numpy(sentinel),
                               t_new=torch.from_numpy(tsent))
        ref = O.validate_pairs(s, a, d, adaptive=adaptive, s_new_init=sentinel,
                               t_new_init=tsent, nthreads=8)
        gpu_t = (np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags), u32(res.counts))
        assert_pairs_equal(gpu_t, ref, f"edge/ad{adaptive}", resolve=resolver(T, s, a, d, adaptive))
        # rows the reference never assigns keep the caller's contents, bit for bit
        assert np.all(same_f64(gpu_t[1], ref[1]))
        assert np.all(same_f64(gpu_t[2], ref[2]))


def test_validate_pairs_host_entry(gpu):
    data, T, O = terrain_pair("synth-rough-256")
    s, a, d, _, _ = attempts_oracle(O, 3000, seed=9)
    out = T.validate_pairs_host(s, a, d)
    # the host entry re-decides FRAGILE attempts itself: its outputs are final
    assert_pairs_equal(out, O.validate_pairs(s, a, d, nthreads=8), "host", resolve=lambda g: g)


# ---- samplers ---------------------------------------------------------------------
@pytest.mark.parametrize("name", ["synth-rough-256", "slope-gridmap"])
def test_samplers_match_oracle(gpu, name):
    data, T, O = terrain_pair(name)
    n = 20000
    g, gt = T.sample_states(n, 31, 1, 0, require_phase=L.STANCE, max_tries=256)
    r, rt = O.sample_states(n, 31, 1, 0, L.STANCE, 256, nthreads=8)
    assert np.array_equal(np_(gt), rt)  # same accepted draw for every index
    # the samplers' transcendentals are the engine's reproducible rm_* routines,
    # restated by the oracle: every draw is bit-identical
    assert np.all(same_f64(np_(g), r))
    nrm = O.normal_batch(r[:, :2])[0]
    ga = T.sample_actions(torch.from_numpy(nrm), 31, 3)
    ra = oracle.sample_actions(nrm, 31, 3)
    assert np.array_equal(bits(np_(ga)), bits(ra))


# ---- extend -------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["synth-rough-256", "rough_terrain-gridmap"])
def test_extend_parity(gpu, name):
    data, T, O = terrain_pair(name)
    n = 6000
    s_near, _, d, target, _ = attempts_oracle(O, n, seed=41)
    base = 1000
    r = T.extend(torch.from_numpy(s_near), torch.from_numpy(target), torch.from_numpy(d),
                 seed=41, extend_base=base)
    # the engine's candidate actions, regenerated through the public sampler:
    # candidate j of extend i is stream EXTD (0x45585444), index (base+i)*8+j
    nrm = O.normal_batch(target[:, :2])[0]
    dense = np_(T.sample_actions(torch.from_numpy(np.repeat(nrm, 8, axis=0)), 41, 0x45585444,
                                 base * 8)).reshape(n, 8, 10)
    cand = np.ascontiguousarray(dense[:, :6])
    rr, rch, rsn, ran, rc = O.extend_batch(s_near, target, cand, d, nthreads=8)
    assert np.array_equal(np_(r.result), rr)
    assert np.array_equal(np_(r.chosen), rch)
    assert np.array_equal(u32(r.counts), rc)
    acc = rr != L.TRAPPED
    assert np.array_equal(bits(np_(r.s_new)[acc]), bits(rsn[acc]))
    assert np.array_equal(bits(np_(r.a_new)[acc]), bits(ran[acc]))
    assert (rch >= 0).sum() > 0


# ---- nearest neighbour ------------------------------------------------------------------
def test_nearest_parity(gpu):
    import global_body_planner_amd as gbp
    rng = np.random.default_rng(3)
    verts = rng.normal(size=(5000, 8))
    verts[100] = verts[7]          # exact duplicate: tie -> lowest index
    q = np.concatenate([rng.normal(size=(2000, 8)), verts[[7, 100, 4999]]])
    idx, dist = gbp.nearest(torch.from_numpy(q).cuda(), torch.from_numpy(verts).cuda())
    ri, rd = oracle.nearest_batch(q, verts)
    assert np.array_equal(np_(idx), ri)
    assert np.array_equal(bits(np_(dist)), bits(rd))
    assert np_(idx)[-3] == 7 and np_(idx)[-2] == 7
    # few queries take the one-workgroup-per-query kernel, many the LDS-tiled one
    i2, d2 = gbp.nearest(torch.from_numpy(q[:100]).cuda(), torch.from_numpy(verts).cuda())
    assert np.array_equal(np_(i2), ri[:100]) and np.array_equal(bits(np_(d2)), bits(rd[:100]))
    qn = q[:600].copy()
    qn[5] = np.nan                 # NaN query: no distance is < inf -> index 0
    i3, _ = gbp.nearest(torch.from_numpy(qn).cuda(), torch.from_numpy(verts[:300]).cuda())
    r3, _ = oracle.nearest_batch(qn, verts[:300])
    assert np.array_equal(np_(i3), r3) and np_(i3)[5] == 0
    # empty tree keeps index 0 with +inf, like the reference's initial values
    idx0, d0 = gbp.nearest(torch.from_numpy(q[:4]).cuda(), torch.empty((0, 8), dtype=torch.float64).cuda())
    assert np.all(np_(idx0) == 0) and np.all(np.isinf(np_(d0)))


def test_neighbors_parity(gpu):
    """PlannerClass::neighborhoodDist (planner_class.cpp:173-182) on the engine
    vs the oracle: same members, ascending index, self (distance 0) excluded,
    counts beyond max_out reported."""
    import global_body_planner_amd as gbp
    rng = np.random.default_rng(4)
    verts = rng.normal(size=(3000, 8)) * 0.8
    q = np.concatenate([rng.normal(size=(700, 8)) * 0.8, verts[[0, 17, 2999]]])
    counts = {}
    for radius, max_out in ((3.0, 512), (1.5, 16), (0.0, 8)):
        out, cnt = gbp.neighbors(torch.from_numpy(q).cuda(), torch.from_numpy(verts).cuda(),
                                 radius, max_out)
        ro, rc = oracle.neighbors_batch(q, verts, radius, max_out)
        assert np.array_equal(np_(cnt), rc)
        assert np.array_equal(np_(out), ro)
        counts[radius] = rc
    assert (counts[1.5] > 16).any()      # truncation exercised at max_out 16
    assert not counts[0.0].any()         # distance 0 (the vertex itself) is excluded


# ---- full-size, size-independent properties --------------------------------------------
def test_full_size_batch_properties(gpu):
    """BASELINE config 3 size (256k attempts, synth-rough-1024): direct == persistent
    bit for bit, determinism, slice independence, and parity with the oracle."""
    import global_body_planner_amd as gbp
    from global_body_planner_amd import workload as W
    data = td.synth_rough(1024)
    T = gbp.Terrain.from_data(data, device=0)
    O = oracle.OracleTerrain.from_data(data)
    n = 262144
    s, a, d, tgt, tries = W.make_attempts(T, n, W.CONFIG_SEEDS[3])
    assert int((tries < 0).sum()) == 0
    outs = []
    for kernel in (L.KERNEL_DIRECT, L.KERNEL_PERSISTENT, L.KERNEL_PERSISTENT):
        T.set_option(L.OPT_KERNEL, kernel)
        r = T.validate_pairs(s, a, d)
        outs.append((np_(r.valid), np_(r.s_new), np_(r.t_new), u32(r.flags), u32(r.counts)))
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    # slice independence: the second half generated on its own equals the full batch's half
    s2, a2, d2, _, _ = W.make_attempts(T, n // 2, W.CONFIG_SEEDS[3], index_base=n // 2)
    assert torch.equal(s2, s[n // 2:]) and torch.equal(a2, a[n // 2:]) and torch.equal(d2, d[n // 2:])
    ref = O.validate_pairs(np_(s), np_(a), np_(d), nthreads=16)
    nfrag = assert_pairs_equal(outs[0], ref, "full", resolve=resolver(T, s, a, d))
    assert nfrag < 50
    assert 0 < ref[0].sum() < n


@pytest.mark.parametrize("coords", [0, 1, 2])
@pytest.mark.parametrize("helpers", [0, 1])
@pytest.mark.parametrize("waves", [2, 3, 4])
def test_validate_pairs_variants(gpu, coords, helpers, waves):
    """Every coordinate source of the persistent kernel (0 global vectors, 1
    LDS-staged, 2 computed from the verified affine form), with and without
    tail helper lanes, at every register budget, computes the same answers."""
    data, T, O = terrain_pair("synth-rough-256")
    T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT)
    T.set_option(L.OPT_LDS_COORDS, 1 if coords == 1 else 0)
    T.set_option(L.OPT_AFFINE_COORDS, 1 if coords == 2 else 0)
    T.set_option(L.OPT_HELPERS, helpers)
    T.set_option(L.OPT_WAVES, waves)
    # four 256-lane workgroups of attempt rows + coordinates exceed a CU's
    # 160 KB of LDS: the kernel then reads the vectors from global memory
    assert T.get_option(L.OPT_COORD_MODE) == (0 if coords == 1 and waves == 4 else coords)
    try:
        for n in (1, 63, 5000):
            s, a, d, _, _ = attempts_oracle(O, n, seed=1000 + n)
            res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d))
            gpu_t = (np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags), u32(res.counts))
            assert_pairs_equal(gpu_t, O.validate_pairs(s, a, d, nthreads=8),
                               f"c{coords}h{helpers}w{waves}n{n}", resolve=resolver(T, s, a, d))
    finally:
        T.set_option(L.OPT_LDS_COORDS, 1)
        T.set_option(L.OPT_AFFINE_COORDS, 1)
        T.set_option(L.OPT_HELPERS, 1)
        T.set_option(L.OPT_WAVES, 2)


@pytest.mark.parametrize("name", ["synth-rough-256", "rough_terrain-gridmap"])
def test_validate_pairs_xcd_map(gpu, name):
    """XCD-major slice numbering (GBP_OPT_XCD_MAP) only changes which wave
    evaluates an attempt: outputs are bit-identical to the default numbering and
    to the oracle, on a batch ordered by position (the case it is for) and on
    grids that are not a multiple of 8 workgroups (identity numbering)."""
    data, T, O = terrain_pair(name)
    T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT)
    try:
        for n in (9000, 20011, 700):
            s, a, d, _, _ = attempts_oracle(O, n, seed=4242 + n)
            order = np.argsort(s[:, 0], kind="stable")
            s, a, d = s[order].copy(), a[order].copy(), d[order].copy()
            outs = []
            for xm in (0, 1):
                T.set_option(L.OPT_XCD_MAP, xm)
                assert T.get_option(L.OPT_XCD_MAP) == xm
                res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d))
                outs.append((np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags),
                             u32(res.counts)))
            for x, y in zip(outs[0], outs[1]):
                assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
            assert_pairs_equal(outs[1], O.validate_pairs(s, a, d, nthreads=16), f"xcd n{n}",
                               resolve=resolver(T, s, a, d))
    finally:
        T.set_option(L.OPT_XCD_MAP, 0)


@pytest.mark.parametrize("name", TERRAINS)
def test_fast_reciprocal_bit_exact(gpu, name):
    """The bilinear 1/((x2-x1)(y2-y1)) by two Newton steps (GBP_OPT_FAST_RCP,
    enabled by gbp_terrain_create only after checking every spacing pair
    bit-for-bit) gives the same heights, pair results and flags as the IEEE
    division, and the oracle."""
    data, T, O = terrain_pair(name)
    used = T.get_option(L.OPT_FAST_RCP)
    print(name, "fast reciprocal in use:", used)
    if name.startswith("synth") or name.endswith("gridmap"):
        assert used == 1  # affine / grid_map geometry: a handful of spacings
    n = 6000
    s, a, d, _, _ = attempts_oracle(O, n, seed=777)
    rng = np.random.default_rng(5)
    xy = np.stack([rng.uniform(data.x[0], data.x[-1], 20000), rng.uniform(data.y[0], data.y[-1], 20000)], 1)
    outs = []
    try:
        for f in (0, 1):
            T.set_option(L.OPT_FAST_RCP, f)
            h, _, _ = T.height(torch.from_numpy(xy))
            res = T.validate_pairs(torch.from_numpy(s), torch.from_numpy(a), torch.from_numpy(d))
            outs.append((np_(h), np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags),
                         u32(res.counts)))
    finally:
        T.set_option(L.OPT_FAST_RCP, 1)
    for x, y in zip(outs[0], outs[1]):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    assert_pairs_equal(outs[1][1:], O.validate_pairs(s, a, d, nthreads=16), f"rcp {name}",
                       resolve=resolver(T, s, a, d))


def test_engine_matches_golden_vectors(gpu):
    """The engine against the committed oracle vectors (tests/golden)."""
    import os
    from tests.helpers import same_f64
    path = os.path.join(os.path.dirname(__file__), "golden", "oracle_vectors.npz")
    g = np.load(path)
    for name in ["slope-gridmap", "rough_terrain-gridmap", "synth-rough-256"]:
        data, T, O = terrain_pair(name)
        T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT)
        p = name + "/"
        h, isn, ood = T.height(torch.from_numpy(g[p + "xy"]))
        assert np.all(same_f64(np_(h), g[p + "h"]))
        assert np.array_equal(np_(isn), g[p + "is_nan"]) and np.array_equal(np_(ood), g[p + "ood"])
        for ad in (0, 1):
            res = T.validate_pairs(torch.from_numpy(g[p + "pair_s"]), torch.from_numpy(g[p + "pair_a"]),
                                   torch.from_numpy(g[p + "pair_dir"]), adaptive=bool(ad))
            out = (np_(res.valid), np_(res.s_new), np_(res.t_new), u32(res.flags), u32(res.counts))
            ref = tuple(g[p + f"pair_{k}_{ad}"] for k in ("valid", "s_new", "t_new", "flags", "counts"))
            assert_pairs_equal(out, ref, f"golden-gpu {name} ad{ad}",
                               resolve=resolver(T, g[p + "pair_s"], g[p + "pair_a"], g[p + "pair_dir"],
                                                bool(ad)))


def test_config2_exact_batches(gpu):
    """Config 2's own batches: synth-rough-256, the
    65,536-attempt seed-20251017 batch bench.py times (workload.make_attempts)
    and the next one of the 8 it cycles through, through the persistent kernel
    at the bench's 2-wave launch, against the oracle on every attempt (FRAGILE
    ones re-decided by the product's own host check, none excluded)."""
    import global_body_planner_amd as gbp
    from global_body_planner_amd import workload as W
    data = td.by_name("synth-rough-256")
    T = gbp.Terrain.from_data(data, device=0)
    T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT)
    T.set_option(L.OPT_WAVES, 2)
    O = oracle.OracleTerrain.from_data(data)
    n = 65536
    for k in (0, 1):
        s, a, d, _, tries = W.make_attempts(T, n, W.CONFIG_SEEDS[2], index_base=k * n)
        assert int((tries < 0).sum()) == 0
        r = T.validate_pairs(s, a, d)
        gpu_t = (np_(r.valid), np_(r.s_new), np_(r.t_new), u32(r.flags), u32(r.counts))
        ref = O.validate_pairs(np_(s), np_(a), np_(d), nthreads=16)
        nfrag = assert_pairs_equal(gpu_t, ref, f"config2 batch {k}", resolve=resolver(T, s, a, d))
        assert nfrag < 50
        assert 0 < ref[0].sum() < n
