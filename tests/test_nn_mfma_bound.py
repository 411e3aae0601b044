"""The matrix-core nearest-neighbour search's threshold (global_body_planner_amd/
csrc/gbp_plan.hip: k_nn_mfma, nn_put_hrow, nh_eps, nh_threshold) restated in
numpy and checked on the CPU: the scores S~_j = |F_j|^2 - 2 G.F_j are formed as
the two v_mfma_f32_32x32x16_f16 do (F = 64 v and G = 64 q split into fp16
hi + lo, the squared norm times 2^-14 in three fp16 parts against the query
side's 2^14, fp16 x fp16 products exact, fp32 accumulation) and for every query
the exact fp64 minimiser of stateDistance (planning_utils.cpp:116-127; the
lowest index among equal distances, planner_class.cpp:185-200) and every index
tying with it must score <= T(B), B = min_j S~_j.  The accumulation is run
both rounding to nearest and truncating (the bound assumes either).  The GPU
test (tests/test_gpu_device_loop.py::test_tree_nearest_fp32_filter_exact) checks
the kernels' indices bit for bit."""
import numpy as np
import pytest

SCALE, LIM, NSCALE = 64.0, 8192.0, 2.0 ** -14


def _h(x):
    """fp64 -> fp32 -> fp16, as the kernels convert (values back in fp64)."""
    return np.asarray(x, np.float64).astype(np.float32).astype(np.float16).astype(np.float64)


def split(x):
    hi = _h(x)
    return hi, _h(x - hi)


def rows(V):
    F = V * SCALE
    assert np.all(np.abs(F) < LIM)  # the tree is representable (else the fp64 scan)
    fh, fl = split(F)
    ns = (F * F).sum(axis=1) * NSCALE
    n1 = _h(ns)
    r1 = ns - n1
    n2 = _h(r1)
    n3 = _h(r1 - n2)
    hmax = np.abs(F).max(axis=0).astype(np.float32).astype(np.float64)
    return fh, fl, np.stack([n1, n2, n3], axis=1), hmax


def _acc32(terms, mode):
    """Sequential fp32 accumulation of the exact products (columns in order)."""
    acc = np.zeros(terms.shape[0], np.float32)
    for k in range(terms.shape[1]):
        x = acc.astype(np.float64) + terms[:, k]
        r = x.astype(np.float32)
        if mode == "rz":  # truncation: step back toward zero where rounding went away
            away = np.abs(r.astype(np.float64)) > np.abs(x)
            r[away] = np.nextafter(r[away], np.float32(0))
        acc = r
    return acc


def scores(R, q, mode):
    fh, fl, nparts, _ = R
    G = q * SCALE
    gh, gl = split(G)
    t1 = np.concatenate([fh * (-2.0 * gh), fl * (-2.0 * gh)], axis=1)   # MFMA 1, K = 16
    t2 = np.concatenate([fh * (-2.0 * gl), nparts * 16384.0], axis=1)   # MFMA 2
    return _acc32(np.concatenate([t1, t2], axis=1), mode), G


def eps(G, hmax):
    m = hmax * (1.0 + 2.0 ** -22)
    ag = np.abs(G)
    mm, gm = float((m * m).sum()), float((ag * m).sum())
    lin = float(((4.0 * 2.0 ** -20 * ag + 1.01 * 2.0 ** -14) * m + 1.01 * 2.0 ** -14 * ag
                 + 2.0 ** -27).sum())
    gamma = 33.0 * 2.0 ** -23
    return gamma * (1.01 * mm + 2.02 * gm) + 2.0 ** -29 * mm + 1.0 + 2.0 * lin


def threshold(B, e, g2):
    t = float(B) + 2.0 * e + 1e-14 * (abs(float(B)) + e + g2)
    return np.nextafter(np.float32(t), np.float32(np.inf))


def check_set(V, Q, mode="rn"):
    R = rows(V)
    ncand = []
    for q in Q:
        S, G = scores(R, q, mode)
        B = S.min()
        T = threshold(B, eps(G, R[3]), float((G * G).sum()))
        d = np.sqrt(((V - q) ** 2).sum(axis=1))
        ties = np.flatnonzero(d == d.min())
        assert np.all(S[ties] <= T), (S[ties], T, B)
        ncand.append(int((S <= T).sum()))
    return np.array(ncand)


def _states(rng, n, off=0.0, span=20.0):
    X = np.empty((n, 8))
    X[:, :2] = rng.uniform(0, span, size=(n, 2)) + off
    X[:, 2] = rng.uniform(0.2, 1.2, size=n)
    X[:, 3:6] = rng.normal(scale=1.0, size=(n, 3))
    X[:, 6:8] = rng.normal(scale=0.3, size=(n, 2))
    return X


@pytest.mark.parametrize("mode", ["rn", "rz"])
def test_bound_random_states(mode):
    rng = np.random.default_rng(21)
    V, Q = _states(rng, 3000), _states(rng, 200)
    nc = check_set(V, Q, mode)
    assert np.median(nc) <= 2 and nc.max() <= 8   # one or two half-chunks to re-check


@pytest.mark.parametrize("off", [-100.0, 40.0, 100.0])
def test_bound_offsets(off):
    """|F| up to 2^13 (|v| < 128): the widest representable trees."""
    rng = np.random.default_rng(22)
    V, Q = _states(rng, 2000, off, span=20.0), _states(rng, 100, off, span=20.0)
    check_set(V, Q, "rz")


def test_bound_near_ties_and_duplicates():
    """Exact duplicates, fp16-identical clusters (1e-9 apart), mirror images
    exactly equidistant from the query: every tying index scores <= T."""
    rng = np.random.default_rng(23)
    base = _states(rng, 50)
    V = np.repeat(base, 20, axis=0) + rng.normal(scale=1e-9, size=(1000, 8))
    V[::5] = np.repeat(base, 20, axis=0)[::5]
    Q = base + rng.normal(scale=1e-10, size=base.shape)
    Q[::2] = base[::2]
    m = base[:10].copy()
    e = np.zeros(8)
    e[0] = 0.5
    V2 = np.concatenate([V, m + e, m - e])
    check_set(V2, np.concatenate([Q, m]), "rz")


@pytest.mark.parametrize("mode", ["rn", "rz"])
def test_bound_shell_of_near_equal_distances(mode):
    """Vertices on a unit shell around each query, radii 1 + O(1e-8): the
    fp16-split scores order them almost at random; only T keeps the fp64
    minimiser."""
    rng = np.random.default_rng(24)
    Q = _states(rng, 40)
    V = []
    for q in Q:
        dirs = rng.normal(size=(50, 8))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        V.append(q + dirs * (1.0 + rng.normal(scale=1e-8, size=(50, 1))))
    check_set(np.concatenate(V), Q, mode)


def test_subnormal_low_parts():
    """Coordinates near zero: the lo parts are fp16 subnormals (or flushed);
    the bound's 2^-14 terms cover them."""
    rng = np.random.default_rng(25)
    V = rng.normal(scale=1e-5, size=(500, 8))
    Q = rng.normal(scale=1e-5, size=(50, 8))
    check_set(V, Q, "rz")
    # and flushed: the lo parts below 2^-14 set to zero
    R = rows(V)
    fh, fl, nparts, hmax = R
    fl = np.where(np.abs(fl) < 2.0 ** -14, 0.0, fl)
    R2 = (fh, fl, nparts, hmax)
    for q in Q:
        S, G = scores(R2, q, "rz")
        T = threshold(S.min(), eps(G, hmax), float((G * G).sum()))
        d = np.sqrt(((V - q) ** 2).sum(axis=1))
        assert np.all(S[d == d.min()] <= T)
