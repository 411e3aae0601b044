"""The nearest-neighbour filter's threshold (global_body_planner_amd/csrc/
gbp_plan.hip, k_nn_filter / nn_threshold) restated in numpy and checked on the
CPU: for every query the exact fp64 minimiser of stateDistance
(planning_utils.cpp:116-127, the lowest index among equal distances,
planner_class.cpp:185-200) must satisfy S_j* <= T(B), where S_j = n_j - 2 g.f_j
is evaluated as the kernel does (fp32 roundings of the rows and the query, the
fp64-summed norm rounded to fp32, an 8-step fp32 FMA chain), B = min_j S_j and
T the kernel's bound.  This pins the filter's exactness argument on adversarial
sets without a GPU; the GPU test (tests/test_gpu_device_loop.py) checks the
kernel's indices bit for bit."""
import numpy as np
import pytest

U = 2.0 ** -24


def _f32(x):
    return np.asarray(x, dtype=np.float64).astype(np.float32)


def _fma32(a, b, c):
    # a * b is exact in fp64 for fp32 operands; the fp64 add then one rounding
    # to fp32 (double rounding differs from a true fma by at most 1 ulp in
    # rare ties, far inside the bound's slack)
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def filter_scores(V, q):
    """S_j for one query against rows V (the kernel's nn_s2 chain)."""
    f = _f32(V)
    n = (f.astype(np.float64) ** 2).sum(axis=1).astype(np.float32)   # nn_put_row
    a = (np.float32(-2.0) * _f32(q)).astype(np.float32)
    acc = n.copy()
    for k in range(8):
        acc = _fma32(f[:, k], np.full(f.shape[0], a[k], np.float32), acc)
    return acc, f


def threshold(B, q, vmax):
    g = np.abs(_f32(q).astype(np.float64))
    g2 = float((g * g).sum())
    r2 = float(((vmax.astype(np.float64) + g) ** 2).sum())
    eps, dl = 10.0 * U * r2, 2.0 * U * np.sqrt(r2)
    r0 = np.sqrt(max(0.0, float(B) + g2 + eps))
    r1 = (r0 + dl) * (1.0 + 4e-15) + dl
    return np.nextafter(np.float32(r1 * r1 * (1.0 + 1e-12) - g2 + eps), np.float32(np.inf))


def exact_argmin(V, q):
    d = np.sqrt(((V - q) ** 2).sum(axis=1))
    return int(np.flatnonzero(d == d.min())[0]), d


def check_set(V, Q):
    f_all = _f32(V)
    vmax = np.abs(f_all).max(axis=0).astype(np.float32)
    ncand = []
    for q in Q:
        S, _ = filter_scores(V, q)
        B = S.min()
        T = threshold(B, q, vmax)
        j, d = exact_argmin(V, q)
        ties = np.flatnonzero(d == d[j])
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


def test_bound_random_states():
    rng = np.random.default_rng(11)
    V, Q = _states(rng, 3000), _states(rng, 200)
    nc = check_set(V, Q)
    assert nc.max() <= 4  # one or two candidates on planner-like sets


@pytest.mark.parametrize("off", [40.0, 300.0, 5000.0, 1e5])
def test_bound_far_offsets(off):
    """Cancellation in n_j - 2 g.f_j grows with |f| + |g|: T widens, the
    minimiser stays inside it (the kernel then may take its overflow scan)."""
    rng = np.random.default_rng(12)
    V, Q = _states(rng, 2000, off), _states(rng, 100, off)
    check_set(V, Q)


def test_bound_near_ties_and_duplicates():
    """Vertices at fp64 distances equal or 1 ulp apart from the query, fp32-
    identical clusters, exact duplicates: every tying index stays a
    candidate."""
    rng = np.random.default_rng(13)
    base = _states(rng, 50)
    V = np.repeat(base, 20, axis=0) + rng.normal(scale=1e-9, size=(1000, 8))
    V[::5] = np.repeat(base, 20, axis=0)[::5]
    Q = base + rng.normal(scale=1e-10, size=base.shape)
    Q[::2] = base[::2]
    # mirror images: q +- e along one axis are exactly equidistant
    m = base[:10].copy()
    V2 = np.concatenate([V, m + [0.5, 0, 0, 0, 0, 0, 0, 0], m - [0.5, 0, 0, 0, 0, 0, 0, 0]])
    check_set(V2, np.concatenate([Q, m]))


@pytest.mark.parametrize("off", [0.0, 300.0])
def test_bound_shell_of_near_equal_distances(off):
    """Vertices on a unit shell around each query, radii 1 + O(1e-8): the fp32
    scores order them almost at random, so only the bound (not the fp32 argmin)
    keeps the fp64 minimiser."""
    rng = np.random.default_rng(14)
    Q = _states(rng, 40, off)
    V = []
    for q in Q:
        dirs = rng.normal(size=(50, 8))
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        V.append(q + dirs * (1.0 + rng.normal(scale=1e-8, size=(50, 1))))
    V = np.concatenate(V)
    check_set(V, Q)
