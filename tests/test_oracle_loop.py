"""CPU checks of the oracle's planner loop (oracle/gbp_oracle.c orc_plan,
orc_post_process_path) — the checker tests/test_gpu_oracle_loop.py pins the
engine's planner to.

  * orc_plan equals a second, independent restatement of the batch-synchronous
    half-iteration written here in Python from the oracle's primitives
    (randomState + isValidState(STANCE), nearest vertex, newConfig's six
    candidates on the engine's candidate stream, extend acceptance, ordered
    insertion, connect through the recursive attemptConnect, alternation;
    rrt_connect.cpp:230-314, rrt.cpp:77-102, :98-120) — trees compared bit for
    bit, at batch 1 (the reference's runRRTConnect) and batch 8;
  * orc_post_process_path equals a Python restatement of rrt_connect.cpp:139-227;
  * tree invariants of RRT-Connect and RRT*-Connect runs: parents precede
    children (RRT-Connect) / form a tree rooted at 0 (RRT*, after rewiring),
    g[i] == g[parent] + poseDistance (graph_class.cpp:36-42, :131-138), every
    edge passes the pair check it was accepted by;
  * the samplers' reproducible transcendentals (rm_*) against numpy.
"""
import numpy as np
import pytest

import oracle
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td
from tests.helpers import bits, same_f64

EXTD = 0x45585444
FORWARD, REVERSE, STANCE = 0, 1, 1
TRAPPED, ADVANCED, REACHED = 0, 1, 2


@pytest.fixture(scope="module")
def synth():
    data = td.synth_rough(256)
    O = oracle.OracleTerrain.from_data(data)
    oracle.set_scan_mode(1)
    hs, _ = O.ground_height(1.0, 2.55)
    hg, _ = O.ground_height(4.02, 2.55)
    return O, planner.start_goal_state(hs, 1.0, 2.55), planner.start_goal_state(hg, 4.02, 2.55)


def py_plan(O, start, goal, batch, seed, max_halves, sampling=None):
    """The half-iteration from the oracle's primitives (see module docstring)."""
    sm = sampling or {}
    trees = []
    for root in (start, goal):
        trees.append(dict(v=[np.array(root)], act=[np.zeros(10)], parent=[-1], g=[0.0], y=[0.0]))
    streams, draws, ext = (101, 102), [0, 0], 0
    for h in range(max_halves):
        k = h & 1
        T, Ot = trees[k], trees[k ^ 1]
        d = FORWARD if k == 0 else REVERSE
        last, root = T["v"][-1], Ot["v"][0]
        s_from, s_to = (last, root) if d == FORWARD else (root, last)
        cand = O.sample_states_dir(batch, seed, streams[k], s_from, s_to, index_base=draws[k],
                                   state_flag=sm.get("state_flag", False),
                                   state_p=sm.get("state_p", 0.0),
                                   speed_direction=sm.get("speed_direction", False))
        draws[k] += batch
        ok, _, _ = O.valid_states(cand, STANCE)
        tgt = cand[ok != 0]
        snap = np.array(T["v"])
        added = []
        for i, q in enumerate(tgt):
            nn = int(oracle.nearest_batch(q[None], snap)[0][0])
            s_near = snap[nn]
            nrm, _ = O.normal_batch(q[None, :2])
            acts = oracle.sample_actions_dir(np.repeat(nrm, 6, 0), np.repeat(q[None], 6, 0),
                                             np.repeat(s_near[None], 6, 0), d, seed, EXTD,
                                             (ext + i) * 8, action_flag=sm.get("action_flag", False),
                                             action_p=sm.get("action_p", 0.0))
            r, _, sn, an, _ = O.extend_batch(s_near[None], q[None], acts[None], d)
            if r[0] == TRAPPED:
                continue
            T["v"].append(sn[0])
            T["act"].append(an[0])
            T["parent"].append(nn)
            T["g"].append(T["g"][nn] + oracle.pose_distance(s_near, sn[0]))
            T["y"].append(T["y"][nn] + oracle.state_yaw_distance(s_near, sn[0]))
            added.append(len(T["v"]) - 1)
        ext += len(tgt)
        osnap = np.array(Ot["v"])
        meet = None
        for idx in added:
            q = T["v"][idx]
            nn = int(oracle.nearest_batch(q[None], osnap)[0][0])
            s_ex = osnap[nn]
            r, sn, an = O.attempt_connect(s_ex, q, REVERSE if d == FORWARD else FORWARD,
                                          t_s=oracle.pose_distance(q, s_ex) / 0.75)
            if r == TRAPPED:
                continue
            Ot["v"].append(sn)
            Ot["act"].append(an)
            Ot["parent"].append(nn)
            Ot["g"].append(Ot["g"][nn] + oracle.pose_distance(s_ex, sn))
            Ot["y"].append(Ot["y"][nn] + oracle.state_yaw_distance(s_ex, sn))
            if r == REACHED and meet is None:
                meet = (idx, len(Ot["v"]) - 1) if k == 0 else (len(Ot["v"]) - 1, idx)
        if meet is not None:
            return trees, meet, h + 1
    return trees, None, max_halves


@pytest.mark.parametrize("batch,seed,halves,sampling", [
    (1, 11, 3000, None),
    (8, 5, 400, None),
    (8, 5, 400, dict(state_flag=True, state_p=0.3, speed_direction=True, action_flag=True,
                     action_p=0.3)),
])
def test_orc_plan_equals_python_restatement(synth, batch, seed, halves, sampling):
    O, start, goal = synth
    trees, meet, ran = py_plan(O, start, goal, batch, seed, halves, sampling)
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=halves, sampling=sampling)
    assert ref["halves"] == ran
    assert bool(ref["found"]) == (meet is not None)
    if meet is not None:
        assert (ref["meet_a"], ref["meet_b"]) == meet
    for name, t in zip("ab", trees):
        r = ref[name]
        assert r["v"].shape[0] == len(t["v"])
        assert np.all(same_f64(r["v"], np.array(t["v"])))
        assert np.all(same_f64(r["act"], np.array(t["act"])))
        assert np.array_equal(r["parent"], np.array(t["parent"]))
        assert np.array_equal(bits(r["g"]), bits(np.array(t["g"])))
        assert np.array_equal(bits(r["y"]), bits(np.array(t["y"])))


def py_post_process(O, S, A):
    """rrt_connect.cpp:139-227."""
    s, s_goal = S[0], S[-1]
    out_s, out_a = [s], []
    length = yaw = cost = 0.0
    a_new = None
    while not np.array_equal(s, s_goal):
        last, old = len(S) - 1, None
        while True:
            r, _, an = O.attempt_connect(s, S[last], FORWARD)
            a_new = an
            if r == REACHED or np.array_equal(s, S[last]):
                break
            old = last
            last -= 1
        if not np.array_equal(s, S[last]):
            out_s.append(S[last])
            out_a.append(a_new)
            dl, dy = oracle.pose_distance(s, S[last]), oracle.state_yaw_distance(s, S[last])
            length += dl
            yaw += dy
            cost += dl
            s = S[last]
        else:
            out_s.append(S[old])
            out_a.append(A[old - 1])
            cost += oracle.pose_distance(s, S[old])
            s = S[old]
    return np.array(out_s), np.array(out_a), length, yaw, cost


@pytest.mark.parametrize("batch,seed", [(1, 11), (64, 11), (64, 3)])
def test_post_process_path(synth, batch, seed):
    O, start, goal = synth
    ref = O.plan(start, goal, batch=batch, seed=seed)
    assert ref["found"]
    S, A = ref["states"], ref["actions"]
    assert np.array_equal(S[0], start) and np.array_equal(S[-1], goal)
    ps, pa, L, Y, C = O.post_process_path(S, A)
    qs, qa, L2, Y2, C2 = py_post_process(O, S, A)
    assert np.array_equal(bits(ps), bits(qs)) and np.array_equal(bits(pa), bits(qa))
    assert (L, Y, C) == (L2, Y2, C2)
    assert np.array_equal(ps[0], start) and np.array_equal(ps[-1], goal)
    assert ps.shape[0] <= S.shape[0] and L <= C
    # every shortcut edge is a connect the reference's attemptConnect REACHES
    for i in range(ps.shape[0] - 1):
        if pa[i][7] == 0:
            r, _, _ = O.attempt_connect(ps[i], ps[i + 1], FORWARD)
            assert r == REACHED or any(np.array_equal(ps[i + 1], x) for x in S)


def _check_tree(O, t, direction, rooted_order):
    n = t["v"].shape[0]
    p = t["parent"]
    assert p[0] == -1
    if rooted_order:
        assert np.all(p[1:] < np.arange(1, n)) and np.all(p[1:] >= 0)
    # g[i] == g[parent] + poseDistance, and the parent chain reaches the root
    for i in range(1, n):
        assert t["g"][i] == t["g"][p[i]] + oracle.pose_distance(t["v"][p[i]], t["v"][i])
        j, steps = i, 0
        while j != 0:
            j = p[j]
            steps += 1
            assert 0 <= j < n and steps <= n
    # every edge passed the pair check of its tree's direction from the parent:
    # Ta's extends and connects FORWARD from s_near / s_existing, Tb's REVERSE
    # (rrt.cpp:36-39, rrt_connect.cpp:70-71; RRT*'s choose-parent / rewire
    # connects the same way, rrt_star_connect.cpp:36, :59)
    v = O.validate_pairs(t["v"][p[1:]], t["act"][1:], direction)[0]
    assert np.all(v != 0)


def test_tree_invariants(synth):
    O, start, goal = synth
    ref = O.plan(start, goal, batch=256, seed=7, max_halves=200)
    _check_tree(O, ref["a"], FORWARD, True)
    _check_tree(O, ref["b"], REVERSE, True)
    star = O.plan(start, goal, batch=1024, seed=3, max_halves=300, star=True, stream_a=401,
                  stream_b=402)
    assert star["rewires"] > 0 and star["found"]
    _check_tree(O, star["a"], FORWARD, False)
    _check_tree(O, star["b"], REVERSE, False)
    assert star["best_cost"] == star["a"]["g"][star["best_a"]] + star["b"]["g"][star["best_b"]]


def test_rmath_accuracy():
    """The samplers' log / sincos / atan2 / acos (gbp_device.h rm_*, restated
    by the oracle) are within a few ulp of correctly rounded (numpy), keep
    glibc's signed-zero / axis conventions, and are exact where it matters
    (log 1 = 0, sin 0 = 0, cos 0 = 1, acos(+-1))."""
    rng = np.random.default_rng(0)

    def ulp(a, b):
        return np.abs(a - b) / np.spacing(np.maximum(np.abs(b), 1e-300))
    x = np.concatenate([rng.uniform(0, 1, 200000), 2.0 ** -rng.uniform(0, 53, 20000),
                        [1.0, 2.0 ** -53, 0.5]])
    assert ulp(oracle.rmath(0, x), np.log(x)).max() <= 4
    assert oracle.rmath(0, [1.0])[0] == 0.0
    x = np.concatenate([rng.uniform(-4, 7, 200000), np.arange(-8, 9) * np.pi / 4])
    sc = oracle.rmath(1, x)
    assert np.abs(sc[:, 0] - np.sin(x)).max() <= 2.3e-16
    assert np.abs(sc[:, 1] - np.cos(x)).max() <= 2.3e-16
    assert np.array_equal(oracle.rmath(1, [0.0])[0], [0.0, 1.0])
    y, xx = rng.normal(size=200000), rng.normal(size=200000)
    assert ulp(oracle.rmath(2, xx, y), np.arctan2(y, xx)).max() <= 8
    for yy, xv in [(0.0, 1.0), (-0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0),
                   (0.0, 0.0), (-0.0, -0.0)]:
        assert bits(oracle.rmath(2, [xv], [yy]))[0] == bits(np.arctan2(yy, xv))
    c = np.concatenate([rng.uniform(-1, 1, 200000), [-1.0, 1.0, 0.0]])
    assert ulp(oracle.rmath(3, c), np.arccos(c)).max() <= 8
    assert oracle.rmath(3, [1.0])[0] == 0.0 and oracle.rmath(3, [-1.0])[0] == np.pi


@pytest.mark.parametrize("star", [False, True])
def test_orc_plan_threads_identical(synth, star):
    """orc_plan's per-item passes on OpenMP threads (the config-3-scale GPU
    test runs it on the box's cores) give the serial run's trees, counters and
    meeting vertices bit for bit: each item reads only the half's snapshot and
    insertion stays in order."""
    O, start, goal = synth
    kw = dict(batch=1024, seed=5, max_halves=40 if star else 0, star=star)
    if star:
        kw.update(stream_a=401, stream_b=402)
    one = O.plan(start, goal, nthreads=1, **kw)
    many = O.plan(start, goal, nthreads=4, **kw)
    for k, v in one.items():
        if k in ("a", "b"):
            for f in ("v", "act", "parent", "g", "y"):
                assert np.array_equal(bits(v[f]), bits(many[k][f])), (k, f)
        elif k in ("states", "actions"):
            assert np.array_equal(bits(v), bits(many[k])), k
        else:
            assert (v == many[k]) or (v != v and many[k] != many[k]), k


def test_orc_plan_warm_start_is_continuation(synth):
    """A warm start (the trees after h0 half-iterations, the draw indices of
    half h0, the candidate stream at the extend counter) continues the search
    exactly: the same trees as the uninterrupted run (the config-3-scale GPU
    test continues device-grown trees this way)."""
    O, start, goal = synth
    kw = dict(batch=512, seed=9)
    full = O.plan(start, goal, max_halves=30, **kw)
    assert not full["found"]
    first = O.plan(start, goal, max_halves=17, **kw)
    init = tuple({k: first[t][k] for k in ("v", "act", "parent")} for t in "ab")
    cont = O.plan(start, goal, max_halves=13, init_trees=init, first_half=17,
                  extend_base=first["ext_counter"], nthreads=2, **kw)
    assert cont["halves"] == 13
    assert cont["targets"] + first["targets"] == full["targets"]
    assert cont["attempts"] + first["attempts"] == full["attempts"]
    for t in "ab":
        for f in ("v", "act", "parent", "g", "y"):
            assert np.array_equal(bits(cont[t][f]), bits(full[t][f])), (t, f)
