"""The device planner pinned to the oracle at the bench's own scale (VERDICT r04
"next" #1, "weak" #1).

tests/test_gpu_oracle_loop.py pins gbp_plan_halves_dev (algorithm 3) to
oracle/gbp_oracle.c orc_plan on synth-256 and the slope CSV at batch <= 4096,
with trees of a few hundred vertices.  The planner figure bench.py reports runs
on synth-rough-1024 at SURVEY §8(d)'s 43,690 targets per half-iteration
(92,749 randomState draws at the terrain's STANCE-valid fraction), where the
machinery that small batches never reach is active:

  * the next half's targets drawn inside the current half's matrix-core search
    launch and committed by its last append (gbp_plan.hip NhDraw, commit_pre);
  * the ordered look-back over ~360 tiles of draws and ~170 of targets;
  * trees of tens of thousands of vertices, so the MFMA nearest-vertex search
    re-checks units in fp64 and runs whole-segment scans (nn_scans > 0) on the
    clustered trees;
  * validate launches of up to 262,144 candidate pair checks.

Same bar as the small cases: every vertex, action, parent and g of both trees,
the meeting vertices, the path and the counters bit for bit against orc_plan
(rrt_connect.cpp:230-314, rrt.cpp:77-102, :98-120; graph_class.cpp:36-42).  The
oracle's per-target / per-connection passes run on the box's host threads
(tests/test_oracle_loop.py::test_orc_plan_threads_identical: same result as
serial).
"""
import os
import time

import numpy as np
import pytest

import oracle
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td
from tests.test_gpu_oracle_loop import assert_counters_equal, assert_trees_equal
from tests.test_gpu_planner import _start_goal
from tests.helpers import bits

pytestmark = pytest.mark.gpu

# 262,144 candidate pair checks per half = 43,690
# targets x 6; bench.py draws targets / STANCE-valid fraction per half
DRAWS = 92749
NTHREADS = max(1, min(16, os.cpu_count() or 1))

_cache = {}


def _terrain():
    if "t" not in _cache:
        data = td.by_name("synth-rough-1024")
        _cache["t"] = (data, oracle.OracleTerrain.from_data(data))
    oracle.set_scan_mode(1)
    return _cache["t"]


def _compare(dev, ref):
    assert dev["found"] == ref["found"]
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)
    if ref["found"]:
        assert (dev["meet_a"], dev["meet_b"]) == (ref["meet_a"], ref["meet_b"])
        assert np.array_equal(bits(dev["states"]), bits(ref["states"]))
        assert np.array_equal(bits(dev["actions"]), bits(ref["actions"]))
        assert dev["reported_length"] == ref["path_length"]


def test_config3_scale_from_roots(gpu):
    """The bench's "before the wall" pair ((1.0, 10.23) -> (6.8, 10.23)) at
    92,749 draws per half from the roots to its first solution: draw-ahead
    and the folded commit at full batch, the meet inside a group of halves."""
    data, O = _terrain()
    start, goal = _start_goal(O, 1.0, 10.23, 6.8, 10.23)
    dev = planner.plan_rrt_connect(data, start, goal, algorithm=3, batch=DRAWS, max_time=300.0,
                                   seed=20251018, trees=True, tree_capacity=1 << 17)
    ref = O.plan(start, goal, batch=DRAWS, seed=20251018, capacity=1 << 17, nthreads=NTHREADS)
    print(f"from the roots: found {ref['found']} at half {ref['meet_half']}, trees "
          f"{len(ref['a']['v'])}+{len(ref['b']['v'])}, {ref['targets']} targets, "
          f"{ref['attempts']} pair checks")
    assert ref["found"] and ref["targets"] >= 40000 * ref["halves"] // 2
    _compare(dev, ref)


# trees of tens of thousands of vertices take thousands of half-iterations on
# synth-rough-1024 (most extends are TRAPPED: ~30 vertices per half), far past
# what the oracle replays in a test; the device grows them (an input like any
# other), then the device and the oracle continue from the same trees
GROW_HALVES = 20000
CONT_HALVES = 40


def test_config3_scale_warm_continuation(gpu):
    """SURVEY's pair ((1.0, 10.23) -> (19.42, 10.23)): the trees the device
    grows in GROW_HALVES half-iterations, then CONT_HALVES more at 92,749
    draws each from the device and from orc_plan, bit for bit — the targets'
    matrix-core search against trees past 10k vertices with its fp64
    re-checks and segment scans, validate launches of ~262k pair checks.  The
    warm start itself is checked against the uninterrupted device run."""
    data, O = _terrain()
    start, goal = _start_goal(O, 1.0, 10.23, 19.42, 10.23)
    cap = 1 << 18
    t0 = time.time()
    grown = planner.plan_rrt_connect(data, start, goal, algorithm=3, batch=DRAWS, max_time=300.0,
                                     seed=20251018, max_halves=GROW_HALVES, trees=True,
                                     tree_capacity=cap)
    t_grow = time.time() - t0
    assert not grown["found"] and grown["halves"] == GROW_HALVES
    init = tuple({k: grown[t][k] for k in ("v", "act", "parent")} for t in "ab")
    n0 = (len(init[0]["v"]), len(init[1]["v"]))
    assert max(n0) > 10000, n0
    warm = dict(batch=DRAWS, seed=20251018, max_halves=CONT_HALVES)
    dev = planner.plan_rrt_connect(data, start, goal, algorithm=3, max_time=300.0, trees=True,
                                   tree_capacity=cap, nn_stats=True, init_trees=init,
                                   first_half=GROW_HALVES, extend_base=grown["extends"], **warm)
    t0 = time.time()
    ref = O.plan(start, goal, capacity=cap, nthreads=NTHREADS, init_trees=init,
                 first_half=GROW_HALVES, extend_base=grown["extends"], **warm)
    t_ref = time.time() - t0
    print(f"grown {GROW_HALVES} halves in {t_grow:.2f} s: trees {n0[0]}+{n0[1]}; continuation "
          f"{CONT_HALVES} halves: +{len(ref['a']['v']) - n0[0]}+{len(ref['b']['v']) - n0[1]} "
          f"vertices, {ref['targets']} targets, {ref['attempts']} pair checks; device nn "
          f"re-checks {dev['nn_rechecks']}, segment scans {dev['nn_scans']}, "
          f"{dev['fragile_resolved']} re-decided with glibc; oracle {t_ref:.1f} s on "
          f"{NTHREADS} threads")
    assert ref["halves"] == CONT_HALVES and ref["targets"] >= 40000 * CONT_HALVES
    _compare(dev, ref)
    assert dev["nn_scans"] > 0
    # the warm start is the continuation: the uninterrupted device run to
    # GROW_HALVES + CONT_HALVES grows the same trees
    full = planner.plan_rrt_connect(data, start, goal, algorithm=3, batch=DRAWS, max_time=300.0,
                                    seed=20251018, max_halves=GROW_HALVES + CONT_HALVES,
                                    trees=True, tree_capacity=cap)
    for t in "ab":
        for k in ("v", "act", "parent", "g"):
            assert np.array_equal(bits(full[t][k]), bits(dev[t][k])), (t, k)


def test_config3_scale_scan_list_overflow(gpu, monkeypatch):
    """The reduce's list of segment scans (k_nn_scan) full: with a list of 2
    entries (GBP_NSC_CAP, read when the planner creates its workspace) every
    further query with scans becomes a whole-tree fp64 scan in the reduce.
    The warm continuation of the test above, against the oracle."""
    data, O = _terrain()
    start, goal = _start_goal(O, 1.0, 10.23, 19.42, 10.23)
    cap = 1 << 18
    grown = planner.plan_rrt_connect(data, start, goal, algorithm=3, batch=DRAWS, max_time=300.0,
                                     seed=20251018, max_halves=GROW_HALVES, trees=True,
                                     tree_capacity=cap)
    init = tuple({k: grown[t][k] for k in ("v", "act", "parent")} for t in "ab")
    warm = dict(batch=DRAWS, seed=20251018, max_halves=CONT_HALVES)
    monkeypatch.setenv("GBP_NSC_CAP", "2")
    dev = planner.plan_rrt_connect(data, start, goal, algorithm=3, max_time=300.0, trees=True,
                                   tree_capacity=cap, nn_stats=True, init_trees=init,
                                   first_half=GROW_HALVES, extend_base=grown["extends"], **warm)
    monkeypatch.delenv("GBP_NSC_CAP")
    ref = O.plan(start, goal, capacity=cap, nthreads=NTHREADS, init_trees=init,
                 first_half=GROW_HALVES, extend_base=grown["extends"], **warm)
    _compare(dev, ref)
    assert dev["nn_scans"] > 2 * 2 * CONT_HALVES  # more than the lists held


# ---- config 5: RRT*-Connect on synth-fractal-4096 at the bench's own scale ------
# (VERDICT r05 "next" #2).  bench.py's config5 runs 4096 draws per half for 10 s:
# ~24.5k halves, trees of ~58k + 53k vertices, ~147k rewires.  The device grows
# the trees past 40k vertices each; then the device and orc_plan(star) continue
# from the same trees, bit for bit: neighbourhoods of ~60 vertices in the map's
# iteration order over chunked scans, rewired subtrees' g updates through deep
# subtrees (k_star_replay's subtree_g), the look-ahead search on RRT* trees.
STAR_DRAWS = 4096
STAR_SEED = 20251020
STAR_GROW = 18000
STAR_CONT = 24


def _star_terrain():
    if "f" not in _cache:
        data = td.by_name("synth-fractal-4096")
        _cache["f"] = (data, oracle.OracleTerrain.from_data(data))
    oracle.set_scan_mode(1)
    return _cache["f"]


def _first_valid(O, x, y, step, n=400):
    """tools/config5.py first_valid on the oracle: z = 0.375 + ground, v = (1, 0, 0)."""
    xs = x + step * np.arange(n)
    h, _, _ = O.height_batch(np.stack([xs, np.full(n, y)], 1))
    st = np.zeros((n, 8))
    st[:, 0], st[:, 1], st[:, 2], st[:, 3] = xs, y, 0.375 + h, 1.0
    v, _, _ = O.valid_states(st, 1)
    return st[int(np.argmax(v > 0))]


def test_config5_star_scale_warm_continuation(gpu):
    """Config 5's own scale: trees grown by the device past 40k vertices each
    (STAR_GROW halves at 4096 draws), then STAR_CONT more halves from the
    device (algorithm 5) and from orc_plan(star) — vertices, actions, parents,
    g, rewires and the best connection bit for bit.  The warm start derives g
    from the root down on both sides; that equals the grown trees' g (every
    updateGYValue keeps g[c] = g[parent] + poseDistance), and the continuation
    equals the uninterrupted device run."""
    data, O = _star_terrain()
    L = data.x[-1]
    start = _first_valid(O, 1.0, L / 2, 0.02)
    goal = _first_valid(O, 9.0, L / 2, -0.02)
    cap = 1 << 17
    t0 = time.time()
    grown = planner.plan_rrt_star_connect(data, start, goal, batch=STAR_DRAWS, max_time=300.0,
                                          seed=STAR_SEED, max_halves=STAR_GROW, trees=True,
                                          tree_capacity=cap, device_loop=True)
    t_grow = time.time() - t0
    assert grown["halves"] == STAR_GROW
    init = tuple({k: grown[t][k] for k in ("v", "act", "parent")} for t in "ab")
    n0 = (len(init[0]["v"]), len(init[1]["v"]))
    assert min(n0) > 40000, n0
    # RRT* trees: rewiring gave vertices later parents
    assert any(np.any(grown[t]["parent"][1:] > np.arange(1, len(grown[t]["parent"]))) for t in "ab")
    warm = dict(batch=STAR_DRAWS, seed=STAR_SEED, max_halves=STAR_CONT)
    dev = planner.plan_rrt_star_connect(data, start, goal, max_time=300.0, trees=True,
                                        tree_capacity=cap, device_loop=True, init_trees=init,
                                        first_half=STAR_GROW, extend_base=grown["extends"], **warm)
    t0 = time.time()
    ref = O.plan(start, goal, capacity=cap, nthreads=NTHREADS, init_trees=init, star=True,
                 stream_a=401, stream_b=402, first_half=STAR_GROW, extend_base=grown["extends"],
                 **warm)
    t_ref = time.time() - t0
    print(f"config 5: grown {STAR_GROW} halves in {t_grow:.2f} s: trees {n0[0]}+{n0[1]} "
          f"({grown['rewires']} rewires); continuation {STAR_CONT} halves: "
          f"+{len(ref['a']['v']) - n0[0]}+{len(ref['b']['v']) - n0[1]} vertices, "
          f"{ref['rewires']} rewires, {ref['targets']} targets, {ref['attempts']} pair checks, "
          f"{ref['solutions']} connections; device {dev['rewires']} rewires, "
          f"{dev['fragile_resolved']} re-decided; oracle {t_ref:.1f} s on {NTHREADS} threads")
    assert dev["halves"] == ref["halves"] == STAR_CONT
    assert dev["rewires"] == ref["rewires"] > 0
    assert dev["solutions"] == ref["solutions"]
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)
    if ref["best_a"] >= 0:
        assert (dev["meet_a"], dev["meet_b"]) == (ref["best_a"], ref["best_b"])
        assert dev["path_cost"] == ref["best_cost"]
    # the warm start's g, derived from the root down, is the grown trees' g
    for i, t in enumerate("ab"):
        par, v = init[i]["parent"], init[i]["v"]
        kids = [[] for _ in range(len(par))]
        for c in range(1, len(par)):
            kids[par[c]].append(c)
        g = np.zeros(len(par))
        queue = [0]
        for u in queue:
            for c in kids[u]:
                g[c] = g[u] + oracle.pose_distance(v[u], v[c])
                queue.append(c)
        assert len(queue) == len(par)
        assert np.array_equal(bits(g), bits(grown[t]["g"])), t
    # a rewire re-rooted a subtree: vertices below a rewired one, parent kept, g lowered
    lowered = sum(int(np.sum((ref[t]["parent"][:len(init[i]["v"])] == init[i]["parent"]) &
                             (ref[t]["g"][:len(init[i]["v"])] < grown[t]["g"][:len(init[i]["v"])])))
                  for i, t in enumerate("ab"))
    assert lowered > 0
    # the continuation is the uninterrupted run's
    full = planner.plan_rrt_star_connect(data, start, goal, batch=STAR_DRAWS, max_time=300.0,
                                         seed=STAR_SEED, max_halves=STAR_GROW + STAR_CONT,
                                         trees=True, tree_capacity=cap, device_loop=True)
    for t in "ab":
        for k in ("v", "act", "parent", "g"):
            assert np.array_equal(bits(full[t][k]), bits(dev[t][k])), (t, k)
