"""The planner loop pinned to the oracle (VERDICT r03 "next" #1).

The device-resident search (algorithm 3: gbp_plan_halves_dev, csrc/gbp_plan.hip)
and the host-driven batched planner (algorithm 0, csrc/host/gbp_planner.cpp)
against oracle/gbp_oracle.c orc_plan: a CPU restatement of the batch-synchronous
half-iteration — targets drawn on the engine's Philox streams (the samplers'
transcendentals are the reproducible rm_* routines on both sides) and filtered
by isValidState(STANCE) (rrt_connect.cpp:248-254), extend = nearest vertex +
newConfig + acceptance + ordered insertion with g = g[parent] + poseDistance
(rrt.cpp:77-102, graph_class.cpp:36-42), the connect of every new vertex to the
other tree through the recursive attemptConnect (rrt_connect.cpp:20-120), the
alternation of the trees (:230-314) — and against orc_post_process_path
(:139-227, its path_length_ quirk included) and the RRT* insertion
(rrt_star_connect.cpp:12-67: choose-parent, rewire, recursive g/y updates).

Bar: bit for bit — every vertex (NaN == NaN), action, parent and g of both
trees, the meeting vertices, the path, path_length_ / path_cost_ and the
counters (targets, extends, pair checks, connects, depth-capped connects).
Batch 1 is the reference's own sequential runRRTConnect on the engine's
streams.  FRAGILE decisions are the product's own host re-decisions with
glibc (counted in `fragile_resolved`); the oracle decides everything with
glibc directly.
"""
import numpy as np
import pytest

import oracle
from global_body_planner_amd import planner
from global_body_planner_amd import terrain_data as td
from tests.helpers import bits, same_f64
from tests.test_gpu_planner import _start_goal

pytestmark = pytest.mark.gpu

_cache = {}


def _setup(name, xy):
    if name not in _cache:
        data = td.by_name(name)
        O = oracle.OracleTerrain.from_data(data)
        _cache[name] = (data, O)
    data, O = _cache[name]
    oracle.set_scan_mode(1)   # bisection: the reference's brackets, quickly
    start, goal = _start_goal(O, *xy)
    return data, O, start, goal


def assert_trees_equal(dev, ref):
    for t in "ab":
        d, r = dev[t], ref[t]
        n = r["v"].shape[0]
        assert d["v"].shape[0] == n, (t, d["v"].shape[0], n)
        bad = np.flatnonzero(~np.all(same_f64(d["v"], r["v"]), axis=1))
        assert bad.size == 0, (t, "vertex", bad[:5], d["v"][bad[:1]], r["v"][bad[:1]])
        bad = np.flatnonzero(~np.all(same_f64(d["act"], r["act"]), axis=1))
        assert bad.size == 0, (t, "action", bad[:5])
        assert np.array_equal(d["parent"], r["parent"]), (t, "parent")
        assert np.array_equal(bits(d["g"]), bits(r["g"])), (t, "g")


def assert_counters_equal(dev, ref):
    assert dev["targets"] == ref["targets"]
    assert dev["extends"] == ref["extends"]
    assert dev["attempts_checked"] == ref["attempts"]
    assert dev["connects"] == ref["connects"]
    assert dev["depth_capped"] == ref["depth_capped"]
    assert dev["halves"] == ref["halves"]


DIR_ON = dict(state_flag=True, state_p=0.3, speed_direction=True, action_flag=True, action_p=0.3)

CASES = [
    # name, (start x, y, goal x, y), batch, seed, max_halves, sampling, adaptive
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1, 11, 0, None, False),
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 64, 11, 0, None, False),
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 4096, 3, 0, DIR_ON, False),
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 64, 3, 0, None, True),
    ("slope-gridmap", (1.0, 0.0, 8.0, 0.0), 1, 3, 20000, None, False),
    ("slope-gridmap", (1.0, 0.0, 8.0, 0.0), 256, 7, 0, None, False),
]


@pytest.mark.parametrize("algorithm", [3, 0])
@pytest.mark.parametrize("name,xy,batch,seed,max_halves,sampling,adaptive", CASES)
def test_planner_loop_equals_oracle(gpu, algorithm, name, xy, batch, seed, max_halves, sampling,
                                    adaptive):
    from global_body_planner_amd import _lib as L
    data, O, start, goal = _setup(name, xy)
    kw = dict(batch=batch, max_time=300.0, seed=seed, max_halves=max_halves, trees=True,
              adaptive=adaptive)
    if sampling is not None:
        kw["sampling"] = L.sampling(**sampling)
    dev = planner.plan_rrt_connect(data, start, goal, algorithm=algorithm, **kw)
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=max_halves, sampling=sampling,
                 adaptive=adaptive)
    assert dev["found"] == ref["found"]
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)
    if ref["found"]:
        assert (dev["meet_a"], dev["meet_b"]) == (ref["meet_a"], ref["meet_b"])
        assert np.array_equal(bits(dev["states"]), bits(ref["states"]))
        assert np.array_equal(bits(dev["actions"]), bits(ref["actions"]))
        # rrt_connect.cpp:304-313: g of the meeting vertices (no yaw weight)
        assert dev["reported_length"] == ref["path_length"]
        assert dev["path_cost"] == ref["path_length"]
        assert dev["reported_yaw"] == ref["path_yaw"]
    print(f"{name} batch {batch} alg {algorithm}: found {ref['found']} after {ref['halves']} "
          f"halves, trees {len(ref['a']['v'])}+{len(ref['b']['v'])}, {ref['attempts']} pair "
          f"checks, {dev['fragile_resolved']} re-decided with glibc by the product")


@pytest.mark.parametrize("algorithm", [3, 0])
@pytest.mark.parametrize("name,xy,batch,seed", [
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 64, 11),
    ("slope-gridmap", (1.0, 0.0, 8.0, 0.0), 256, 7),
])
def test_post_process_equals_oracle(gpu, algorithm, name, xy, batch, seed):
    """postProcessPath (rrt_connect.cpp:139-227) on the found path: the
    shortcut states and connect actions, path_length_ with the reference's
    quirk (the fallback branch adds to path_cost_ only, :202-215), path_yaw_
    and path_cost_."""
    data, O, start, goal = _setup(name, xy)
    raw = O.plan(start, goal, batch=batch, seed=seed)
    assert raw["found"]
    ps, pa, plen, pyaw, pcost = O.post_process_path(raw["states"], raw["actions"])
    dev = planner.plan_rrt_connect(data, start, goal, batch=batch, max_time=300.0, seed=seed,
                                   algorithm=algorithm, post_process=True)
    assert dev["found"] == 1
    assert np.array_equal(bits(dev["states"]), bits(ps))
    assert np.array_equal(bits(dev["actions"]), bits(pa))
    assert dev["reported_length"] == plen
    assert dev["reported_yaw"] == pyaw
    assert dev["path_cost"] == pcost
    print(f"{name}: {raw['states'].shape[0]} -> {ps.shape[0]} states, path_length_ {plen:.4f}, "
          f"path_cost_ {pcost:.4f}")


@pytest.mark.parametrize("algorithm,fragile_eps", [(1, None), (5, None), (5, 1e-5)])
@pytest.mark.parametrize("name,xy,batch,seed,halves", [
    ("synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1024, 3, 300),
    ("slope-gridmap", (1.0, 0.0, 8.0, 0.0), 512, 5, 200),
])
def test_rrt_star_equals_oracle(gpu, name, xy, batch, seed, halves, algorithm, fragile_eps):
    """Batched RRT*-Connect — algorithm 1 (host-driven insertion replay) and
    algorithm 5 (the search resident on the device: neighbourhoods, the
    insertions' connect checks and the ordered choose-parent / rewire replay
    in HBM, gbp_plan_star_config): choose-parent + rewire of every new vertex
    in order (rrt_star_connect.cpp:18-66, neighbourhoods within delta among
    the vertices before it), the recursive g updates of rewired subtrees
    (graph_class.cpp:131-138), and the best connection ranked after every
    iteration, against the oracle's RRT* loop.  A wider FRAGILE margin forces
    the device loop's halts (the insertion checks' included) and host
    re-decisions: same trees."""
    data, O, start, goal = _setup(name, xy)
    dev = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=600.0, seed=seed,
                                        max_halves=halves, trees=True,
                                        device_loop=algorithm == 5, fragile_eps=fragile_eps)
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=halves, star=True, stream_a=401,
                 stream_b=402)
    assert dev["halves"] == ref["halves"] == halves
    assert dev["found"] == ref["found"]
    assert dev["rewires"] == ref["rewires"]
    assert dev["solutions"] == ref["solutions"]
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)
    if ref["found"]:
        assert (dev["meet_a"], dev["meet_b"]) == (ref["best_a"], ref["best_b"])
        assert dev["path_cost"] == ref["best_cost"]
    if fragile_eps is not None:
        assert dev["fragile_resolved"] > 0
        if algorithm == 5:  # the insertion checks' own halt (resume at the replay) ran
            assert dev["halts"][3] > 0, dev["halts"]
    print(f"{name} RRT* batch {batch} alg {algorithm}: {halves} halves, trees {len(ref['a']['v'])}+"
          f"{len(ref['b']['v'])}, {ref['rewires']} rewires, {ref['solutions']} connections, "
          f"{dev['fragile_resolved']} re-decided, halts {dev['halts']}")


def test_rrt_star_small_item_capacity_equals_oracle(gpu, monkeypatch):
    """The device RRT*'s neighbourhood scan with its sizes forced small (read
    when the planner creates its workspace): items of one map position and
    room for only the batch's 1,024 items per half (k_star_count / k_star_fill
    double the chunk until a half's items fit), over 2 workgroups (each takes
    several items; the last of the two to finish scans them all), and the
    connect checks on 2 workgroups of 4 waves (each wave several checks).
    Same trees as the oracle."""
    name, xy, batch, seed, halves = "synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1024, 3, 300
    data, O, start, goal = _setup(name, xy)
    monkeypatch.setenv("GBP_STAR_ITEMS", "1")  # (raised to the batch)
    monkeypatch.setenv("GBP_STAR_CH", "1")
    monkeypatch.setenv("GBP_STAR_GRID", "2")
    dev = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=600.0, seed=seed,
                                        max_halves=halves, trees=True, device_loop=True)
    for k in ("GBP_STAR_ITEMS", "GBP_STAR_CH", "GBP_STAR_GRID"):
        monkeypatch.delenv(k)
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=halves, star=True, stream_a=401,
                 stream_b=402)
    assert dev["halves"] == ref["halves"] == halves
    assert dev["rewires"] == ref["rewires"] > 0
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)


def test_rrt_star_replay_global_paths_equal_oracle(gpu, monkeypatch):
    """k_star_replay with its LDS holdings cut to 2 pairs, 1 new vertex and a
    1-entry subtree queue (GBP_STAR_LDS, read when the planner configures
    the insertion): every later pair, vertex and queued subtree vertex is
    read from / written to global memory, the paths config 5's halves never
    reach (~300 pairs, ~3 vertices).  Same trees as the oracle."""
    name, xy, batch, seed, halves = "synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1024, 3, 300
    data, O, start, goal = _setup(name, xy)
    monkeypatch.setenv("GBP_STAR_LDS", "2,1,1")
    dev = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=600.0, seed=seed,
                                        max_halves=halves, trees=True, device_loop=True)
    monkeypatch.delenv("GBP_STAR_LDS")
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=halves, star=True, stream_a=401,
                 stream_b=402)
    assert dev["halves"] == ref["halves"] == halves
    assert dev["rewires"] == ref["rewires"] > 0
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)


def test_rrt_star_insertion_sets_grow_equals_oracle(gpu, monkeypatch):
    """The device RRT*'s insertion sets sized for 16 neighbour pairs
    (GBP_STAR_PAIRS, read when the planner first configures them): every
    half with more halts at its neighbourhood scan (GBP_PLAN_HALT_STAR_PAIRS),
    the host grows the sets (keeping the run's list of kept connections) and
    the half redoes its stage 6.  Same trees, rewires and best connection as
    the oracle."""
    name, xy, batch, seed, halves = "synth-rough-256", (1.0, 2.55, 4.02, 2.55), 1024, 3, 300
    data, O, start, goal = _setup(name, xy)
    monkeypatch.setenv("GBP_STAR_PAIRS", "16")
    dev = planner.plan_rrt_star_connect(data, start, goal, batch=batch, max_time=600.0, seed=seed,
                                        max_halves=halves, trees=True, device_loop=True)
    monkeypatch.delenv("GBP_STAR_PAIRS")
    ref = O.plan(start, goal, batch=batch, seed=seed, max_halves=halves, star=True, stream_a=401,
                 stream_b=402)
    assert dev["halves"] == ref["halves"] == halves
    assert dev["rewires"] == ref["rewires"] > 0
    assert dev["found"] == ref["found"] and dev["solutions"] == ref["solutions"]
    assert_counters_equal(dev, ref)
    assert_trees_equal(dev, ref)
    if ref["found"]:
        assert (dev["meet_a"], dev["meet_b"]) == (ref["best_a"], ref["best_b"])
        assert dev["path_cost"] == ref["best_cost"]
