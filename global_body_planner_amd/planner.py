"""Python binding of the batched RRT-Connect planner (lib/libgbp_planner.so).

The planner itself is C++ (csrc/host/gbp_planner.cpp, declared in
include/gbp_planner.h): a host mirror of the reference's FastTerrainMap /
planning_utils / PlannerClass / RRTConnectClass whose every validity check,
terrain query, nearest-neighbour scan and candidate draw runs on the HIP engine.
This module only marshals `gbp_plan_rrt_connect` (the flat C entry) — the call
the reference's GlobalBodyPlanner::callPlanner makes
(global_body_planner.cpp:89-131 -> RRTConnectClass::buildRRTConnect).
"""
import ctypes
import os

import numpy as np

from . import _lib

PLANNER_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libgbp_planner.so")

_D = ctypes.c_double
_P = ctypes.c_void_p


class PlanParams(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int), ("nx", ctypes.c_int), ("ny", ctypes.c_int),
                ("x", _P), ("y", _P), ("z", _P), ("dx", _P), ("dy", _P), ("dz", _P),
                ("start", _D * 8), ("goal", _D * 8), ("batch", ctypes.c_int),
                ("max_time", _D), ("seed", ctypes.c_uint64), ("post_process", ctypes.c_int),
                ("algorithm", ctypes.c_int), ("max_time_opt", _D),
                ("sampling", _lib.Sampling), ("fragile_eps_fm", ctypes.c_int64),
                ("adaptive", ctypes.c_int), ("nn_stats", ctypes.c_int),
                ("max_halves", ctypes.c_int64),
                ("tree_capacity", ctypes.c_int64), ("tree_v", _P * 2), ("tree_a", _P * 2),
                ("tree_parent", _P * 2), ("tree_g", _P * 2), ("stop_poll", _P),
                ("stop_ctx", _P), ("init_n", ctypes.c_int64 * 2), ("init_v", _P * 2),
                ("init_a", _P * 2), ("init_parent", _P * 2), ("first_half", ctypes.c_int64),
                ("extend_base", ctypes.c_int64), ("stage_timing", ctypes.c_int)]

# int (*stop_poll)(void *ctx, int local_stop, int found)
StopPoll = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int)


class PlanResult(ctypes.Structure):
    _fields_ = [("found", ctypes.c_int), ("time_to_first", _D), ("total_time", _D),
                ("iterations", ctypes.c_int64), ("targets", ctypes.c_int64),
                ("extends", ctypes.c_int64), ("attempts_checked", ctypes.c_int64),
                ("connects", ctypes.c_int64), ("vertices_a", ctypes.c_int64),
                ("vertices_b", ctypes.c_int64), ("n_states", ctypes.c_int),
                ("path_length", _D), ("path_cost", _D), ("path_duration", _D),
                ("rewires", ctypes.c_int64), ("solutions", ctypes.c_int64),
                ("extent_a", _D * 4), ("extent_b", _D * 4),
                ("fragile_resolved", ctypes.c_int64), ("depth_capped", ctypes.c_int64),
                ("status_reads", ctypes.c_int64), ("halts", ctypes.c_int64 * 4),
                ("nn_rechecks", ctypes.c_int64), ("nn_scans", ctypes.c_int64),
                ("reported_length", _D), ("reported_yaw", _D), ("meet_a", ctypes.c_int32),
                ("meet_b", ctypes.c_int32), ("halves", ctypes.c_int64),
                ("polls", ctypes.c_int64), ("stopped_by_peer", ctypes.c_int32),
                ("stage_us", _D * 7), ("stage_halves", ctypes.c_int64)]


_planner = None


def load():
    """Load libgbp_planner.so (raises if it is not built: no fallback)."""
    global _planner
    if _planner is None:
        _lib.load()   # libgbp.so first (the planner links it by rpath)
        if not os.path.exists(PLANNER_PATH):
            raise FileNotFoundError(f"{PLANNER_PATH} is missing: run __graft_entry__.build()")
        L = ctypes.CDLL(PLANNER_PATH)
        L.gbp_plan_rrt_connect.restype = ctypes.c_int
        L.gbp_plan_rrt_connect.argtypes = [ctypes.POINTER(PlanParams), ctypes.POINTER(PlanResult),
                                           _P, _P, ctypes.c_int]
        L.gbp_terrain_arrays_from_csv.restype = ctypes.c_int
        L.gbp_terrain_arrays_from_csv.argtypes = [ctypes.c_char_p, _P, _P, _P, _P, _P, _P, _P, _P,
                                                  ctypes.c_int64]
        L.gbp_attempt_connect_batch.restype = ctypes.c_int
        L.gbp_attempt_connect_batch.argtypes = [_P, ctypes.c_int64, _P, _P, _P, ctypes.c_int,
                                                ctypes.c_int, _P, _P, _P]
        _planner = L
    return _planner


def terrain_from_csv(directory):
    """The C++ ingest (gbp_terrain_arrays_from_csv: TerrainMapPublisher::loadCSV
    + loadMapFromCSV's grid_map geometry + FastTerrainMap::loadDataFromGridMap)
    of the reference CSVs in `directory` -> terrain_data.TerrainData."""
    from .terrain_data import TerrainData
    L = load()
    d = os.fsencode(str(directory))
    nx, ny = ctypes.c_int(0), ctypes.c_int(0)
    rc = L.gbp_terrain_arrays_from_csv(d, ctypes.byref(nx), ctypes.byref(ny), None, None, None,
                                       None, None, None, 0)
    if rc != 0:
        raise _lib.GbpError(rc, f"gbp_terrain_arrays_from_csv({directory})")
    x, y = np.empty(nx.value), np.empty(ny.value)
    z, dx, dy, dz = (np.empty((nx.value, ny.value)) for _ in range(4))
    rc = L.gbp_terrain_arrays_from_csv(d, ctypes.byref(nx), ctypes.byref(ny), x.ctypes.data,
                                       y.ctypes.data, z.ctypes.data, dx.ctypes.data, dy.ctypes.data,
                                       dz.ctypes.data, z.size)
    if rc != 0:
        raise _lib.GbpError(rc, f"gbp_terrain_arrays_from_csv({directory})")
    return TerrainData(x, y, z, dx, dy, dz, name=os.path.basename(str(directory)) + "-cpp-csv")


def start_goal_state(height, x, y):
    """GlobalBodyPlanner::setStartAndGoalStates (global_body_planner.cpp:219-264):
    z = 0.375 + ground height, v = (1, 0, 0), pitch and pitch rate 0."""
    return np.array([x, y, 0.375 + height, 1.0, 0.0, 0.0, 0.0, 0.0], dtype=np.float64)


def plan_rrt_connect(data, start, goal, *, batch=64, max_time=5.0, seed=20251018,
                     post_process=False, device=0, capacity=4096, algorithm=0, max_time_opt=0.0,
                     sampling=None, fragile_eps=None, adaptive=False, nn_stats=False,
                     max_halves=0, trees=False,
                     tree_capacity=1 << 18, stop_poll=None, init_trees=None, first_half=0,
                     extend_base=0, stage_timing=False):
    """Plan start -> goal on terrain `data` (terrain_data.TerrainData).

    algorithm 0: batch-synchronous RRT-Connect, stops at the first solution;
    algorithm 1: batch-synchronous RRT*-Connect, anytime until max_time;
    algorithm 3: as 0, with the search resident on the device (trees in HBM,
      one stream-ordered kernel sequence per half-iteration; same trees and
      path as algorithm 0 for the same seed and batch);
    algorithm 4: as 2, each restart's search resident on the device (what
      buildRRTConnect does by default, RRTConnectClass::set_engine_batch);
    algorithm 5: as 1, the search resident on the device (buildRRTStarConnectDevice:
      same trees, counters and best connection as algorithm 1);
    algorithm 2: RRTConnectClass::buildRRTConnect's anytime restarts
      (rrt_connect.cpp:323-467) on batch-synchronous trees: restart on the
      growing horizon, post-process every solution, keep the cheapest, stop
      once a solution exists and `max_time_opt` seconds have passed.
    Returns a dict with the C result fields plus `states` [n][8] and
    `actions` [n-1][10] (the found path; empty if none).
    sampling: a _lib.Sampling (direction-biased draws, params.yaml:21-27);
    fragile_eps: a wider FRAGILE margin (forces host re-decisions: tests);
    adaptive: the adaptive-step pair checks (params.yaml:16);
    nn_stats: count the matrix-core search's fp64 re-checks (diagnostics);
    max_halves: algorithms 0, 1, 3 stop after this many half-iterations (a
      replayable run; 0 = no limit);
    trees: also return the final trees (out["a"], out["b"]: v, act, parent, g;
      algorithms 0, 1, 3), at most tree_capacity rows each;
    stop_poll: algorithm 3 — f(local_stop, found) -> bool called after every
      group of half-iterations; True stops the search (sharding.stop_together:
      config 4's ranks stop at the first solution of any of them);
    init_trees, first_half, extend_base: algorithms 3 and 5 — a warm start,
      the continuation of a search: init_trees = (a, b) dicts of v [n][8], act
      [n][10], parent [n] (root first, -1; algorithm 3: parents before
      children; algorithm 5: any tree rooted at 0, since rewiring gives
      vertices later parents), the first half-iteration (its targets are the
      draws a search from the roots makes there; even for algorithm 5) and the
      candidate stream's first extend index; max_halves then counts the
      continuation's halves.
    stage_timing: algorithms 3 / 5 — time every half-iteration's stage groups
      with hipEvents (diagnostics): out["stage_us"] = summed microseconds of
      [the half, stages 0-3, 6, 7 (its own stream), 4-5] over
      out["stage_halves"] halves."""
    L = load()
    x = np.ascontiguousarray(data.x, dtype=np.float64)
    y = np.ascontiguousarray(data.y, dtype=np.float64)
    z = np.ascontiguousarray(data.z, dtype=np.float64)
    slopes = [None if getattr(data, k, None) is None else
              np.ascontiguousarray(getattr(data, k), dtype=np.float64) for k in ("dx", "dy", "dz")]
    p = PlanParams()
    p.device, p.nx, p.ny = device, x.size, y.size
    p.x, p.y, p.z = x.ctypes.data, y.ctypes.data, z.ctypes.data
    p.dx, p.dy, p.dz = [None if s is None else s.ctypes.data for s in slopes]
    p.start[:] = [float(v) for v in start]
    p.goal[:] = [float(v) for v in goal]
    p.batch, p.max_time, p.seed, p.post_process = int(batch), float(max_time), int(seed), int(post_process)
    p.algorithm = int(algorithm)
    p.max_time_opt = float(max_time_opt)
    if sampling is not None:
        p.sampling = sampling
    p.fragile_eps_fm = 0 if fragile_eps is None else int(round(fragile_eps * 1e15))
    p.adaptive = int(bool(adaptive))
    p.nn_stats = int(bool(nn_stats))
    p.stage_timing = int(bool(stage_timing))
    p.max_halves = int(max_halves)
    p.first_half, p.extend_base = int(first_half), int(extend_base)
    warm = []
    if init_trees is not None:
        for k, t in enumerate(init_trees):
            arrs = (np.ascontiguousarray(t["v"], np.float64).reshape(-1, 8),
                    np.ascontiguousarray(t["act"], np.float64).reshape(-1, 10),
                    np.ascontiguousarray(t["parent"], np.int32).reshape(-1))
            warm.append(arrs)
            p.init_n[k] = arrs[0].shape[0]
            p.init_v[k], p.init_a[k], p.init_parent[k] = (x.ctypes.data for x in arrs)
    poll_cb = None
    if stop_poll is not None:
        def _poll(ctx, local, found):
            # fail safe: an exception cannot cross ctypes (it would read as 0 =
            # continue), so a poll that raises answers "stop"
            try:
                return 1 if stop_poll(bool(local), bool(found)) else 0
            except BaseException:  # noqa: BLE001 - reported as stop
                return 1
        poll_cb = StopPoll(_poll)
        p.stop_poll = ctypes.cast(poll_cb, _P)
    tb = []
    if trees:
        p.tree_capacity = int(tree_capacity)
        for k in range(2):
            arrs = dict(v=np.zeros((tree_capacity, 8)), act=np.zeros((tree_capacity, 10)),
                        parent=np.zeros(tree_capacity, np.int32), g=np.zeros(tree_capacity))
            tb.append(arrs)
            p.tree_v[k], p.tree_a[k] = arrs["v"].ctypes.data, arrs["act"].ctypes.data
            p.tree_parent[k], p.tree_g[k] = arrs["parent"].ctypes.data, arrs["g"].ctypes.data
    r = PlanResult()
    states = np.zeros((capacity, 8))
    actions = np.zeros((capacity, 10))
    rc = L.gbp_plan_rrt_connect(ctypes.byref(p), ctypes.byref(r), states.ctypes.data,
                                actions.ctypes.data, capacity)
    del poll_cb, warm
    if rc != 0:
        raise _lib.GbpError(rc, "gbp_plan_rrt_connect")
    out = {k: getattr(r, k) for k, _ in PlanResult._fields_}
    out["extent_a"], out["extent_b"] = list(r.extent_a), list(r.extent_b)
    out["halts"] = list(r.halts)
    out["stage_us"] = list(r.stage_us)
    for name, arrs, nv in zip("ab", tb, (r.vertices_a, r.vertices_b)):
        m = min(int(nv), tree_capacity)
        out[name] = {k: v[:m].copy() for k, v in arrs.items()}
    n = r.n_states
    out["states"] = states[:n].copy()
    out["actions"] = actions[:max(n - 1, 0)].copy()
    return out


def plan_rrt_connect_device(data, start, goal, **kw):
    """buildRRTConnectBatched with the search resident on the device (algorithm 3)."""
    return plan_rrt_connect(data, start, goal, algorithm=3, **kw)


def plan_rrt_star_connect(data, start, goal, device_loop=False, **kw):
    """RRTStarConnectClass::buildRRTStarConnect, batch-synchronous (algorithm 1;
    algorithm 5 with device_loop: the search resident on the device, the
    insertions' choose-parent / rewire replayed in HBM)."""
    return plan_rrt_connect(data, start, goal, algorithm=5 if device_loop else 1, **kw)


def plan_rrt_connect_anytime(data, start, goal, max_time_opt=1.0, device_loop=False, **kw):
    """RRTConnectClass::buildRRTConnect's anytime restarts, batch-synchronous
    (algorithm 2; algorithm 4 with device_loop: every restart's search resident
    on the device); `cost_history` is not returned, `solutions` counts the
    restarts that reached the goal."""
    return plan_rrt_connect(data, start, goal, algorithm=4 if device_loop else 2,
                            max_time_opt=max_time_opt, **kw)


def attempt_connect(terrain, s_existing, s, direction, t_s=None, adaptive=False, s_new=None,
                    a_new=None):
    """RRTConnectClass::attemptConnect (rrt_connect.cpp:20-91) for n pairs on an
    engine Terrain (engine.Terrain).  Returns (result[n], s_new[n][8], a_new[n][10]);
    s_new / a_new start as the given arrays (NaN if None) and are written only
    where the reference writes them."""
    L = load()
    se = np.ascontiguousarray(s_existing, np.float64).reshape(-1, 8)
    sq = np.ascontiguousarray(s, np.float64).reshape(-1, 8)
    n = se.shape[0]
    ts = None if t_s is None else np.ascontiguousarray(t_s, np.float64).reshape(n)
    sn = np.full((n, 8), np.nan) if s_new is None else np.array(s_new, np.float64).reshape(n, 8)
    an = np.full((n, 10), np.nan) if a_new is None else np.array(a_new, np.float64).reshape(n, 10)
    res = np.empty(n, np.int32)
    rc = L.gbp_attempt_connect_batch(terrain._h, n, se.ctypes.data, sq.ctypes.data,
                                     None if ts is None else ts.ctypes.data, int(direction),
                                     int(bool(adaptive)), res.ctypes.data, sn.ctypes.data,
                                     an.ctypes.data)
    if rc != 0:
        raise _lib.GbpError(rc, "gbp_attempt_connect_batch")
    return res, sn, an
