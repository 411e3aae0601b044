"""ctypes binding of the CPU restatement (oracle/gbp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package
(global_body_planner_amd/), which must fail loudly without its HIP library.

Parity status: the reference's tests pin nothing and the reference cannot be
compiled in this image (its headers include ROS / grid_map / Eigen), so
bit-level parity against reference OUTPUTS is unpinned; see DESIGN.md and
tests/test_oracle_pins.py for the survey-recorded reference outputs this
restatement is pinned to.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

FORWARD, REVERSE = 0, 1
FLIGHT, STANCE = 0, 1
TRAPPED, ADVANCED, REACHED = 0, 1, 2


def build(force=False):
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    src = os.path.join(_HERE, "gbp_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


class _Terrain(ctypes.Structure):
    _fields_ = [
        ("nx", ctypes.c_int),
        ("ny", ctypes.c_int),
        ("x", ctypes.c_void_p),
        ("y", ctypes.c_void_p),
        ("z", ctypes.c_void_p),
        ("dx", ctypes.c_void_p),
        ("dy", ctypes.c_void_p),
        ("dz", ctypes.c_void_p),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P, I, D, U64, I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_int64
        sig = {
            "orc_set_scan_mode": (None, [I]),
            "orc_get_scan_mode": (I, []),
            "orc_ground_height": (D, [P, D, D, P]),
            "orc_height_is_nan": (I, [P, D, D, P]),
            "orc_surface_normal": (None, [P, D, D, P, P]),
            "orc_apply_stance": (None, [P, P, D, P]),
            "orc_apply_flight": (None, [P, D, P]),
            "orc_apply_stance_reverse": (None, [P, P, D, P]),
            "orc_is_valid_action": (I, [P]),
            "orc_is_valid_pair": (I, [P, P, P, I, I, P, P, P, P]),
            "orc_pose_distance": (D, [P, P]),
            "orc_state_distance": (D, [P, P]),
            "orc_state_yaw_distance": (D, [P, P]),
            "orc_attempt_connect": (I, [P, P, P, D, P, P, I, I]),
            "orc_validate_pairs": (None, [P, I64, P, P, P, I, I, P, P, P, P, P, I]),
            "orc_valid_states": (None, [P, I64, P, P, I, P, P, P, I]),
            "orc_height_batch": (None, [P, I64, P, P, P, P, I]),
            "orc_normal_batch": (None, [P, I64, P, P, P, I]),
            "orc_extend_batch": (None, [P, I64, P, P, P, P, I, I, P, P, P, P, P, I]),
            "orc_nearest_batch": (None, [I64, P, I, P, P, P, I]),
            "orc_neighbors_batch": (None, [I64, P, I, P, D, I, P, P, I]),
            "orc_neighbors_batch_ordered": (None, [I64, P, I, P, D, I, P, P, I, I]),
            "orc_um_rank": (I64, [I64, I64]),
            "orc_um_order": (None, [I64, P]),
            "orc_star_insert_one": (I, [P, P, I, I, P, D, I, I, I, P]),
            "orc_star_stats": (None, [P, I]),
            "orc_knn_batch": (None, [I64, P, I, P, I, P, P, I]),
            "orc_knn_yaw_batch": (None, [I64, P, I, P, I, I, D, D, P, P, I]),
            "orc_state_distance_yaw": (D, [P, P, I, D, D]),
            "orc_sample_states": (None, [P, I64, U64, U64, I64, I, I, P, P, I]),
            "orc_sample_actions": (None, [I64, P, U64, U64, I64, P, I]),
            "orc_sample_states_dir": (None, [P, I64, U64, U64, I64, I, D, I, P, P, P, I]),
            "orc_sample_actions_dir": (None, [I64, P, P, P, P, I, I, D, U64, U64, I64, P, I]),
            "orc_philox4x32_10": (None, [P, P, P]),
            "orc_uniform2": (None, [U64, U64, ctypes.c_uint32, I64, ctypes.c_uint32, P]),
            "orc_rmath": (None, [I, I64, P, P, P]),
            "orc_plan": (I, [P, P, P, P, P, P]),
            "orc_post_process_path": (I, [P, I, P, P, I, P, P, P, P, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


class _Tree(ctypes.Structure):
    _fields_ = [("cap", ctypes.c_int), ("n", ctypes.c_int), ("v", ctypes.c_void_p),
                ("a", ctypes.c_void_p), ("parent", ctypes.c_void_p), ("g", ctypes.c_void_p),
                ("y", ctypes.c_void_p), ("child", ctypes.c_void_p), ("sibling", ctypes.c_void_p)]


class _PlanCfg(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int), ("seed", ctypes.c_uint64), ("stream_a", ctypes.c_uint64),
                ("stream_b", ctypes.c_uint64), ("adaptive", ctypes.c_int),
                ("state_flag", ctypes.c_int), ("state_speed_direction", ctypes.c_int),
                ("action_flag", ctypes.c_int), ("state_p", ctypes.c_double),
                ("action_p", ctypes.c_double), ("extend_base", ctypes.c_int64),
                ("max_halves", ctypes.c_int64), ("star", ctypes.c_int),
                ("star_delta", ctypes.c_double), ("nthreads", ctypes.c_int),
                ("first_half", ctypes.c_int64), ("warm", ctypes.c_int),
                ("star_order", ctypes.c_int)]


class _PlanOut(ctypes.Structure):
    _fields_ = [("found", ctypes.c_int), ("meet_a", ctypes.c_int), ("meet_b", ctypes.c_int),
                ("meet_half", ctypes.c_int64), ("halves", ctypes.c_int64),
                ("targets", ctypes.c_int64), ("extends", ctypes.c_int64),
                ("attempts", ctypes.c_int64), ("connects", ctypes.c_int64),
                ("depth_capped", ctypes.c_int64), ("rewires", ctypes.c_int64),
                ("solutions", ctypes.c_int64), ("ext_counter", ctypes.c_int64),
                ("draws_a", ctypes.c_int64), ("draws_b", ctypes.c_int64),
                ("path_length", ctypes.c_double), ("path_yaw", ctypes.c_double),
                ("best_a", ctypes.c_int), ("best_b", ctypes.c_int),
                ("best_cost", ctypes.c_double)]


class OracleTerrain:
    """A FastTerrainMap restated on the CPU (x-major arrays, float64)."""

    def __init__(self, x, y, z, dx=None, dy=None, dz=None):
        self.x = _c(x, np.float64)
        self.y = _c(y, np.float64)
        self.z = _c(z, np.float64)
        self.nx, self.ny = self.x.size, self.y.size
        assert self.z.shape == (self.nx, self.ny)
        self.dx = None if dx is None else _c(dx, np.float64)
        self.dy = None if dy is None else _c(dy, np.float64)
        self.dz = None if dz is None else _c(dz, np.float64)
        self._s = _Terrain(self.nx, self.ny, self.x.ctypes.data, self.y.ctypes.data,
                           self.z.ctypes.data,
                           None if self.dx is None else self.dx.ctypes.data,
                           None if self.dy is None else self.dy.ctypes.data,
                           None if self.dz is None else self.dz.ctypes.data)

    @classmethod
    def from_data(cls, td):
        return cls(td.x, td.y, td.z, td.dx, td.dy, td.dz)

    @property
    def ref(self):
        return ctypes.byref(self._s)

    # scalar reference calls -------------------------------------------------
    def ground_height(self, x, y):
        o = ctypes.c_int(0)
        h = lib().orc_ground_height(self.ref, x, y, ctypes.byref(o))
        return h, bool(o.value)

    def height_is_nan(self, x, y):
        o = ctypes.c_int(0)
        r = lib().orc_height_is_nan(self.ref, x, y, ctypes.byref(o))
        return bool(r), bool(o.value)

    # batches ------------------------------------------------------------------
    def height_batch(self, xy, nthreads=1):
        xy = _c(xy, np.float64).reshape(-1, 2)
        n = xy.shape[0]
        h = np.empty(n)
        nan = np.empty(n, np.uint8)
        ood = np.empty(n, np.uint8)
        lib().orc_height_batch(self.ref, n, _p(xy), _p(h), _p(nan), _p(ood), nthreads)
        return h, nan, ood

    def normal_batch(self, xy, nthreads=1):
        xy = _c(xy, np.float64).reshape(-1, 2)
        n = xy.shape[0]
        nrm = np.empty((n, 3))
        ood = np.empty(n, np.uint8)
        lib().orc_normal_batch(self.ref, n, _p(xy), _p(nrm), _p(ood), nthreads)
        return nrm, ood

    def valid_states(self, states, phase, nthreads=1):
        states = _c(states, np.float64).reshape(-1, 8)
        n = states.shape[0]
        valid = np.empty(n, np.uint8)
        flags = np.empty(n, np.uint32)
        counts = np.empty(n, np.uint32)
        ph = None
        pall = 0
        if np.ndim(phase) == 0:
            pall = int(phase)
        else:
            ph = _c(phase, np.uint8)
        lib().orc_valid_states(self.ref, n, _p(states), _p(ph), pall, _p(valid), _p(flags),
                               _p(counts), nthreads)
        return valid, flags, counts

    def validate_pairs(self, s, a, direction, adaptive=False, s_new_init=None, t_new_init=None,
                       nthreads=1):
        s = _c(s, np.float64).reshape(-1, 8)
        a = _c(a, np.float64).reshape(-1, 10)
        n = s.shape[0]
        valid = np.empty(n, np.uint8)
        s_new = np.full((n, 8), np.nan) if s_new_init is None else _c(s_new_init, np.float64).copy()
        t_new = np.full(n, np.nan) if t_new_init is None else _c(t_new_init, np.float64).copy()
        flags = np.empty(n, np.uint32)
        counts = np.empty(n, np.uint32)
        d = None
        dall = 0
        if np.ndim(direction) == 0:
            dall = int(direction)
        else:
            d = _c(direction, np.uint8)
        lib().orc_validate_pairs(self.ref, n, _p(s), _p(a), _p(d), dall, int(bool(adaptive)),
                                 _p(valid), _p(s_new), _p(t_new), _p(flags), _p(counts), nthreads)
        return valid, s_new, t_new, flags, counts

    def extend_batch(self, s_near, target, actions, direction, adaptive=False, nthreads=1):
        s_near = _c(s_near, np.float64).reshape(-1, 8)
        target = _c(target, np.float64).reshape(-1, 8)
        n = s_near.shape[0]
        actions = _c(actions, np.float64).reshape(n, 6, 10)
        result = np.empty(n, np.int32)
        chosen = np.empty(n, np.int32)
        s_new = np.full((n, 8), np.nan)
        a_new = np.full((n, 10), np.nan)
        counts = np.empty(n, np.uint32)
        d = None
        dall = 0
        if np.ndim(direction) == 0:
            dall = int(direction)
        else:
            d = _c(direction, np.uint8)
        lib().orc_extend_batch(self.ref, n, _p(s_near), _p(target), _p(actions), _p(d), dall,
                               int(bool(adaptive)), _p(result), _p(chosen), _p(s_new), _p(a_new),
                               _p(counts), nthreads)
        return result, chosen, s_new, a_new, counts

    def sample_states(self, n, seed, stream_id, index_base=0, require_phase=-1, max_tries=1,
                      nthreads=1):
        st = np.empty((n, 8))
        tries = np.empty(n, np.int32)
        lib().orc_sample_states(self.ref, n, seed, stream_id, index_base, require_phase,
                                max_tries, _p(st), _p(tries), nthreads)
        return st, tries

    def sample_states_dir(self, n, seed, stream_id, s_from, s_to, index_base=0, state_flag=True,
                          state_p=0.05, speed_direction=False, nthreads=1):
        """PlannerClass::randomState(terrain, flag, p, speed, s_from, s_to)
        (planner_class.cpp:22-35, :82-148), one try per index."""
        st = np.empty((n, 8))
        f, t = _c(s_from, np.float64), _c(s_to, np.float64)
        lib().orc_sample_states_dir(self.ref, n, seed, stream_id, index_base, int(bool(state_flag)),
                                    float(state_p), int(bool(speed_direction)), _p(f), _p(t),
                                    _p(st), nthreads)
        return st

    def plan(self, start, goal, *, batch, seed, stream_a=101, stream_b=102, max_halves=0,
             adaptive=False, sampling=None, star=False, star_delta=3.0, extend_base=0,
             capacity=200000, nthreads=1, init_trees=None, first_half=0,
             star_order="reference"):
        """The batch-synchronous RRT-Connect (RRT*-Connect with star=True) the
        engine runs, restated on the CPU (orc_plan): returns a dict with the
        counters, the meeting / best vertices, and each tree's arrays
        ("a"/"b": v, act, parent, g, y).  sampling: dict of gbp_sampling
        fields (state_flag, state_p, speed_direction, action_flag, action_p).
        nthreads: OpenMP threads for the per-target / per-connection passes
        (same result for any count: insertion stays in order).
        init_trees / first_half: a warm start (the continuation of a search):
        (a, b) dicts of v [n][8], act [n][10], parent [n] (root first, -1),
        the first half-iteration; max_halves counts the continuation's.
        star_order: RRT* neighbourhoods in the vertex map's iteration order
        ("reference", planner_class.cpp:176-179) or "ascending" index (the
        pre-round-6 form, kept to show the two build different trees)."""
        trees, keep = [], []
        for k in range(2):
            arrs = dict(v=np.zeros((capacity, 8)), act=np.zeros((capacity, 10)),
                        parent=np.zeros(capacity, np.int32), g=np.zeros(capacity),
                        y=np.zeros(capacity), child=np.zeros(capacity, np.int32),
                        sibling=np.zeros(capacity, np.int32))
            n0 = 0
            if init_trees is not None:
                t = init_trees[k]
                n0 = int(np.asarray(t["parent"]).shape[0])
                arrs["v"][:n0] = np.asarray(t["v"], np.float64).reshape(-1, 8)
                arrs["act"][:n0] = np.asarray(t["act"], np.float64).reshape(-1, 10)
                arrs["parent"][:n0] = np.asarray(t["parent"], np.int32)
            keep.append(arrs)
            trees.append(_Tree(capacity, n0, *(arrs[k].ctypes.data for k in
                                               ("v", "act", "parent", "g", "y", "child", "sibling"))))
        tr = (_Tree * 2)(*trees)
        sm = sampling or {}
        cfg = _PlanCfg(int(batch), int(seed), int(stream_a), int(stream_b), int(bool(adaptive)),
                       int(bool(sm.get("state_flag", False))),
                       int(bool(sm.get("speed_direction", False))),
                       int(bool(sm.get("action_flag", False))), float(sm.get("state_p", 0.0)),
                       float(sm.get("action_p", 0.0)), int(extend_base), int(max_halves),
                       int(bool(star)), float(star_delta), int(nthreads), int(first_half),
                       int(init_trees is not None), {"reference": 0, "ascending": 1}[star_order])
        out = _PlanOut()
        st, gl = _c(start, np.float64), _c(goal, np.float64)
        rc = lib().orc_plan(self.ref, _p(st), _p(gl), ctypes.byref(cfg), tr, ctypes.byref(out))
        if rc != 0:
            raise RuntimeError(f"orc_plan returned {rc}")
        res = {k: getattr(out, k) for k, _ in _PlanOut._fields_}
        for name, t, arrs in zip("ab", tr, keep):
            n = t.n
            res[name] = {k: arrs[k][:n].copy() for k in ("v", "act", "parent", "g", "y")}
        if res["found"] and not star:
            res["states"], res["actions"] = _join_path(res["a"], res["b"], res["meet_a"],
                                                       res["meet_b"])
        return res

    def star_insert_one(self, v, parent, idx, nn, a_new, direction, delta=3.0,
                        order="reference", adaptive=False):
        """One RRT* insertion (rrt_star_connect.cpp:18-66, orc_star_insert_one):
        v [idx+1][8] (vertex idx newly added), parent [idx] a tree rooted at 0,
        nearest vertex nn, newConfig's action a_new.  Returns the tree after
        choose-parent and rewire (v, act, parent, g, y) and the rewire count."""
        v = _c(v, np.float64).reshape(-1, 8)
        n = idx + 1
        arrs = dict(v=v[:n].copy(), act=np.zeros((n, 10)), parent=np.full(n, -1, np.int32),
                    g=np.zeros(n), y=np.zeros(n), child=np.zeros(n, np.int32),
                    sibling=np.zeros(n, np.int32))
        arrs["parent"][:idx] = np.asarray(parent, np.int32)[:idx]
        arrs["act"][idx] = _c(a_new, np.float64)
        t = _Tree(n, n, *(arrs[k].ctypes.data for k in
                          ("v", "act", "parent", "g", "y", "child", "sibling")))
        rw = ctypes.c_int64(0)
        rc = lib().orc_star_insert_one(self.ref, ctypes.byref(t), int(idx), int(nn),
                                       _p(arrs["act"][idx].copy()), float(delta), int(direction),
                                       int(bool(adaptive)),
                                       {"reference": 0, "ascending": 1}[order], ctypes.byref(rw))
        if rc != 0:
            raise RuntimeError(f"orc_star_insert_one returned {rc}")
        return {k: arrs[k] for k in ("v", "act", "parent", "g", "y")}, rw.value

    def post_process_path(self, states, actions, adaptive=False):
        """rrt_connect.cpp:139-227 -> (states, actions, path_length_, path_yaw_, path_cost_)."""
        st = _c(states, np.float64).reshape(-1, 8)
        ac = _c(actions, np.float64).reshape(-1, 10)
        n = st.shape[0]
        os_, oa = np.zeros((n, 8)), np.zeros((max(n - 1, 1), 10))
        L, Y, C = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        m = lib().orc_post_process_path(self.ref, n, _p(st), _p(ac), int(bool(adaptive)), _p(os_),
                                        _p(oa), ctypes.byref(L), ctypes.byref(Y), ctypes.byref(C))
        return os_[:m].copy(), oa[:m - 1].copy(), L.value, Y.value, C.value

    def attempt_connect(self, s_existing, s, direction, t_s=0.0, adaptive=False):
        s_existing = _c(s_existing, np.float64)
        s = _c(s, np.float64)
        s_new = np.full(8, np.nan)
        a_new = np.full(10, np.nan)
        r = lib().orc_attempt_connect(self.ref, _p(s_existing), _p(s), float(t_s), _p(s_new),
                                      _p(a_new), int(direction), int(bool(adaptive)))
        return r, s_new, a_new


def _path_from_start(tree, idx):  # rrt.cpp:107-118
    path = [idx]
    while idx != 0:
        idx = int(tree["parent"][idx])
        path.append(idx)
    return path[::-1]


def _join_path(ta, tb, ia, ib):
    """rrt_connect.cpp:386-401: Ta's root -> ia, then Tb's ib -> root (ib itself
    dropped), with Tb's actions in reverse (getActionSequenceReverse)."""
    pa = _path_from_start(ta, ia)
    pb = _path_from_start(tb, ib)[::-1]
    act_b = [tb["act"][i] for i in pb[:-1]]
    pb = pb[1:]
    states = np.array([ta["v"][i] for i in pa] + [tb["v"][i] for i in pb])
    actions = np.array([ta["act"][i] for i in pa[1:]] + act_b).reshape(-1, 10)
    return states, actions


def sample_actions(normals, seed, stream_id, index_base=0, nthreads=1):
    normals = _c(normals, np.float64).reshape(-1, 3)
    n = normals.shape[0]
    out = np.empty((n, 10))
    lib().orc_sample_actions(n, _p(normals), seed, stream_id, index_base, _p(out), nthreads)
    return out


def sample_actions_dir(normals, s, s_near, direction, seed, stream_id, index_base=0,
                       action_flag=True, action_p=0.15, nthreads=1):
    """getRandomAction(surf_norm, direction, flag, p, s, s_near)
    (planning_utils.cpp:379-391, :443-515)."""
    normals = _c(normals, np.float64).reshape(-1, 3)
    n = normals.shape[0]
    s = _c(s, np.float64).reshape(n, 8)
    s_near = _c(s_near, np.float64).reshape(n, 8)
    if np.ndim(direction) > 0:
        d, dall = _c(direction, np.uint8), 0
    else:
        d, dall = None, int(direction)
    out = np.empty((n, 10))
    lib().orc_sample_actions_dir(n, _p(normals), _p(s), _p(s_near), _p(d), dall,
                                 int(bool(action_flag)), float(action_p), seed, stream_id,
                                 index_base, _p(out), nthreads)
    return out


def nearest_batch(queries, verts, nthreads=1):
    q = _c(queries, np.float64).reshape(-1, 8)
    v = _c(verts, np.float64).reshape(-1, 8)
    idx = np.empty(q.shape[0], np.int32)
    dist = np.empty(q.shape[0])
    lib().orc_nearest_batch(q.shape[0], _p(q), v.shape[0], _p(v), _p(idx), _p(dist), nthreads)
    return idx, dist


def neighbors_batch(queries, verts, radius, max_out=256, nthreads=1, order="reference"):
    """planner_class.cpp:173-182 over a map holding the rows of `verts` as keys
    0..n-1, in its iteration order ("reference") or ascending index:
    (out [n, max_out] -1 padded, count [n])."""
    q = _c(queries, np.float64).reshape(-1, 8)
    v = _c(verts, np.float64).reshape(-1, 8)
    out = np.full((q.shape[0], max_out), -1, np.int32)
    cnt = np.empty(q.shape[0], np.int32)
    lib().orc_neighbors_batch_ordered(q.shape[0], _p(q), v.shape[0], _p(v), float(radius),
                                      int(max_out), _p(out), _p(cnt),
                                      {"reference": 0, "ascending": 1}[order], nthreads)
    return out, cnt


def star_stats(reset=False):
    """orc_star_stats: RRT* insertion diagnostics (see gbp_oracle.h)."""
    out = np.zeros(8, np.int64)
    lib().orc_star_stats(_p(out), int(bool(reset)))
    keys = ("insertions", "neighbours", "max_neighbours", "rewires", "subtree_vertices",
            "max_subtree", "subtree_depth_sum", "max_depth")
    return dict(zip(keys, out.tolist()))


def um_rank(keys, n):
    """Positions of `keys` when a std::unordered_map<int, State> holding keys
    0..n-1 (graph_class.h:155) is iterated (libstdc++, orc_um_rank)."""
    return np.array([lib().orc_um_rank(int(k), int(n)) for k in np.atleast_1d(keys)], np.int64)


def um_order(n):
    """The keys 0..n-1 in that map's iteration order (orc_um_order)."""
    out = np.empty(int(n), np.int32)
    lib().orc_um_order(int(n), _p(out))
    return out


def knn_batch(queries, verts, n_nearest, nthreads=1):
    """planner_class.cpp:151-171 (neighborhoodN): (idx [n, k], dist [n, k])."""
    q = _c(queries, np.float64).reshape(-1, 8)
    v = _c(verts, np.float64).reshape(-1, 8)
    out = np.empty((q.shape[0], n_nearest), np.int32)
    dist = np.empty((q.shape[0], n_nearest))
    lib().orc_knn_batch(q.shape[0], _p(q), v.shape[0], _p(v), int(n_nearest), _p(out), _p(dist),
                        nthreads)
    return out, dist


def knn_yaw_batch(queries, verts, n_nearest, length_weight, yaw_weight, nthreads=1):
    """neighborhoodN with cost_add_yaw set (planner_class.cpp:157-158): the key
    poseDistance * length_weight + stateYawDistance * yaw_weight (glibc atan2)."""
    q = _c(queries, np.float64).reshape(-1, 8)
    v = _c(verts, np.float64).reshape(-1, 8)
    out = np.empty((q.shape[0], n_nearest), np.int32)
    dist = np.empty((q.shape[0], n_nearest))
    lib().orc_knn_yaw_batch(q.shape[0], _p(q), v.shape[0], _p(v), int(n_nearest), 1,
                            float(length_weight), float(yaw_weight), _p(out), _p(dist), nthreads)
    return out, dist


def state_distance_yaw(q1, q2, length_weight, yaw_weight):
    return lib().orc_state_distance_yaw(_p(_c(q1, np.float64)), _p(_c(q2, np.float64)), 1,
                                        float(length_weight), float(yaw_weight))


def apply_stance(s, a, t):
    o = np.empty(8)
    lib().orc_apply_stance(_p(_c(s, np.float64)), _p(_c(a, np.float64)), float(t), _p(o))
    return o


def apply_flight(s, t):
    o = np.empty(8)
    lib().orc_apply_flight(_p(_c(s, np.float64)), float(t), _p(o))
    return o


def apply_stance_reverse(s, a, t):
    o = np.empty(8)
    lib().orc_apply_stance_reverse(_p(_c(s, np.float64)), _p(_c(a, np.float64)), float(t), _p(o))
    return o


def is_valid_action(a):
    return bool(lib().orc_is_valid_action(_p(_c(a, np.float64))))


def state_distance(q1, q2):
    return lib().orc_state_distance(_p(_c(q1, np.float64)), _p(_c(q2, np.float64)))


def pose_distance(q1, q2):
    return lib().orc_pose_distance(_p(_c(q1, np.float64)), _p(_c(q2, np.float64)))


def state_yaw_distance(q1, q2):
    return lib().orc_state_yaw_distance(_p(_c(q1, np.float64)), _p(_c(q2, np.float64)))


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    o = np.empty(4, np.uint32)
    lib().orc_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def rmath(fn, x, y=None):
    """The samplers' reproducible log / sincos / atan2 / acos (orc_rmath)."""
    x = _c(x, np.float64).ravel()
    yy = None if y is None else _c(y, np.float64).ravel()
    out = np.empty(2 * x.size if fn == 1 else x.size)
    lib().orc_rmath(int(fn), x.size, _p(x), _p(yy), _p(out))
    return out.reshape(-1, 2) if fn == 1 else out


def set_scan_mode(mode):
    lib().orc_set_scan_mode(int(mode))


def get_scan_mode():
    return lib().orc_get_scan_mode()
