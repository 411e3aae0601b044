"""Device-side engine API over the C ABI (torch tensors for HBM residency/streams).

`Terrain` owns one gbp_terrain handle (one GPU).  Every batched call takes
device tensors (float64 AoS states [n, 8] / actions [n, 10]) and enqueues the
HIP kernels on torch's current stream for that device; results are device
tensors.  Host (numpy) variants mirror the `_host` C entry points.
"""
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib as L
from ._lib import check

_VP = ctypes.c_void_p


def _ptr(t):
    return None if t is None else _VP(t.data_ptr())


def _np_ptr(a):
    return None if a is None else a.ctypes.data_as(_VP)


def _np(x):
    return x.detach().cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def _stream(device):
    return _VP(torch.cuda.current_stream(device).cuda_stream)


@dataclass
class PairResult:
    valid: torch.Tensor     # uint8 [n]
    s_new: torch.Tensor     # float64 [n, 8] (rows untouched where flags lack SNEW_SET)
    t_new: torch.Tensor     # float64 [n]
    flags: torch.Tensor     # int32 view of the uint32 flag word [n]
    counts: torch.Tensor    # int32 view of G | V << 16 [n]


@dataclass
class ExtendResult:
    result: torch.Tensor    # int32 TRAPPED / ADVANCED / REACHED
    chosen: torch.Tensor    # int32 candidate index or -1
    s_new: torch.Tensor
    a_new: torch.Tensor
    counts: torch.Tensor
    flags: torch.Tensor     # int32 view: OR of the executed candidates' flags


class Terrain:
    """A FastTerrainMap resident in HBM (x-major heights, fp32 when lossless)."""

    def __init__(self, x, y, z, dx=None, dy=None, dz=None, device=0,
                 storage=L.STORAGE_AUTO, kernel=None, lib=None):
        self._lib = lib if lib is not None else L.load()
        self.device = int(device)
        self.torch_device = torch.device("cuda", self.device)
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        z = np.ascontiguousarray(z, np.float64)
        if z.shape != (x.size, y.size):
            raise ValueError(f"z must be x-major [{x.size}][{y.size}], got {z.shape}")
        nl = [None if v is None else np.ascontiguousarray(v, np.float64) for v in (dx, dy, dz)]
        h = _VP()
        check(self._lib.gbp_terrain_create(self.device, x.size, y.size, _np_ptr(x), _np_ptr(y),
                                           _np_ptr(z), *[_np_ptr(v) for v in nl], int(storage),
                                           ctypes.byref(h)), "gbp_terrain_create")
        self._h = h
        self.nx, self.ny = x.size, y.size
        if kernel is not None:
            self.set_option(L.OPT_KERNEL, kernel)

    @classmethod
    def from_data(cls, td, **kw):
        return cls(td.x, td.y, td.z, td.dx, td.dy, td.dz, **kw)

    # ---- handle ---------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.gbp_terrain_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        nx, ny, st, dev = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        b = (ctypes.c_double * 4)()
        check(self._lib.gbp_terrain_info(self._h, ctypes.byref(nx), ctypes.byref(ny),
                                         ctypes.byref(st), b, ctypes.byref(dev)), "info")
        return {"nx": nx.value, "ny": ny.value, "storage": st.value, "bounds": tuple(b),
                "device": dev.value}

    def set_option(self, key, value):
        check(self._lib.gbp_terrain_set_option(self._h, int(key), int(value)), "set_option")

    def get_option(self, key):
        v = ctypes.c_int64()
        check(self._lib.gbp_terrain_get_option(self._h, int(key), ctypes.byref(v)), "get_option")
        return v.value

    # ---- helpers --------------------------------------------------------------
    def _dev(self, t, dtype, shape_tail=None, name="tensor"):
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t))
        t = t.to(device=self.torch_device, dtype=dtype).contiguous()
        if shape_tail is not None:
            t = t.reshape(-1, *shape_tail)
        return t

    def _empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.torch_device)

    # ---- K1 -------------------------------------------------------------------
    def height(self, xy):
        xy = self._dev(xy, torch.float64, (2,))
        n = xy.shape[0]
        h = self._empty(n, torch.float64)
        nan = self._empty(n, torch.uint8)
        ood = self._empty(n, torch.uint8)
        check(self._lib.gbp_height_batch_dev(self._h, n, _ptr(xy), _ptr(h), _ptr(nan), _ptr(ood),
                                             _stream(self.device)), "height")
        return h, nan, ood

    def normal(self, xy):
        xy = self._dev(xy, torch.float64, (2,))
        n = xy.shape[0]
        nrm = self._empty((n, 3), torch.float64)
        ood = self._empty(n, torch.uint8)
        check(self._lib.gbp_normal_batch_dev(self._h, n, _ptr(xy), _ptr(nrm), _ptr(ood),
                                             _stream(self.device)), "normal")
        return nrm, ood

    def valid_states(self, states, phase):
        s = self._dev(states, torch.float64, (8,))
        n = s.shape[0]
        ph, pall = (None, int(phase)) if np.ndim(phase) == 0 and not isinstance(phase, torch.Tensor) \
            else (self._dev(phase, torch.uint8), 0)
        v = self._empty(n, torch.uint8)
        f = self._empty(n, torch.int32)
        c = self._empty(n, torch.int32)
        check(self._lib.gbp_valid_states_dev(self._h, n, _ptr(s), _ptr(ph), pall, _ptr(v), _ptr(f),
                                             _ptr(c), _stream(self.device)), "valid_states")
        return v, f, c

    # ---- K2: the hot path -----------------------------------------------------
    def validate_pairs(self, s, a, direction, adaptive=False, s_new=None, t_new=None,
                       out=None):
        """Batched isValidStateActionPair[Reverse] (planning_utils.cpp:645-881).

        `s_new` / `t_new` (optional, device) are in/out like the reference's
        reference parameters: rows the reference would not assign keep their
        contents.  `out` may carry preallocated PairResult buffers (bench)."""
        s = self._dev(s, torch.float64, (8,))
        a = self._dev(a, torch.float64, (10,))
        n = s.shape[0]
        if a.shape[0] != n:
            raise ValueError("s and a batch sizes differ")
        if isinstance(direction, torch.Tensor) or np.ndim(direction) > 0:
            d, dall = self._dev(direction, torch.uint8), 0
        else:
            d, dall = None, int(direction)
        if out is None:
            out = PairResult(
                valid=self._empty(n, torch.uint8),
                s_new=self._dev(s_new, torch.float64, (8,)) if s_new is not None
                else torch.full((n, 8), float("nan"), dtype=torch.float64, device=self.torch_device),
                t_new=self._dev(t_new, torch.float64) if t_new is not None
                else torch.full((n,), float("nan"), dtype=torch.float64, device=self.torch_device),
                flags=self._empty(n, torch.int32),
                counts=self._empty(n, torch.int32))
        check(self._lib.gbp_validate_pairs_dev(
            self._h, n, _ptr(s), _ptr(a), _ptr(d), dall, int(bool(adaptive)), _ptr(out.valid),
            _ptr(out.s_new), _ptr(out.t_new), _ptr(out.flags), _ptr(out.counts),
            _stream(self.device)), "validate_pairs")
        return out

    def validate_pairs_raw(self, n, s_ptr, a_ptr, d_ptr, dall, adaptive, valid_ptr, snew_ptr,
                           tnew_ptr, flags_ptr, counts_ptr, stream_ptr):
        """Pointer-level call for the timed loop (no allocation, no checks)."""
        return self._lib.gbp_validate_pairs_dev(self._h, n, s_ptr, a_ptr, d_ptr, dall, adaptive,
                                                valid_ptr, snew_ptr, tnew_ptr, flags_ptr,
                                                counts_ptr, stream_ptr)

    # ---- K3 -------------------------------------------------------------------
    def sample_states(self, n, seed, stream_id, index_base=0, require_phase=-1, max_tries=1):
        st = self._empty((n, 8), torch.float64)
        tries = self._empty(n, torch.int32)
        check(self._lib.gbp_sample_states_dev(self._h, n, seed, stream_id, index_base,
                                              int(require_phase), int(max_tries), _ptr(st),
                                              _ptr(tries), _stream(self.device)), "sample_states")
        return st, tries

    def sample_actions(self, normals, seed, stream_id, index_base=0):
        nr = self._dev(normals, torch.float64, (3,))
        n = nr.shape[0]
        a = self._empty((n, 10), torch.float64)
        check(self._lib.gbp_sample_actions_dev(n, _ptr(nr), seed, stream_id, index_base, _ptr(a),
                                               _stream(self.device)), "sample_actions")
        return a

    # ---- direction-biased sampling (gbp_sampling, params.yaml:21-27) --------------
    def set_sampling(self, cfg=None):
        """Install a _lib.Sampling on the handle (None: off); newConfig's candidates
        (extend, extend_host) and the device planner loop's targets use it."""
        check(self._lib.gbp_terrain_set_sampling(self._h, None if cfg is None else ctypes.byref(cfg)),
              "set_sampling")

    def get_sampling(self):
        cfg = L.Sampling()
        check(self._lib.gbp_terrain_get_sampling(self._h, ctypes.byref(cfg)), "get_sampling")
        return cfg

    def sample_states_dir(self, n, seed, stream_id, s_from, s_to, index_base=0, cfg=None):
        """PlannerClass::randomState(terrain, flag, p, speed, s_from, s_to)
        (planner_class.cpp:22-35, :82-148); cfg None: the handle's."""
        st = self._empty((n, 8), torch.float64)
        f = np.ascontiguousarray(s_from, np.float64).reshape(8)
        t = np.ascontiguousarray(s_to, np.float64).reshape(8)
        check(self._lib.gbp_sample_states_dir_dev(
            self._h, n, seed, stream_id, index_base, None if cfg is None else ctypes.byref(cfg),
            _np_ptr(f), _np_ptr(t), _ptr(st), _stream(self.device)), "sample_states_dir")
        return st

    def sample_actions_dir(self, normals, s, s_near, direction, seed, stream_id, index_base=0,
                           cfg=None):
        """getRandomAction(surf_norm, direction, flag, p, s, s_near)
        (planning_utils.cpp:379-391, :443-515); cfg None: the handle's."""
        nr = self._dev(normals, torch.float64, (3,))
        sv = self._dev(s, torch.float64, (8,))
        sn = self._dev(s_near, torch.float64, (8,))
        n = nr.shape[0]
        if isinstance(direction, torch.Tensor) or np.ndim(direction) > 0:
            d, dall = self._dev(direction, torch.uint8), 0
        else:
            d, dall = None, int(direction)
        a = self._empty((n, 10), torch.float64)
        check(self._lib.gbp_sample_actions_dir_dev(
            self._h, n, _ptr(nr), _ptr(sv), _ptr(sn), _ptr(d), dall,
            None if cfg is None else ctypes.byref(cfg), seed, stream_id, index_base, _ptr(a),
            _stream(self.device)), "sample_actions_dir")
        return a

    def extend(self, s_near, target, direction, seed, extend_base=0, adaptive=False):
        """Batched RRTClass::newConfig + extend acceptance (rrt.cpp:20-102)."""
        sn = self._dev(s_near, torch.float64, (8,))
        tg = self._dev(target, torch.float64, (8,))
        n = sn.shape[0]
        if isinstance(direction, torch.Tensor) or np.ndim(direction) > 0:
            d, dall = self._dev(direction, torch.uint8), 0
        else:
            d, dall = None, int(direction)
        r = ExtendResult(
            result=self._empty(n, torch.int32), chosen=self._empty(n, torch.int32),
            s_new=torch.full((n, 8), float("nan"), dtype=torch.float64, device=self.torch_device),
            a_new=torch.full((n, 10), float("nan"), dtype=torch.float64, device=self.torch_device),
            counts=self._empty(n, torch.int32), flags=self._empty(n, torch.int32))
        check(self._lib.gbp_extend_batch_dev(self._h, n, _ptr(sn), _ptr(tg), _ptr(d), dall,
                                             int(bool(adaptive)), seed, extend_base, _ptr(r.result),
                                             _ptr(r.chosen), _ptr(r.s_new), _ptr(r.a_new),
                                             _ptr(r.counts), _ptr(r.flags), _stream(self.device)),
              "extend")
        return r

    # ---- host variants (numpy in/out) -------------------------------------------
    def validate_pairs_host(self, s, a, direction, adaptive=False):
        s = np.ascontiguousarray(s, np.float64).reshape(-1, 8)
        a = np.ascontiguousarray(a, np.float64).reshape(-1, 10)
        n = s.shape[0]
        if np.ndim(direction) > 0:
            d, dall = np.ascontiguousarray(direction, np.uint8), 0
        else:
            d, dall = None, int(direction)
        valid = np.empty(n, np.uint8)
        s_new = np.full((n, 8), np.nan)
        t_new = np.full(n, np.nan)
        flags = np.empty(n, np.uint32)
        counts = np.empty(n, np.uint32)
        check(self._lib.gbp_validate_pairs_host(self._h, n, _np_ptr(s), _np_ptr(a), _np_ptr(d),
                                                dall, int(bool(adaptive)), _np_ptr(valid),
                                                _np_ptr(s_new), _np_ptr(t_new), _np_ptr(flags),
                                                _np_ptr(counts)), "validate_pairs_host")
        return valid, s_new, t_new, flags, counts

    def resolve_fragile(self, s, a, direction, res, adaptive=False):
        """gbp_resolve_fragile_host on a validate_pairs result: numpy copies
        (valid, s_new, t_new, flags, counts) with every GBP_F_FRAGILE attempt
        re-decided on the host with glibc trig; returns them and the number
        re-decided."""
        s = np.ascontiguousarray(_np(s), np.float64).reshape(-1, 8)
        a = np.ascontiguousarray(_np(a), np.float64).reshape(-1, 10)
        n = s.shape[0]
        if np.ndim(direction) > 0 or isinstance(direction, torch.Tensor):
            d, dall = np.ascontiguousarray(_np(direction), np.uint8), 0
        else:
            d, dall = None, int(direction)
        valid = np.ascontiguousarray(_np(res.valid), np.uint8).copy()
        s_new = np.ascontiguousarray(_np(res.s_new), np.float64).copy()
        t_new = np.ascontiguousarray(_np(res.t_new), np.float64).copy()
        flags = np.ascontiguousarray(_np(res.flags)).view(np.uint32).copy()
        counts = np.ascontiguousarray(_np(res.counts)).view(np.uint32).copy()
        k = ctypes.c_int64(0)
        check(self._lib.gbp_resolve_fragile_host(self._h, n, _np_ptr(s), _np_ptr(a), _np_ptr(d),
                                                 dall, int(bool(adaptive)), _np_ptr(valid),
                                                 _np_ptr(s_new), _np_ptr(t_new), _np_ptr(flags),
                                                 _np_ptr(counts), ctypes.byref(k)),
              "resolve_fragile")
        return (valid, s_new, t_new, flags, counts), k.value

    def valid_states_host(self, states, phase):
        """gbp_valid_states_host (FRAGILE states re-decided on the host):
        (valid, flags, counts) numpy."""
        st = np.ascontiguousarray(_np(states), np.float64).reshape(-1, 8)
        n = st.shape[0]
        if np.ndim(phase) > 0:
            ph, pall = np.ascontiguousarray(_np(phase), np.uint8), 0
        else:
            ph, pall = None, int(phase)
        valid = np.empty(n, np.uint8)
        flags = np.empty(n, np.uint32)
        counts = np.empty(n, np.uint32)
        check(self._lib.gbp_valid_states_host(self._h, n, _np_ptr(st), _np_ptr(ph), pall,
                                              _np_ptr(valid), _np_ptr(flags), _np_ptr(counts)),
              "valid_states_host")
        return valid, flags, counts

    def extend_host(self, s_near, target, direction, seed, extend_base=0, adaptive=False):
        """gbp_extend_batch_host (FRAGILE extends re-decided on the host):
        (result, chosen, s_new, a_new, counts, flags) numpy; s_new / a_new NaN
        where the extend is TRAPPED (written only where the reference writes)."""
        sn = np.ascontiguousarray(_np(s_near), np.float64).reshape(-1, 8)
        tg = np.ascontiguousarray(_np(target), np.float64).reshape(-1, 8)
        n = sn.shape[0]
        if np.ndim(direction) > 0 or isinstance(direction, torch.Tensor):
            d, dall = np.ascontiguousarray(_np(direction), np.uint8), 0
        else:
            d, dall = None, int(direction)
        res = np.empty(n, np.int32)
        cho = np.empty(n, np.int32)
        s_new = np.full((n, 8), np.nan)
        a_new = np.full((n, 10), np.nan)
        counts = np.empty(n, np.uint32)
        flags = np.empty(n, np.uint32)
        check(self._lib.gbp_extend_batch_host(self._h, n, _np_ptr(sn), _np_ptr(tg), _np_ptr(d), dall,
                                              int(bool(adaptive)), seed, extend_base, _np_ptr(res),
                                              _np_ptr(cho), _np_ptr(s_new), _np_ptr(a_new),
                                              _np_ptr(counts), _np_ptr(flags)), "extend_host")
        return res, cho, s_new, a_new, counts, flags

    def height_host(self, xy):
        xy = np.ascontiguousarray(xy, np.float64).reshape(-1, 2)
        n = xy.shape[0]
        h = np.empty(n)
        nan = np.empty(n, np.uint8)
        ood = np.empty(n, np.uint8)
        check(self._lib.gbp_height_batch_host(self._h, n, _np_ptr(xy), _np_ptr(h), _np_ptr(nan),
                                              _np_ptr(ood)), "height_host")
        return h, nan, ood


class DeviceTree:
    """A GraphClass / PlannerClass tree resident in HBM (gbp_tree_*): states,
    actions, parents and g on the device, its vertex count too."""

    def __init__(self, root, device=0, capacity=1 << 16):
        self._lib = L.load()
        self.device = int(device)
        h = ctypes.c_void_p()
        check(self._lib.gbp_tree_create(self.device, int(capacity), ctypes.byref(h)), "tree_create")
        self._h = h
        r = np.ascontiguousarray(root, np.float64).reshape(8)
        check(self._lib.gbp_tree_init(self._h, _np_ptr(r), None), "tree_init")

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.gbp_tree_destroy(self._h)
            self._h = None

    def __len__(self):
        c = ctypes.c_int64(0)
        check(self._lib.gbp_tree_size(self._h, ctypes.byref(c), None), "tree_size")
        return c.value

    def append(self, states, actions, parents):
        s = np.ascontiguousarray(states, np.float64).reshape(-1, 8)
        a = np.ascontiguousarray(actions, np.float64).reshape(-1, 10)
        p = np.ascontiguousarray(parents, np.int32).reshape(-1)
        check(self._lib.gbp_tree_append_host(self._h, s.shape[0], _np_ptr(s), _np_ptr(a), _np_ptr(p),
                                             None), "tree_append")

    def read(self):
        """(states [n][8], actions [n][10], parents [n], g [n]) numpy."""
        n = len(self)
        s, a = np.empty((n, 8)), np.empty((n, 10))
        p, g = np.empty(n, np.int32), np.empty(n)
        check(self._lib.gbp_tree_read(self._h, 0, n, _np_ptr(s), _np_ptr(a), _np_ptr(p), _np_ptr(g),
                                      None), "tree_read")
        return s, a, p, g


class PlanStatus(ctypes.Structure):
    """gbp_plan_status (include/gbp.h)."""
    _fields_ = [("halt", ctypes.c_uint32), ("done", ctypes.c_uint32), ("error", ctypes.c_uint32),
                ("halt_half", ctypes.c_int32), ("n_targets", ctypes.c_int32),
                ("n_validate", ctypes.c_int32), ("n_added", ctypes.c_int32),
                ("added_base", ctypes.c_int32), ("n_conn_added", ctypes.c_int32),
                ("meet_half", ctypes.c_int32), ("meet", ctypes.c_uint64),
                ("ext_base", ctypes.c_int64), ("ext_counter", ctypes.c_int64),
                ("stat_targets", ctypes.c_int64), ("stat_attempts", ctypes.c_int64),
                ("stat_added", ctypes.c_int64), ("stat_conn_added", ctypes.c_int64),
                ("stat_fragile_resolved", ctypes.c_int64), ("stat_depth_capped", ctypes.c_int64),
                ("gate_seq", ctypes.c_uint64), ("stat_nn_rechecks", ctypes.c_int64),
                ("stat_nn_scans", ctypes.c_int64), ("ext_half", ctypes.c_int32),
                ("commit_fin", ctypes.c_uint32), ("ext_prev", ctypes.c_int64),
                ("stat_targets_prev", ctypes.c_int64), ("pre_targets", ctypes.c_int32),
                ("pre_fragile", ctypes.c_int32), ("star_pairs", ctypes.c_int32),
                ("star_rows", ctypes.c_int32), ("n_shared", ctypes.c_int32),
                ("best_a", ctypes.c_int32), ("best_b", ctypes.c_int32), ("star_vrows", ctypes.c_int32),
                ("best_cost", ctypes.c_double), ("stat_star_connects", ctypes.c_int64),
                ("stat_rewires", ctypes.c_int64)]


class PlanWorkspace:
    """Scratch and status of the device planner loop (gbp_plan_ws_*)."""

    def __init__(self, terrain, max_batch):
        self._lib = L.load()
        h = ctypes.c_void_p()
        check(self._lib.gbp_plan_ws_create(terrain._h, int(max_batch), ctypes.byref(h)), "plan_ws")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.gbp_plan_ws_destroy(self._h)
            self._h = None

    def status(self, device=0):
        """gbp_plan_status_read as a dict."""
        st = PlanStatus()
        check(self._lib.gbp_plan_status_read(self._h, ctypes.byref(st), _stream(device)), "status")
        return {k: getattr(st, k) for k, _ in PlanStatus._fields_}

    def reset(self, device=0):
        check(self._lib.gbp_plan_reset(self._h, 0, _stream(device)), "plan_reset")

    def halves(self, terrain, ta, tb, first_half, n_halves, batch, seed, stream_a=101,
               stream_b=102, adaptive=False, first_stage=0, device=0):
        """gbp_plan_halves_dev: enqueue half-iterations first_half ..
        first_half + n_halves - 1 of the device planner loop (no host sync)."""
        check(self._lib.gbp_plan_halves_dev(terrain._h, self._h, ta._h, tb._h, int(first_half),
                                            int(n_halves), int(batch), int(seed), int(stream_a),
                                            int(stream_b), int(bool(adaptive)), int(first_stage),
                                            _stream(device)), "plan_halves")

    def nearest(self, tree, queries):
        """gbp_tree_nearest_dev: nearest vertex of `tree` per query (device tensors)."""
        q = queries.contiguous()
        idx = torch.empty(q.shape[0], dtype=torch.int32, device=q.device)
        check(self._lib.gbp_tree_nearest_dev(self._h, tree._h, q.shape[0], _ptr(q), _ptr(idx),
                                             _stream(q.device.index or 0)), "tree_nearest")
        return idx

    def extend_tree_host(self, terrain, tree, targets, direction, seed, extend_base=0,
                         adaptive=False):
        """gbp_extend_tree_host: RRTClass::extend (rrt.cpp:77-102) of `tree`
        toward every target, nearest neighbour on the device, successors
        appended in target order: (result, new_vertex, n_resolved)."""
        tg = np.ascontiguousarray(targets, np.float64).reshape(-1, 8)
        n = tg.shape[0]
        res, vtx = np.empty(n, np.int32), np.empty(n, np.int32)
        k = ctypes.c_int64(0)
        check(self._lib.gbp_extend_tree_host(terrain._h, self._h, tree._h, n, _np_ptr(tg),
                                             int(direction), int(bool(adaptive)), seed, extend_base,
                                             _np_ptr(res), _np_ptr(vtx), ctypes.byref(k)),
              "extend_tree_host")
        return res, vtx, k.value


def nearest(queries, vertices):
    """Batched PlannerClass::getNearestNeighbor (planner_class.cpp:185-200)."""
    lib = L.load()
    q = queries.contiguous()
    v = vertices.contiguous()
    n = q.shape[0]
    idx = torch.empty(n, dtype=torch.int32, device=q.device)
    dist = torch.empty(n, dtype=torch.float64, device=q.device)
    check(lib.gbp_nearest_batch_dev(n, _ptr(q), v.shape[0], _ptr(v), _ptr(idx), _ptr(dist),
                                    _stream(q.device.index or 0)), "nearest")
    return idx, dist


def neighbors(queries, vertices, radius, max_out=256):
    """Batched PlannerClass::neighborhoodDist (planner_class.cpp:173-182):
    (idx [n, max_out] int32, -1 padded, ascending vertex index; count [n])."""
    lib = L.load()
    q = queries.contiguous()
    v = vertices.contiguous()
    n = q.shape[0]
    out = torch.full((n, max_out), -1, dtype=torch.int32, device=q.device)
    cnt = torch.empty(n, dtype=torch.int32, device=q.device)
    check(lib.gbp_neighbors_batch_dev(n, _ptr(q), v.shape[0], _ptr(v), float(radius), max_out,
                                      _ptr(out), _ptr(cnt), _stream(q.device.index or 0)),
          "neighbors")
    return out, cnt


KNN_MAX = 64


def knn(queries, vertices, n_nearest):
    """Batched PlannerClass::neighborhoodN (planner_class.cpp:151-171) on the
    device: (idx [n, n_nearest] int32, dist [n, n_nearest]) in ascending
    (distance, index) order, -1 / NaN past the tree's size; n_nearest <= 64."""
    lib = L.load()
    q = queries.contiguous()
    v = vertices.contiguous()
    n = q.shape[0]
    out = torch.empty((n, int(n_nearest)), dtype=torch.int32, device=q.device)
    dist = torch.empty((n, int(n_nearest)), dtype=torch.float64, device=q.device)
    check(lib.gbp_knn_batch_dev(n, _ptr(q), v.shape[0], _ptr(v), int(n_nearest), _ptr(out),
                                _ptr(dist), _stream(q.device.index or 0)), "knn")
    return out, dist


def knn_yaw(queries, vertices, n_nearest, length_weight=1.0, yaw_weight=1.0):
    """PlannerClass::neighborhoodN with cost_add_yaw set (planner_class.cpp:157-158):
    the key poseDistance * length_weight + stateYawDistance * yaw_weight, the
    yaws formed with glibc on the host (gbp_knn_yaw_batch_host; the scan runs
    on the device).  numpy in, (idx [n, n_nearest] int32, dist) numpy out."""
    lib = L.load()
    q = np.ascontiguousarray(queries, np.float64).reshape(-1, 8)
    v = np.ascontiguousarray(vertices, np.float64).reshape(-1, 8)
    out = np.empty((q.shape[0], int(n_nearest)), np.int32)
    dist = np.empty((q.shape[0], int(n_nearest)))
    check(lib.gbp_knn_yaw_batch_host(q.shape[0], _np_ptr(q), v.shape[0], _np_ptr(v),
                                     float(length_weight), float(yaw_weight), int(n_nearest),
                                     _np_ptr(out), _np_ptr(dist)), "knn_yaw")
    return out, dist


def device_count():
    lib = L.load()
    c = ctypes.c_int(0)
    lib.gbp_device_count(ctypes.byref(c))
    return c.value
