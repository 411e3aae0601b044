"""ctypes binding of libgbp.so (the C ABI in include/gbp.h).

The library is built in-tree (global_body_planner_amd/lib/libgbp.so) by
__graft_entry__.build() / `make -C global_body_planner_amd/csrc`.  There is no
fallback: if the library is missing or fails to load, importing the engine
raises, so a GPU run can never silently compute on the CPU.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgbp.so")

# ---- constants mirrored from include/gbp.h ---------------------------------
OK = 0
FLIGHT, STANCE, CONNECT_STANCE = 0, 1, 2
FORWARD, REVERSE = 0, 1
TRAPPED, ADVANCED, REACHED = 0, 1, 2
NUM_GEN_STATES = 6
F_VALID, F_OOD, F_NAN, F_SNEW_SET, F_TNEW_SET, F_FRAGILE, F_LIMIT, F_RESOLVED = 1, 2, 4, 8, 16, 32, 64, 128
MAX_SAMPLES = 7000
F_STAGE_SHIFT = 8
F_STAGE_MASK = 0xF << F_STAGE_SHIFT
STORAGE_AUTO, STORAGE_F32, STORAGE_F64 = 0, 1, 2
OPT_KERNEL, OPT_BLOCK, OPT_WAVES, OPT_LDS_COORDS, OPT_HELPERS = 1, 2, 4, 5, 8
OPT_AFFINE_COORDS, OPT_COORD_MODE, OPT_XCD_MAP, OPT_FAST_RCP, OPT_FRAGILE_EPS = 9, 10, 13, 14, 15
OPT_NN_STATS = 18
PLAN_HALT_TARGETS, PLAN_HALT_EXTEND, PLAN_HALT_CONNECT = 1, 2, 4
PLAN_HALT_STAR, PLAN_HALT_STAR_PAIRS = 8, 16
KERNEL_DIRECT, KERNEL_PERSISTENT = 0, 1

EXPORTS = [
    "gbp_version", "gbp_status_string", "gbp_device_count", "gbp_device_alloc",
    "gbp_device_free", "gbp_memcpy_h2d", "gbp_memcpy_d2h", "gbp_stream_synchronize",
    "gbp_terrain_create", "gbp_terrain_destroy", "gbp_terrain_info",
    "gbp_terrain_set_option", "gbp_terrain_get_option",
    "gbp_height_batch_dev", "gbp_height_batch_host",
    "gbp_normal_batch_dev", "gbp_normal_batch_host",
    "gbp_valid_states_dev", "gbp_valid_states_host",
    "gbp_validate_pairs_dev", "gbp_validate_pairs_host",
    "gbp_sample_states_dev", "gbp_sample_states_host", "gbp_sample_actions_dev",
    "gbp_sample_actions_host", "gbp_terrain_set_sampling", "gbp_terrain_get_sampling",
    "gbp_sample_states_dir_dev", "gbp_sample_states_dir_host", "gbp_sample_actions_dir_dev",
    "gbp_sample_actions_dir_host",
    "gbp_extend_batch_dev", "gbp_extend_batch_host",
    "gbp_nearest_batch_dev", "gbp_nearest_batch_host",
    "gbp_neighbors_batch_dev", "gbp_neighbors_batch_host", "gbp_knn_batch_dev", "gbp_knn_batch_host",
    "gbp_knn_yaw_batch_dev", "gbp_knn_yaw_batch_host", "gbp_host_yaw",
    "gbp_resolve_fragile_host", "gbp_resolve_fragile_states_host", "gbp_extend_resolve_host",
    "gbp_stream_create", "gbp_stream_destroy",
    "gbp_tree_create", "gbp_tree_destroy", "gbp_tree_init", "gbp_tree_reserve", "gbp_tree_capacity",
    "gbp_tree_size", "gbp_tree_read", "gbp_tree_append_host", "gbp_tree_load_host",
    "gbp_tree_device_ptrs", "gbp_vertex_map_order", "gbp_vertex_map_rank",
    "gbp_plan_ws_create", "gbp_plan_ws_destroy", "gbp_plan_reset", "gbp_plan_half_dev",
    "gbp_plan_halves_dev", "gbp_plan_star_config", "gbp_plan_stage_timing", "gbp_plan_stage_times",
    "gbp_plan_status_read", "gbp_plan_resolve_host", "gbp_extend_tree_dev",
    "gbp_extend_tree_finish_dev", "gbp_extend_tree_host", "gbp_tree_nearest_dev",
]


class Sampling(ctypes.Structure):
    """gbp_sampling (include/gbp.h): direction-biased sampling, params.yaml:21-27."""
    _fields_ = [("state_flag", ctypes.c_int32), ("state_speed_direction", ctypes.c_int32),
                ("state_p", ctypes.c_double), ("action_flag", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("action_p", ctypes.c_double)]


def sampling(state_flag=False, state_p=0.05, speed_direction=False, action_flag=False,
             action_p=0.15):
    """A Sampling record (defaults: the reference's rrt.h:194-200 thresholds, flags off)."""
    return Sampling(int(bool(state_flag)), int(bool(speed_direction)), float(state_p),
                    int(bool(action_flag)), 0, float(action_p))


class GbpError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        msg = _lib.gbp_status_string(status).decode() if _lib is not None else str(status)
        super().__init__(f"{what}: gbp status {status} ({msg})")


_lib = None


def load(path=None):
    """Load libgbp.so (raises OSError / FileNotFoundError if it is not built).

    `path` loads another build of the same ABI (diagnostic timing builds) as a
    separate handle; the default library is cached."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"{p} is missing: build the HIP engine first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(p)
    P, I, I64, U64, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_size_t
    sig = {
        "gbp_version": (I, []),
        "gbp_status_string": (ctypes.c_char_p, [I]),
        "gbp_device_count": (I, [P]),
        "gbp_device_alloc": (I, [I, SZ, P]),
        "gbp_device_free": (I, [P]),
        "gbp_memcpy_h2d": (I, [P, P, SZ, P]),
        "gbp_memcpy_d2h": (I, [P, P, SZ, P]),
        "gbp_stream_synchronize": (I, [P]),
        "gbp_terrain_create": (I, [I, I, I, P, P, P, P, P, P, I, P]),
        "gbp_terrain_destroy": (I, [P]),
        "gbp_terrain_info": (I, [P, P, P, P, P, P]),
        "gbp_terrain_set_option": (I, [P, I, I64]),
        "gbp_terrain_get_option": (I, [P, I, P]),
        "gbp_height_batch_dev": (I, [P, I64, P, P, P, P, P]),
        "gbp_height_batch_host": (I, [P, I64, P, P, P, P]),
        "gbp_normal_batch_dev": (I, [P, I64, P, P, P, P]),
        "gbp_normal_batch_host": (I, [P, I64, P, P, P]),
        "gbp_valid_states_dev": (I, [P, I64, P, P, I, P, P, P, P]),
        "gbp_valid_states_host": (I, [P, I64, P, P, I, P, P, P]),
        "gbp_validate_pairs_dev": (I, [P, I64, P, P, P, I, I, P, P, P, P, P, P]),
        "gbp_validate_pairs_host": (I, [P, I64, P, P, P, I, I, P, P, P, P, P]),
        "gbp_sample_states_dev": (I, [P, I64, U64, U64, I64, I, I, P, P, P]),
        "gbp_sample_actions_dev": (I, [I64, P, U64, U64, I64, P, P]),
        "gbp_sample_states_host": (I, [P, I64, U64, U64, I64, I, I, P, P]),
        "gbp_sample_actions_host": (I, [P, I64, P, U64, U64, I64, P]),
        "gbp_terrain_set_sampling": (I, [P, P]),
        "gbp_terrain_get_sampling": (I, [P, P]),
        "gbp_sample_states_dir_dev": (I, [P, I64, U64, U64, I64, P, P, P, P, P]),
        "gbp_sample_states_dir_host": (I, [P, I64, U64, U64, I64, P, P, P, P]),
        "gbp_sample_actions_dir_dev": (I, [P, I64, P, P, P, P, I, P, U64, U64, I64, P, P]),
        "gbp_sample_actions_dir_host": (I, [P, I64, P, P, P, P, I, P, U64, U64, I64, P]),
        "gbp_extend_batch_dev": (I, [P, I64, P, P, P, I, I, U64, I64, P, P, P, P, P, P, P]),
        "gbp_extend_batch_host": (I, [P, I64, P, P, P, I, I, U64, I64, P, P, P, P, P, P]),
        "gbp_resolve_fragile_host": (I, [P, I64, P, P, P, I, I, P, P, P, P, P, P]),
        "gbp_resolve_fragile_states_host": (I, [P, I64, P, P, I, P, P, P, P]),
        "gbp_extend_resolve_host": (I, [P, I64, P, P, P, I, I, U64, I64, P, P, P, P, P, P, P]),
        "gbp_stream_create": (I, [I, P]),
        "gbp_stream_destroy": (I, [P]),
        "gbp_tree_create": (I, [I, I64, P]),
        "gbp_tree_destroy": (I, [P]),
        "gbp_tree_init": (I, [P, P, P]),
        "gbp_tree_reserve": (I, [P, I64, P]),
        "gbp_tree_capacity": (I, [P, P]),
        "gbp_tree_size": (I, [P, P, P]),
        "gbp_tree_read": (I, [P, I64, I64, P, P, P, P, P]),
        "gbp_tree_append_host": (I, [P, I64, P, P, P, P]),
        "gbp_tree_load_host": (I, [P, I64, P, P, P, P]),
        "gbp_vertex_map_order": (I, [I64, P]),
        "gbp_vertex_map_rank": (I, [I64, I64, P]),
        "gbp_tree_device_ptrs": (I, [P, P, P]),
        "gbp_plan_ws_create": (I, [P, I64, P]),
        "gbp_plan_ws_destroy": (I, [P]),
        "gbp_plan_reset": (I, [P, I64, P]),
        "gbp_plan_half_dev": (I, [P, P, P, P, ctypes.c_int32, I, I64, U64, U64, I64, I, I, P]),
        "gbp_plan_halves_dev": (I, [P, P, P, P, ctypes.c_int32, ctypes.c_int32, I64, U64, U64, U64,
                                    I, I, P]),
        "gbp_plan_status_read": (I, [P, P, P]),
        "gbp_plan_star_config": (I, [P, I, ctypes.c_double, I64, I64]),
        "gbp_plan_stage_timing": (I, [P, I]),
        "gbp_plan_stage_times": (I, [P, P, I, P, I]),
        "gbp_plan_resolve_host": (I, [P, P, P, P, I, I64, I, P, P, P]),
        "gbp_extend_tree_dev": (I, [P, P, P, I64, P, P, I, I, U64, I64, P, P, P]),
        "gbp_extend_tree_finish_dev": (I, [P, P, P, I64, I, P, P, P]),
        "gbp_extend_tree_host": (I, [P, P, P, I64, P, I, I, U64, I64, P, P, P]),
        "gbp_tree_nearest_dev": (I, [P, P, I64, P, P, P]),
        "gbp_nearest_batch_dev": (I, [I64, P, I64, P, P, P, P]),
        "gbp_nearest_batch_host": (I, [I64, P, I64, P, P, P]),
        "gbp_neighbors_batch_dev": (I, [I64, P, I64, P, ctypes.c_double, I, P, P, P]),
        "gbp_neighbors_batch_host": (I, [I64, P, I64, P, ctypes.c_double, I, P, P]),
        "gbp_knn_batch_dev": (I, [I64, P, I64, P, I, P, P, P]),
        "gbp_knn_batch_host": (I, [I64, P, I64, P, I, P, P]),
        "gbp_knn_yaw_batch_dev": (I, [I64, P, P, I64, P, P, ctypes.c_double, ctypes.c_double, I, P,
                                      P, P]),
        "gbp_knn_yaw_batch_host": (I, [I64, P, I64, P, ctypes.c_double, ctypes.c_double, I, P, P]),
        "gbp_host_yaw": (ctypes.c_double, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name, None)
        if f is None:
            if path is None:  # the product library must export the whole ABI
                raise AttributeError(f"{p}: missing symbol {name}")
            continue  # a diagnostic build of an older ABI (tools/lib_ab.py)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = L
    return L


def check(status, what=""):
    if status != OK:
        raise GbpError(status, what)
    return status
