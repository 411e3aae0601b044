"""MI355X-native batched RRT-Connect extend/validity engine for global_body_planner.

Product layers:
  include/gbp.h + csrc/ (libgbp.so)   HIP kernels for gfx950 behind a C ABI
  engine.py                           device-tensor API over the C ABI
  terrain_data.py                     reference CSV / synthetic terrain ingest
  planner.py                          host mirror of FastTerrainMap / planning_utils /
                                      PlannerClass / RRTConnectClass over the engine
No CPU fallback exists: without lib/libgbp.so every compute call raises.
"""
import torch  # noqa: F401  (load torch's HIP runtime first: one runtime per process)

from . import _lib
from ._lib import (ADVANCED, FLIGHT, FORWARD, REACHED, REVERSE, STANCE, TRAPPED, GbpError,
                   KERNEL_DIRECT, KERNEL_PERSISTENT)
from .terrain_data import TerrainData, csv_gridmap, csv_direct, synth_rough, synth_fractal
from .engine import (Terrain, PairResult, ExtendResult, DeviceTree, PlanWorkspace, nearest,
                     neighbors, knn, knn_yaw, device_count)

__all__ = [
    "ADVANCED", "FLIGHT", "FORWARD", "REACHED", "REVERSE", "STANCE", "TRAPPED", "GbpError",
    "KERNEL_DIRECT", "KERNEL_PERSISTENT", "TerrainData", "csv_gridmap", "csv_direct",
    "synth_rough", "synth_fractal", "Terrain", "PairResult", "ExtendResult", "DeviceTree",
    "PlanWorkspace", "nearest", "neighbors", "knn", "knn_yaw", "device_count",
]
__version__ = "0.2.0"
