"""Lane utilisation of the persistent validate kernel (diagnostic build
lib/diag/libgbp_util.so, -DGBP_DIAG_UTIL) and attempts/s vs batch size.

Prints per batch: wave-steps, mean active lanes per step (of 64), mean / max
wave lifetime (wall_clock64 ticks, 100 MHz) vs kernel time."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

data = td.synth_rough(1024)
ulib = L.load(os.path.join(ROOT, "global_body_planner_amd", "lib", "diag", "libgbp_util.so"))
ulib.gbp_diag_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
Tu = gbp.Terrain.from_data(data, device=0, lib=ulib)
Tr = gbp.Terrain.from_data(data, device=0)
waves = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for T in (Tu, Tr):
    T.set_option(L.OPT_WAVES, waves)
buf = (ctypes.c_ulonglong * 4)()
for B in (65536, 262144, 1048576, 4194304):
    s, a, d, _, _ = W.make_attempts(Tr, B, W.CONFIG_SEEDS[3])
    Tu.validate_pairs(s, a, d)
    torch.cuda.synchronize()
    ulib.gbp_diag_read(buf, 1)
    Tu.validate_pairs(s, a, d)
    torch.cuda.synchronize()
    ulib.gbp_diag_read(buf, 1)
    steps, active, life, lmax = list(buf)
    res = {}
    for hp in (1, 0):
        Tr.set_option(L.OPT_HELPERS, hp)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(2):
            Tr.validate_pairs(s, a, d)
        ev0.record()
        for _ in range(5):
            Tr.validate_pairs(s, a, d)
        ev1.record()
        torch.cuda.synchronize()
        res[hp] = ev0.elapsed_time(ev1) / 5
    Tr.set_option(L.OPT_HELPERS, 1)
    ms = res[1]
    nw = 256 * 4 * waves
    print(f"B={B:8d} kernel {ms:8.3f} ms  {B / ms / 1e3:8.1f} M att/s (no helpers "
          f"{B / res[0] / 1e3:8.1f}) | wave-steps {steps:9d} "
          f"active/step {active / max(steps, 1):5.1f}/64  steps/wave {steps / nw:7.1f}  "
          f"life mean {life / nw / 100:8.1f} us max {lmax / 100:8.1f} us", flush=True)
