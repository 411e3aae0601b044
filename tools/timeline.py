"""Per-wave timeline of one persistent validate launch (diagnostic build
lib/diag/libgbp_util.so, -DGBP_DIAG_UTIL): start skew, end spread, steps and
lifetime per wave, at config 3's batch."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
data = td.synth_rough(1024)
ulib = L.load(os.path.join(ROOT, "global_body_planner_amd", "lib", "diag", "libgbp_util.so"))
ulib.gbp_diag_waves.argtypes = [ctypes.c_void_p, ctypes.c_int]
T = gbp.Terrain.from_data(data, device=0, lib=ulib)
if len(sys.argv) > 2:  # sched[:chunk[:prefix]]
    parts = [int(v) for v in sys.argv[2].split(":")]
    T.set_option(L.OPT_SCHED, parts[0])
    if len(parts) > 1:
        T.set_option(L.OPT_CHUNK, parts[1])
    if len(parts) > 2:
        T.set_option(L.OPT_PREFIX, parts[2])
s, a, d, _, _ = W.make_attempts(T, B, W.CONFIG_SEEDS[3])
for _ in range(3):
    T.validate_pairs(s, a, d)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
T.validate_pairs(s, a, d)
ev1.record()
torch.cuda.synchronize()
print(f"kernel {ev0.elapsed_time(ev1):.4f} ms (this launch is the one recorded below)")
nw = 2048
buf = (ctypes.c_ulonglong * (4 * nw))()
ulib.gbp_diag_waves(buf, nw)
w = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 4).astype(np.int64)
t0 = w[:, 0].min()
beg, end, steps, cu = (w[:, 0] - t0) / 100.0, (w[:, 1] - t0) / 100.0, w[:, 2], w[:, 3]
life = end - beg
q = [0, 10, 50, 90, 100]
print(f"B={B} waves={nw}  (times in us from the first wave's start, 100 MHz clock)")
print("begin pct", np.percentile(beg, q).round(2))
print("end   pct", np.percentile(end, q).round(2))
print("life  pct", np.percentile(life, q).round(2))
print("steps pct", np.percentile(steps, q))
print("us/step pct", np.percentile(life / np.maximum(steps, 1), q).round(3))
# end time vs steps correlation, and per-CU
print("corr(end, steps) %.3f" % np.corrcoef(end, steps)[0, 1])
order = np.argsort(end)[-10:]
print("slowest waves (begin, end, steps, cu):")
for i in order:
    print(f"  wave {i:5d} begin {beg[i]:8.2f} end {end[i]:8.2f} steps {steps[i]:4d} cu {cu[i]}")
wg = np.arange(nw) // 4
xcd = wg % 8
print("per XCD (wg % 8): mean end / mean us-per-step")
for x in range(8):
    m = xcd == x
    print(f"  xcd {x}: end {end[m].mean():8.2f}  step {np.mean(life[m] / steps[m]):7.3f}  max end {end[m].max():8.2f}")
print("per wave-in-WG (wid % 4):")
for k in range(4):
    m = (np.arange(nw) % 4) == k
    print(f"  k {k}: end {end[m].mean():8.2f}")
print("per WG half (first 256 WGs vs last 256):")
for h in range(2):
    m = (wg >= 256 * h) & (wg < 256 * (h + 1))
    print(f"  half {h}: end {end[m].mean():8.2f}")
