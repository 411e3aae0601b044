"""Validate-kernel throughput when independent batches are issued on S streams
(S = 1 is bench.py's timed loop): quantifies the launch-tail idle time that
concurrent kernels can fill."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

B = 262144
data = td.synth_rough(1024)
T = gbp.Terrain.from_data(data, device=0)
s, a, d, _, _ = W.make_attempts(T, B, W.CONFIG_SEEDS[3])
VP = ctypes.c_void_p
for S in (1, 2, 3, 4, 2, 3, 4, 8):
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [T.validate_pairs(s, a, d) for _ in range(S)]
    torch.cuda.synchronize()
    ptrs = [[VP(t.data_ptr()) for t in (o.valid, o.s_new, o.t_new, o.flags, o.counts)] for o in outs]

    def launch(k):
        p = ptrs[k % S]
        rc = T.validate_pairs_raw(B, VP(s.data_ptr()), VP(a.data_ptr()), VP(d.data_ptr()), 0, 0,
                                  p[0], p[1], p[2], p[3], p[4], VP(streams[k % S].cuda_stream))
        assert rc == 0

    K = 200
    for k in range(2 * S):
        launch(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        launch(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"streams {S}: {K * B / dt / 1e9:.3f} G attempts/s  ({dt / K * 1e3:.4f} ms per batch)",
          flush=True)
