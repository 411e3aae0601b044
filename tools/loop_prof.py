"""Where a persistent validate wave spends its cycles (diagnostic build):

    make -C global_body_planner_amd/csrc variant NAME=lp DEFS=-DGBP_LOOP_PROF
    python tools/loop_prof.py ab_libs/libgbp_lp.so

The -DGBP_LOOP_PROF build of k_validate_persistent reads the shader clock
(s_memtime) between the phases of each loop step and accumulates per wave:
refill, the helper plan, sample + isValidState, transition + the helpers'
consumption, outputs + s_new ring; plus the whole loop, tail steps and steps.
Config 3 (synth-rough-1024, 262,144 attempts) and config 2 (synth-rough-256,
65,536), one launch each after a warm-up launch.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402

PHASES = ["refill", "helper_plan", "sample_isvalid", "transition_consume", "outputs_ring"]


def run(lib, terrain, batch, seed, opts=(), waves=2048):
    data = td.by_name(terrain)
    T = gbp.Terrain.from_data(data, device=0, lib=lib)
    for kv in opts:
        k, v = kv.split("=")
        T.set_option(getattr(L, "OPT_" + k), int(v))
    s, act, d, _, _ = W.make_attempts(T, batch, seed)
    out = T.validate_pairs(s, act, d)
    T.validate_pairs(s, act, d, out=out)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (12 * waves))()
    rc = lib.gbp_loop_prof_read(buf, ctypes.c_int(waves))
    assert rc == 0, rc
    raw = np.frombuffer(buf, dtype=np.uint64).reshape(waves, 12)
    a = raw.astype(np.float64)
    keep = a[:, 7] > 0
    a, raw = a[keep], raw[keep]
    if os.environ.get("LOOP_PROF_DUMP"):
        np.save(os.environ["LOOP_PROF_DUMP"] + f"_{terrain}.npy", raw)
    steps = a[:, 7].sum()
    tot = a[:, 5].sum()
    row = {"terrain": terrain, "batch": batch, "waves": int(a.shape[0]),
           "steps_per_wave": float(a[:, 7].mean()), "tail_steps_per_wave": float(a[:, 6].mean()),
           "loop_cycles_per_wave": float(a[:, 5].mean()),
           "loop_cycles_per_wave_max": float(a[:, 5].max()),
           "cycles_per_step": float(tot / steps)}
    for k, nm in enumerate(PHASES):
        row[nm + "_frac"] = float(a[:, k].sum() / tot)
        row[nm + "_per_step"] = float(a[:, k].sum() / steps)
    # wall clock (s_memrealtime, 100 MHz): start skew, per-wave spans, the end
    t0, t1 = a[:, 8], a[:, 9]
    span = (t1 - t0) * 10.0  # ns
    row["start_skew_us"] = float((t0.max() - t0.min()) * 10.0 / 1e3)
    row["kernel_span_us"] = float((t1.max() - t0.min()) * 10.0 / 1e3)
    row["wave_span_us"] = {q: float(np.percentile(span, q) / 1e3) for q in (0, 10, 50, 90, 99, 100)}
    row["steps_quantiles"] = {q: float(np.percentile(a[:, 7], q)) for q in (0, 50, 90, 99, 100)}
    row["corr_span_steps"] = float(np.corrcoef(span, a[:, 7])[0, 1])
    # the slowest decile: its steps and its cycles per step against the rest
    slow = span >= np.percentile(span, 90)
    row["slow_decile"] = {"steps": float(a[slow, 7].mean()), "rest_steps": float(a[~slow, 7].mean()),
                          "cycles_per_step": float(a[slow, 5].sum() / a[slow, 7].sum()),
                          "rest_cycles_per_step": float(a[~slow, 5].sum() / a[~slow, 7].sum())}
    # per XCC and per CU: mean span (contention differences)
    xcc = raw[:, 11] & 0xF
    cu = (raw[:, 10] >> 8) & 0x1FF
    row["span_by_xcc_us"] = [float(span[xcc == x].mean() / 1e3) for x in range(8) if (xcc == x).any()]
    cus = {}
    for x, c, sp in zip(xcc, cu, span):
        cus.setdefault((int(x), int(c)), []).append(sp)
    cm = np.array([np.mean(v) for v in cus.values()]) / 1e3
    row["cu_mean_span_us"] = {"n": len(cus), "min": float(cm.min()), "median": float(np.median(cm)),
                              "max": float(cm.max())}
    return row


def main():
    p = argparse.ArgumentParser()
    p.add_argument("lib")
    p.add_argument("--set", action="append", default=[], help="OPT=value on the handle")
    a = p.parse_args()
    lib = L.load(a.lib)
    lib.gbp_loop_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    for terrain, batch, seed in (("synth-rough-1024", 262144, W.CONFIG_SEEDS[3]),
                                 ("synth-rough-256", 65536, W.CONFIG_SEEDS[2])):
        print(json.dumps(run(lib, terrain, batch, seed, a.set)), flush=True)


if __name__ == "__main__":
    main()
