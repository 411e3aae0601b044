"""Parity soak (test infrastructure, run on the GPU box): many full-size
batches of the bench configuration (persistent kernel, default options) on
every terrain, each compared bit for bit with the CPU oracle (oracle/, the
checker only) by tests/helpers.assert_pairs_equal, both directions, plain and
adaptive loops.  Prints one line per batch and a total; exits 1 on the first
mismatch."""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import global_body_planner_amd as gbp  # noqa: E402
import oracle  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from global_body_planner_amd import workload as W  # noqa: E402
from tests.helpers import assert_pairs_equal, resolver, u32  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--terrains", default="synth-rough-1024,synth-rough-256,slope-gridmap,"
                                         "rough_terrain-gridmap,rough_terrain-direct")
    p.add_argument("--seeds", type=int, default=4)
    p.add_argument("--batch", type=int, default=262144)
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--waves", type=int, default=2,
                   help="GBP_OPT_WAVES of the launches (3: bench.py's headline launch)")
    a = p.parse_args()
    oracle.set_scan_mode(1)  # bisection brackets: equal to the linear scan, faster
    total = frag_total = valid_total = 0
    t0 = time.time()
    for name in a.terrains.split(","):
        data = td.by_name(name)
        T = gbp.Terrain.from_data(data, device=0)
        O = oracle.OracleTerrain.from_data(data)
        T.set_option(L.OPT_KERNEL, L.KERNEL_PERSISTENT)
        T.set_option(L.OPT_WAVES, a.waves)
        print(f"{name}: waves {a.waves}, coordinate mode {T.get_option(L.OPT_COORD_MODE)}", flush=True)
        for k in range(a.seeds):
            seed = 7919 * (k + 1) + len(name)
            s, act, d, _, tries = W.make_attempts(T, a.batch, seed)
            keep = (tries >= 0).cpu().numpy()
            for adaptive in (False, True):
                r = T.validate_pairs(s, act, d, adaptive=adaptive)
                torch.cuda.synchronize()
                gpu_t = tuple(np.asarray(x)[keep] for x in
                              (r.valid.cpu().numpy(), r.s_new.cpu().numpy(), r.t_new.cpu().numpy(),
                               u32(r.flags), u32(r.counts)))
                ref = O.validate_pairs(s.cpu().numpy(), act.cpu().numpy(), d.cpu().numpy(),
                                       adaptive=adaptive, nthreads=a.threads)
                ref = tuple(np.asarray(x)[keep] for x in ref)
                label = f"{name} seed {seed} adaptive {int(adaptive)}"
                try:
                    sk, ak, dk = (x.cpu().numpy()[keep] for x in (s, act, d))
                    nfrag = assert_pairs_equal(gpu_t, ref, label,
                                               resolve=resolver(T, sk, ak, dk, adaptive))
                except AssertionError as e:
                    print(f"MISMATCH {e}", flush=True)
                    sys.exit(1)
                m = int(keep.sum())
                nv = int(ref[0].sum())
                total += m
                frag_total += nfrag
                valid_total += nv
                print(f"{label}: {m} attempts bit-exact, {nv} valid, {nfrag} fragile "
                      f"(re-decided on the host, then compared) [{time.time() - t0:.0f} s]", flush=True)
    print(f"TOTAL {total} attempts bit-exact vs oracle, {valid_total} valid, {frag_total} fragile",
          flush=True)


if __name__ == "__main__":
    main()
