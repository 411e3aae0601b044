"""Is synth-rough-1024's headline pair ((1.0, 10.23) -> (19.42, 10.23))
blocked by its terrain?  (VERDICT r02 "measure time to first solution at 1024²".)

synth-rough-N upsamples the rough-terrain CSV x10 by nearest neighbour, so each
0.2-m CSV cell becomes a flat 10 x 10 block and every CSV height difference a
vertical step (0.02 m of bilinear ramp).  Part 1 (numpy) lists the steps the
straight line start -> goal must cross and how wide they run.  Part 2 (GPU)
searches the dynamics empirically: STANCE-valid states in a band in front of a
step, the engine's candidate actions (getRandomAction / getRandomActionDirection
on the local normal, planning_utils.cpp:379-515), forward pair checks
(isValidStateActionPair, planning_utils.cpp:713-753) — does any primitive land
past the step?  And the same backwards (isValidStateActionPairReverse from states
past the step, the goal tree's direction).  Hits are re-checked with the oracle.

    python tools/wall_check.py --seconds 20 --out profiles/r03_wall_check.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import global_body_planner_amd as gbp  # noqa: E402
from global_body_planner_amd import _lib as L  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402


def steps_along_x(data, y0=10.23, x_lo=1.0, x_hi=19.42, min_jump=0.3):
    """Height steps the line y = y0 crosses, and their extent over all y."""
    z, x = data.z, data.x
    iy = int(np.searchsorted(data.y, y0)) - 1
    out = []
    for ix in range(1, x.size):
        if not (x_lo <= x[ix] <= x_hi):
            continue
        j = z[ix, iy] - z[ix - 1, iy]
        if abs(j) >= min_jump:
            col = z[ix] - z[ix - 1]
            out.append({"x": round(float(x[ix - 1]), 3), "to_x": round(float(x[ix]), 3),
                        "jump_at_y0": round(float(j), 4),
                        "jump_min_over_y": round(float(col.min()), 4),
                        "jump_max_over_y": round(float(col.max()), 4),
                        "full_width": bool(np.all(np.sign(col) == np.sign(j)) and
                                           np.all(np.abs(col) >= min_jump))})
    return out


def band_states(T, n, x_lo, x_hi, y_lo, y_hi, g, dev):
    """Random states over a band: z = ground + U(0.125, 0.45) (randomState's
    height range), horizontal speed up to V_MAX, vertical speed +-3 m/s, pitch
    +-0.6 rad, pitch rate +-3 rad/s; kept if STANCE-valid."""
    s = torch.empty((n, 8), dtype=torch.float64, device=dev)
    s[:, 0].uniform_(x_lo, x_hi, generator=g)
    s[:, 1].uniform_(y_lo, y_hi, generator=g)
    h, _, _ = T.height(s[:, :2].contiguous())
    s[:, 2] = h + torch.empty(n, dtype=torch.float64, device=dev).uniform_(0.125, 0.45, generator=g)
    sp = torch.empty(n, dtype=torch.float64, device=dev).uniform_(0.0, 2.0, generator=g)
    hd = torch.empty(n, dtype=torch.float64, device=dev).uniform_(-0.6, 0.6, generator=g)
    s[:, 3] = sp * torch.cos(hd)
    s[:, 4] = sp * torch.sin(hd)
    s[:, 5].uniform_(-3.0, 3.0, generator=g)
    s[:, 6].uniform_(-0.6, 0.6, generator=g)
    s[:, 7].uniform_(-3.0, 3.0, generator=g)
    v, _, _ = T.valid_states(s, L.STANCE)
    return s[v.bool()].contiguous()


def search(T, O, dev, direction, band, cross, seconds, batch, seed):
    """Attempts from band states; a hit = a valid pair whose s_new lies past
    `cross` (forward: x >= cross; reverse: x <= cross)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    t0, tried, hits, examples, launches = time.perf_counter(), 0, 0, [], 0
    cfg_dir = L.sampling(action_flag=True, action_p=0.5)
    while time.perf_counter() - t0 < seconds:
        s = band_states(T, batch, *band, g, dev)
        n = s.shape[0]
        if n == 0:
            continue
        # the normal at a target ahead of / behind the state, as newConfig draws it (rrt.cpp:25)
        tgt = s[:, :2].clone()
        tgt[:, 0] += 1.0 if direction == L.FORWARD else -1.0
        nrm, _ = T.normal(tgt.contiguous())
        nrm = torch.nan_to_num(nrm, nan=0.0)
        nrm[:, 2] = torch.where(nrm.abs().sum(1) == 0, torch.ones_like(nrm[:, 2]), nrm[:, 2])
        # half plain getRandomAction, half direction-biased toward a state past the wall
        far = s.clone()
        far[:, 3] += 1.0 if direction == L.FORWARD else -1.0
        a = T.sample_actions_dir(nrm, far, s, direction, seed, 7 + launches, 0, cfg=cfg_dir)
        res = T.validate_pairs(s, a, direction)
        ok = res.valid.bool()
        x_new = res.s_new[:, 0]
        past = ok & ((x_new >= cross) if direction == L.FORWARD else (x_new <= cross))
        k = int(past.sum().item())
        tried += n
        hits += k
        launches += 1
        if k and len(examples) < 8:
            idx = torch.nonzero(past).flatten()[:8 - len(examples)].cpu().numpy()
            for i in idx:
                examples.append({"s": s[i].cpu().numpy().tolist(), "a": a[i].cpu().numpy().tolist(),
                                 "s_new": res.s_new[i].cpu().numpy().tolist()})
    # the oracle re-decides the examples (bit-exact on the reference algorithm)
    for e in examples:
        v, sn, tn, f, c = O.validate_pairs(np.array([e["s"]]), np.array([e["a"]]),
                                           np.array([direction], np.uint8))
        e["oracle_valid"] = int(v[0])
        e["oracle_s_new_x"] = float(sn[0][0])
    dt = time.perf_counter() - t0
    return {"direction": "forward" if direction == L.FORWARD else "reverse",
            "band": [round(b, 3) for b in band], "cross": cross, "attempts": tried, "hits": hits,
            "seconds": round(dt, 1), "attempts_per_s": round(tried / dt, 1), "examples": examples}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seconds", type=float, default=20.0, help="per search")
    p.add_argument("--batch", type=int, default=1 << 21)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    data = td.synth_rough(1024)
    out = {"terrain": "synth-rough-1024", "line": "y = 10.23, x 1.0 -> 19.42",
           "steps": steps_along_x(data)}
    if torch.cuda.is_available():
        import oracle
        dev = torch.device("cuda", 0)
        T = gbp.Terrain.from_data(data, device=0)
        O = oracle.OracleTerrain.from_data(data)
        oracle.set_scan_mode(1)
        out["searches"] = [
            # the 0.55-m step up at x = 6.98 -> 7.0: start tree forward, onto the plateau
            search(T, O, dev, L.FORWARD, (6.30, 6.96, 0.5, 19.9), 7.17, a.seconds, a.batch, 1),
            # the goal tree backward across it: from the plateau to the low side
            search(T, O, dev, L.REVERSE, (7.02, 7.70, 0.5, 19.9), 6.83, a.seconds, a.batch, 2),
            # the 0.65-m step down at x = 11.18 -> 11.2: forward off the plateau
            search(T, O, dev, L.FORWARD, (10.50, 11.16, 0.5, 19.9), 11.37, a.seconds, a.batch, 3),
            # the goal tree backward up onto the plateau
            search(T, O, dev, L.REVERSE, (11.22, 11.90, 0.5, 19.9), 11.03, a.seconds, a.batch, 4),
        ]
    line = json.dumps(out, indent=1)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
