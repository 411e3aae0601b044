"""Generate tests/golden/oracle_vectors.npz from the CPU restatement.

The reference's own tests pin nothing (test/test_global_body_planner.cpp
asserts 1+1==2) and the reference cannot be built here, so these vectors
freeze the oracle's outputs (glibc 2.35 libm, -ffp-contract=off) so that any
later change to the restatement or the engine that moves a decision, a flag,
a lookup count or a bit of s_new / t_new is caught.  Inputs are small
(tens of thousands of cases); every array is plain data (np.savez, no pickle).

    python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from global_body_planner_amd import terrain_data as td  # noqa: E402
from tests.helpers import attempts_oracle  # noqa: E402

TERRAINS = ["slope-gridmap", "rough_terrain-gridmap", "synth-rough-256"]


def main(out=os.path.join(ROOT, "tests", "golden", "oracle_vectors.npz")):
    oracle.set_scan_mode(0)
    arrays = {}
    for ti, name in enumerate(TERRAINS):
        data = td.by_name(name)
        O = oracle.OracleTerrain.from_data(data)
        rng = np.random.default_rng(100 + ti)
        x0, xN, y0, yN = data.bounds
        n = 2000
        xy = np.stack([rng.uniform(x0 - 0.2, xN + 0.2, n), rng.uniform(y0 - 0.2, yN + 0.2, n)], 1)
        xy = np.concatenate([xy, np.stack([data.x[1:-1], np.full(data.x.size - 2, data.y[3])], 1),
                             np.array([[xN, y0], [x0, yN], [np.nan, y0], [x0 - 1, y0]])])
        h, isn, ood = O.height_batch(xy)
        nrm, nood = O.normal_batch(xy)
        p = f"{name}/"
        arrays.update({p + "xy": xy, p + "h": h, p + "is_nan": isn, p + "ood": ood,
                       p + "normal": nrm, p + "normal_ood": nood})
        st, _ = O.sample_states(3000, 77, 5, 0)
        for ph in (0, 1):
            v, f, c = O.valid_states(st, ph)
            arrays.update({p + f"states": st, p + f"state_valid_{ph}": v, p + f"state_flags_{ph}": f,
                           p + f"state_counts_{ph}": c})
        s, a, d, tgt, _ = attempts_oracle(O, 3000, seed=500 + ti, nthreads=8)
        arrays.update({p + "pair_s": s, p + "pair_a": a, p + "pair_dir": d})
        for ad in (0, 1):
            v, sn, tn, f, c = O.validate_pairs(s, a, d, adaptive=bool(ad), nthreads=8)
            arrays.update({p + f"pair_valid_{ad}": v, p + f"pair_s_new_{ad}": sn,
                           p + f"pair_t_new_{ad}": tn, p + f"pair_flags_{ad}": f,
                           p + f"pair_counts_{ad}": c})
        # extend with explicit candidates: the oracle's own sampler at the target normal
        m = 1000
        nrm_t, _ = O.normal_batch(tgt[:m, :2])
        cand = oracle.sample_actions(np.repeat(nrm_t, 6, axis=0), 41, 0x45585444, 0).reshape(m, 6, 10)
        r, ch, sn, an, c = O.extend_batch(s[:m], tgt[:m], cand, d[:m])
        arrays.update({p + "ext_s_near": s[:m], p + "ext_target": tgt[:m], p + "ext_cand": cand,
                       p + "ext_dir": d[:m], p + "ext_result": r, p + "ext_chosen": ch,
                       p + "ext_s_new": sn, p + "ext_a_new": an, p + "ext_counts": c})
    # the planner loop (orc_plan): batch 8, synth-256's config-2 pair, 400 halves
    from global_body_planner_amd import planner
    data = td.by_name("synth-rough-256")
    O = oracle.OracleTerrain.from_data(data)
    oracle.set_scan_mode(1)
    hs, _ = O.ground_height(1.0, 2.55)
    hg, _ = O.ground_height(4.02, 2.55)
    start, goal = planner.start_goal_state(hs, 1.0, 2.55), planner.start_goal_state(hg, 4.02, 2.55)
    r = O.plan(start, goal, batch=8, seed=5, max_halves=400)
    arrays["loop/start"], arrays["loop/goal"] = start, goal
    arrays["loop/counters"] = np.array([r[k] for k in ("found", "meet_a", "meet_b", "halves",
                                                        "targets", "attempts", "connects")])
    for t in "ab":
        for k in ("v", "act", "parent", "g", "y"):
            arrays[f"loop/{t}_{k}"] = r[t][k]
    oracle.set_scan_mode(0)
    rng = np.random.default_rng(9)
    verts = rng.normal(size=(3000, 8))
    verts[11] = verts[5]
    q = np.concatenate([rng.normal(size=(500, 8)), verts[[5, 11]]])
    idx, dist = oracle.nearest_batch(q, verts)
    arrays.update({"nn/verts": verts, "nn/q": q, "nn/idx": idx, "nn/dist": dist})
    os.makedirs(os.path.dirname(out), exist_ok=True)
    np.savez_compressed(out, **arrays)
    print(f"wrote {out} ({os.path.getsize(out) / 1e6:.2f} MB, {len(arrays)} arrays)")


if __name__ == "__main__":
    main()
