"""Offline: how much of the planner's O(queries x vertices) nearest-neighbour
scan could an exact bounding-box pruning skip?  

Input: tools/tree_dump.py's trees (the device loop's real trees at several
sizes) and planner-distributed queries.  For a row order (insertion = what the
kernel scans today; Morton orders over a few coordinates) and a chunk size,
every chunk gets its 8-D bounding box; a query can skip a chunk when the box's
lower bound exceeds the query's nearest distance (the best any exact pruning
with a perfect upper bound can do).  On the GPU a wave decides per chunk for
its whole query tile, so the tile-level fraction (tiles of queries sorted the
same way, box-to-box bounds) is the realistic one.

    python tools/nn_prune_eval.py gpurun_out/trees.npz
"""
import argparse
import json
import sys

import numpy as np


def nn_dist(q, v, block=2048):
    best = np.full(q.shape[0], np.inf)
    vn = (v * v).sum(1)
    for i in range(0, v.shape[0], block):
        vb = v[i:i + block]
        d2 = (q * q).sum(1)[:, None] + vn[None, i:i + block] - 2 * q @ vb.T
        best = np.minimum(best, d2.min(1))
    return np.sqrt(np.maximum(best, 0))


def morton_key(x, dims, bits=10):
    """Interleaved-bit key over the chosen columns (each scaled to [0, 2^bits))."""
    cols = []
    for d in dims:
        c = x[:, d]
        lo, hi = c.min(), c.max()
        cols.append(np.clip(((c - lo) / max(hi - lo, 1e-12) * (2 ** bits - 1)).astype(np.int64), 0,
                            2 ** bits - 1))
    key = np.zeros(x.shape[0], dtype=np.int64)
    for b in range(bits):
        for j, c in enumerate(cols):
            key |= ((c >> b) & 1) << (b * len(cols) + j)
    return key


def box_lb(q, lo, hi):
    """Lower bound of the distance from each query to each box: [nq, nb]."""
    d = np.maximum(0, np.maximum(lo[None] - q[:, None], q[:, None] - hi[None]))
    return np.sqrt((d * d).sum(2))


def boxbox_lb(qlo, qhi, lo, hi):
    d = np.maximum(0, np.maximum(lo[None] - qhi[:, None], qlo[:, None] - hi[None]))
    return np.sqrt((d * d).sum(2))


def evaluate(v, q, dstar, order, chunk, qtile):
    n = v.shape[0]
    if order == "insertion":
        perm = np.arange(n)
        qperm = np.arange(q.shape[0])
    else:
        dims = {"xy": [0, 1], "xyv": [0, 1, 3, 4], "all": list(range(8)),
                "xyz-v": [0, 1, 2, 3, 4, 5]}[order]
        allpts = np.concatenate([v, q])
        key = morton_key(allpts, dims, bits=max(2, 30 // len(dims)))
        perm = np.argsort(key[:n], kind="stable")
        qperm = np.argsort(key[n:], kind="stable")
    vs = v[perm]
    nc = (n + chunk - 1) // chunk
    lo = np.stack([vs[c * chunk:(c + 1) * chunk].min(0) for c in range(nc)])
    hi = np.stack([vs[c * chunk:(c + 1) * chunk].max(0) for c in range(nc)])
    lb = box_lb(q, lo, hi)
    ideal = float((lb <= dstar[:, None]).mean())
    qs, ds = q[qperm], dstar[qperm]
    nt = (q.shape[0] + qtile - 1) // qtile
    tl = np.stack([qs[t * qtile:(t + 1) * qtile].min(0) for t in range(nt)])
    th = np.stack([qs[t * qtile:(t + 1) * qtile].max(0) for t in range(nt)])
    tmax = np.array([ds[t * qtile:(t + 1) * qtile].max() for t in range(nt)])
    blb = boxbox_lb(tl, th, lo, hi)
    tile = float((blb <= tmax[:, None]).mean())
    return {"order": order, "chunk": chunk, "qtile": qtile, "ideal_fraction": round(ideal, 4),
            "tile_fraction": round(tile, 4)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("npz")
    p.add_argument("--nq", type=int, default=6000)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    f = np.load(a.npz)
    q = f["queries"][:a.nq]
    res = []
    for key in sorted(k for k in f.files if k.startswith("a_")):
        size = key[2:]
        for tree in ("a", "b"):
            v = f[f"{tree}_{size}"]
            dstar = nn_dist(q, v)
            row = {"tree": tree, "snapshot": int(size), "vertices": int(v.shape[0]),
                   "median_nn_dist": round(float(np.median(dstar)), 3), "evals": []}
            for order in ("insertion", "xy", "xyv", "all"):
                for chunk in (64, 256):
                    row["evals"].append(evaluate(v, q, dstar, order, chunk, 128))
            res.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(res, fo, indent=1)


if __name__ == "__main__":
    sys.exit(main())
