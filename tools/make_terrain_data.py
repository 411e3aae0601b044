"""Convert the reference's terrain CSV data files into one compact .npz.

Run in the build container (the only place /root/reference exists):
    python tools/make_terrain_data.py /root/reference/data global_body_planner_amd/data/terrain_csv.npz

The CSV files are data (x/y/z/dx/dy/dz grids, 31 rows = y, 51/56 columns = x;
reference data/{slope,rough_terrain}/*.csv, read by
terrain_map_publisher.cpp:290-370).  Values are parsed with float() exactly
like std::stod in the reference's loadCSV (:290-328); they are stored as
float64 so nothing is rounded here.
"""
import os
import sys

import numpy as np


def load_csv(path):
    rows = []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line or line.startswith("#"):
                continue
            rows.append([float(v) for v in line.split(",")])
    return np.array(rows, dtype=np.float64)


def main(src, dst):
    out = {}
    for terrain in ("slope", "rough_terrain"):
        for layer in ("x", "y", "z", "dx", "dy", "dz"):
            out[f"{terrain}/{layer}"] = load_csv(os.path.join(src, terrain, f"{layer}data.csv"))
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    np.savez_compressed(dst, **out)
    print(f"wrote {dst}: " + ", ".join(f"{k}{v.shape}" for k, v in out.items()))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
