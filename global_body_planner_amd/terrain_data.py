"""Terrain inputs: the reference CSV maps and the synthetic benchmark maps.

Host-side ingest only (no compute): produces x-major FastTerrainMap arrays
(x[nx], y[ny], z[nx][ny], dx/dy/dz[nx][ny]) exactly as the reference's
FastTerrainMap would hold them (fast_terrain_map.h:97-118).

* ``csv_gridmap(name)`` — the reference's CSV → grid_map → FastTerrainMap path:
  TerrainMapPublisher::loadMapFromCSV (terrain_map_publisher.cpp:330-370) builds
  a grid_map with a FLOAT resolution (:345-346) and float layers, and
  FastTerrainMap::loadDataFromGridMap (fast_terrain_map.cpp:31-91) reads the
  cell-centre positions back in reversed index order and casts float→double.
  grid_map_core (ros-melodic-grid-map, unpinned, not in the image) is restated
  from its published GridMapMath arithmetic: setGeometry rounds
  length/resolution to a cell count and keeps length = size*resolution;
  getPosition(index) = position + (0.5*length - 0.5*resolution) - resolution*index.
  This emulation is unverified against a real grid_map build.
* ``synth_rough(N)`` — SURVEY §8(d) synth-rough-N: z[ix][iy] =
  (double)(float) Zcsv[(iy/10) % 31][(ix/10) % 56] (dx/dy/dz alike), x[i] = i*0.02.
* ``synth_fractal(N)`` — SURVEY §8(d) synth-fractal-4096 (config 5):
  diamond-square, roughness H, amplitude A, float-rounded; normals from
  central differences.
"""
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "terrain_csv.npz")


@dataclass
class TerrainData:
    x: np.ndarray                  # [nx] ascending
    y: np.ndarray                  # [ny] ascending
    z: np.ndarray                  # [nx][ny] x-major
    dx: Optional[np.ndarray] = None
    dy: Optional[np.ndarray] = None
    dz: Optional[np.ndarray] = None
    name: str = ""

    @property
    def shape(self):
        return self.z.shape

    @property
    def bounds(self):
        return float(self.x[0]), float(self.x[-1]), float(self.y[0]), float(self.y[-1])


def _csv(name):
    with np.load(_DATA) as f:
        return {k.split("/", 1)[1]: f[k] for k in f.files if k.startswith(name + "/")}


def csv_raw(name):
    """Raw CSV grids (rows = y, columns = x) of data/<name>/*.csv."""
    return _csv(name)


def csv_gridmap(name):
    """FastTerrainMap arrays after the CSV → grid_map → loadDataFromGridMap path."""
    d = _csv(name)
    xd, yd = d["x"], d["y"]
    x_size = d["z"].shape[1]          # terrain_map_publisher.cpp:341  z_data[0].size()
    y_size = d["z"].shape[0]          # :342  z_data.size()
    f32 = np.float32
    x_res = float(f32(xd[0][1] - xd[0][0]))          # :343 float
    y_res = float(f32(yd[1][0] - yd[0][0]))          # :344 float
    x_length = xd[0][-1] - xd[0][0] + x_res          # :345
    y_length = yd[-1][0] - yd[0][0] + y_res          # :346
    if x_res != y_res:
        raise RuntimeError("Map did not have square elements")
    pos = (xd[0][0] - 0.5 * x_res + 0.5 * x_length,  # :354-356
           yd[0][0] - 0.5 * y_res + 0.5 * y_length)
    res = x_res
    size = (int(np.round(x_length / res)), int(np.round(y_length / res)))  # GridMap::setGeometry
    length = (size[0] * res, size[1] * res)
    assert size == (x_size, y_size), (size, x_size, y_size)

    def position(axis, index):        # GridMapMath getPositionFromIndex (buffer start 0)
        off = 0.5 * length[axis] - 0.5 * res
        return (pos[axis] + off) + res * float(-index)

    x = np.array([position(0, (x_size - 1) - i) for i in range(x_size)])   # fast_terrain_map.cpp:43-48
    y = np.array([position(1, (y_size - 1) - i) for i in range(y_size)])   # :49-54

    def layer(grid):
        # at(index={(x_size-1)-i,(y_size-1)-j}) == grid[j][i] (publisher :363-368), float storage
        return np.ascontiguousarray(grid.T.astype(np.float32).astype(np.float64))

    return TerrainData(x, y, layer(d["z"]), layer(d["dx"]), layer(d["dy"]), layer(d["dz"]),
                       name=f"{name}-gridmap")


def csv_direct(name):
    """FastTerrainMap::loadData straight from the CSV doubles (no grid_map, no float cast)."""
    d = _csv(name)
    x = np.ascontiguousarray(d["x"][0])
    y = np.ascontiguousarray(d["y"][:, 0])
    t = lambda g: np.ascontiguousarray(g.T)
    return TerrainData(x, y, t(d["z"]), t(d["dx"]), t(d["dy"]), t(d["dz"]), name=f"{name}-direct")


def synth_rough(n, spacing=0.02):
    """SURVEY §8(d) synth-rough-N (N = 256, 1024, ...)."""
    d = _csv("rough_terrain")
    ix = np.arange(n)
    iy = np.arange(n)
    rows = (iy // 10) % d["z"].shape[0]
    cols = (ix // 10) % d["z"].shape[1]

    def layer(g):
        return np.ascontiguousarray(g[np.ix_(rows, cols)].T.astype(np.float32).astype(np.float64))

    x = np.arange(n, dtype=np.float64) * spacing
    y = np.arange(n, dtype=np.float64) * spacing
    return TerrainData(x, y, layer(d["z"]), layer(d["dx"]), layer(d["dy"]), layer(d["dz"]),
                       name=f"synth-rough-{n}")


def synth_fractal(n, seed=4096, hurst=0.8, amplitude=0.6, spacing=0.02):
    """SURVEY §8(d) synth-fractal-N: diamond-square height field (float-rounded)."""
    size = 1
    while size + 1 < n:
        size *= 2
    m = size + 1
    rng = np.random.default_rng(seed)
    h = np.zeros((m, m))
    h[0, 0], h[0, -1], h[-1, 0], h[-1, -1] = rng.uniform(-1, 1, 4)
    step, scale = size, 1.0
    while step > 1:
        half = step // 2
        # diamond
        c = (h[0:-1:step, 0:-1:step] + h[step::step, 0:-1:step] + h[0:-1:step, step::step] +
             h[step::step, step::step]) * 0.25
        h[half::step, half::step] = c + rng.uniform(-scale, scale, c.shape)
        # square
        for (ox, oy) in ((half, 0), (0, half)):
            xs = np.arange(ox, m, step)
            ys = np.arange(oy, m, step)
            X, Y = np.meshgrid(xs, ys, indexing="ij")
            acc = np.zeros(X.shape)
            cnt = np.zeros(X.shape)
            for dx_, dy_ in ((-half, 0), (half, 0), (0, -half), (0, half)):
                XX, YY = X + dx_, Y + dy_
                ok = (XX >= 0) & (XX < m) & (YY >= 0) & (YY < m)
                acc[ok] += h[XX[ok], YY[ok]]
                cnt[ok] += 1
            h[X, Y] = acc / cnt + rng.uniform(-scale, scale, X.shape)
        step = half
        scale *= 0.5 ** hurst
    h = h[:n, :n]
    h = (h - h.min()) / max(h.max() - h.min(), 1e-12) * amplitude
    z = h.astype(np.float32).astype(np.float64)
    gx = np.gradient(z, spacing, axis=0)
    gy = np.gradient(z, spacing, axis=1)
    nrm = np.stack([-gx, -gy, np.ones_like(z)])
    nrm /= np.linalg.norm(nrm, axis=0)
    f = lambda a: np.ascontiguousarray(a.astype(np.float32).astype(np.float64))
    x = np.arange(n, dtype=np.float64) * spacing
    return TerrainData(x, x.copy(), np.ascontiguousarray(z), f(nrm[0]), f(nrm[1]), f(nrm[2]),
                       name=f"synth-fractal-{n}")


def by_name(name):
    if name.startswith("synth-rough-"):
        return synth_rough(int(name.rsplit("-", 1)[1]))
    if name.startswith("synth-fractal-"):
        return synth_fractal(int(name.rsplit("-", 1)[1]))
    if name.endswith("-gridmap"):
        return csv_gridmap(name[: -len("-gridmap")])
    if name.endswith("-direct"):
        return csv_direct(name[: -len("-direct")])
    raise KeyError(name)
