// gbp_internal.h — definitions shared by the engine's translation units
// (gbp_engine.hip: terrain, lookups, pair checks, samplers, extend, NN;
// gbp_plan.hip: device trees and the device-resident planner loop).  Not
// part of the C ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "gbp.h"
#include "gbp_device.h"
#include "host/gbp_host_check.h"

constexpr uint64_t GBP_EXTEND_STREAM = 0x45585444ull;  // "EXTD": newConfig's candidate stream

struct gbp_terrain {
  gbp_host::Terrain host;           // host copy (the values the device holds) for the
                                    // glibc re-decision of FRAGILE attempts
  int device = 0;
  int nx = 0, ny = 0;
  int storage = GBP_STORAGE_F64;
  double bounds[4] = {0, 0, 0, 0};
  double xNm = 0, yNm = 0;          // x[nx-2], y[ny-2]
  double inv_hx = 0, inv_hy = 0;
  int one_x = 0, one_y = 0;         // one-step bracket correction is exact (verified)
  double *d_x = nullptr, *d_y = nullptr;
  void *d_z = nullptr;
  double *d_dx = nullptr, *d_dy = nullptr, *d_dz = nullptr;
  int num_cus = 256;
  int64_t opt_kernel = GBP_KERNEL_PERSISTENT;
  int64_t opt_block = 256;
  int64_t opt_waves = 2;            // register budget of the validate kernels (waves/SIMD)
  int64_t opt_lds_coords = 1;       // stage the coordinate vectors in LDS when they fit
  int64_t opt_helpers = 1;          // idle lanes of a drained wave evaluate owners' next samples
  int64_t opt_affine = 1;           // compute coordinates when the affine form is exact
  int64_t opt_fast_rcp = 1;         // cell-area reciprocal by verified Newton steps
  double rcp_seed = 0;              // verified_rcp_seed (0: every spacing pair not exact)
  double fragile_eps = gbp::FRAGILE_EPS;  // GBP_OPT_FRAGILE_EPS (>= the default)
  int64_t opt_xcd_map = 0;          // persistent kernel: slices numbered XCD-major
  int opt_nn_stats = 0;             // 1: the matrix-core NN search counts its fp64 re-checks
  gbp_sampling sampling{};          // direction-biased sampling (gbp_terrain_set_sampling), off
  int affine = 0;                   // host-verified affine coordinates (both axes)
  int bx = 0, by = 0;
  double ax = 0, hx = 0, ay = 0, hy = 0;
  size_t lds_max = 65536;           // LDS bytes a workgroup may use
  hipStream_t host_stream = nullptr;
  void *ws = nullptr;               // grow-only device workspace
  size_t ws_bytes = 0;
  // extend-candidate workspaces, one per stream: _dev calls on one handle may
  // run concurrently on different streams without sharing scratch
  struct StreamWs {
    hipStream_t stream;
    void *ptr;
    size_t bytes;
  };
  std::vector<StreamWs> cand_ws;
};

#define HIPCHK(expr)                      \
  do {                                    \
    hipError_t e_ = (expr);               \
    if (e_ != hipSuccess) return GBP_E_HIP; \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class ZT>
inline gbp::TerrainView<ZT> view(const gbp_terrain *t) {
  gbp::TerrainView<ZT> v;
  v.x = t->d_x;
  v.y = t->d_y;
  v.z = (const ZT *)t->d_z;
  v.dx = t->d_dx;
  v.dy = t->d_dy;
  v.dz = t->d_dz;
  v.nx = t->nx;
  v.ny = t->ny;
  v.x0 = t->bounds[0];
  v.xN = t->bounds[1];
  v.y0 = t->bounds[2];
  v.yN = t->bounds[3];
  v.xNm = t->xNm;
  v.yNm = t->yNm;
  v.inv_hx = t->inv_hx;
  v.inv_hy = t->inv_hy;
  v.one_x = t->one_x;
  v.one_y = t->one_y;
  v.affine = t->affine;
  v.bx = t->bx;
  v.by = t->by;
  v.ax = t->ax;
  v.hx = t->hx;
  v.ay = t->ay;
  v.hy = t->hy;
  v.rcp_seed = t->opt_fast_rcp ? t->rcp_seed : 0.0;
  v.feps = t->fragile_eps;
  return v;
}

inline unsigned grid_for(int64_t n, int block, int cap = 65535 * 8) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

inline int ensure_ws(void **ws, size_t *have, size_t need) {
  if (*have >= need) return GBP_OK;
  if (*ws) (void)hipFree(*ws);
  *ws = nullptr;
  *have = 0;
  size_t sz = std::max(need, (size_t)1 << 20);
  if (hipMalloc(ws, sz) != hipSuccess) {
    *ws = nullptr;
    return GBP_E_ALLOC;
  }
  *have = sz;
  return GBP_OK;
}

// the device's look-ahead stream of the planner loop (created once per
// process and device; null on failure); gbp_plan.hip
hipStream_t gbp_internal_la_stream(int device, int num_cus);

// the persistent validate kernel with the batch size read on the device from
// n_dev (n_max bounds the grid); gbp_engine.hip
int gbp_internal_validate_dev_n(gbp_terrain *t, int64_t n_max, const int *n_dev, const double *s,
                                const double *a, const uint8_t *dir, int dir_all, int adaptive,
                                uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                                uint32_t *counts, hipStream_t st);

