// gbp_device.h — device-side building blocks of the MI355X extend/validity engine.
//
// Everything here is FP64 in the reference's operation order; the translation
// unit is compiled with -ffp-contract=off (and the pragma below) so no
// v_fma_f64 is formed: hipcc contracts a*b+c by default on gfx950.
// Reference citations are given per function (paths relative to the reference
// repository root).
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gbp.h"

namespace gbp {

// ---- constants: include/global_body_planner/planning_utils.h:21-66 --------
constexpr double H_MAX = 0.4;
constexpr double H_MIN = 0.075;
constexpr double V_MAX = 2.0;
constexpr double V_NOM = 0.75;
constexpr double P_MAX = 1.0;
constexpr double ANG_ACC_MAX = 7.0;
constexpr double ROBOT_L = 0.3;
constexpr double ROBOT_W = 0.3;
constexpr double ROBOT_H = 0.05;
constexpr double M_CONST = 13;
constexpr double G_CONST = 9.81;
constexpr double F_MAX = 637;
constexpr double MU = 1.0;
constexpr double T_F_MAX = 0.5;
constexpr double T_F_MIN = 0.0;
constexpr double KINEMATICS_RES = 0.05;
constexpr double BACKUP_RATIO = 0.5;
constexpr double GOAL_BOUNDS = 0.5;
constexpr double MY_PI = 3.14159;
constexpr double FRAGILE_EPS = 1e-12;
constexpr uint32_t PURPOSE_STATE = 1u;
constexpr uint32_t PURPOSE_ACTION = 2u;

__device__ __forceinline__ double std_min(double a, double b) { return (b < a) ? b : a; }
__device__ __forceinline__ double std_max(double a, double b) { return (a < b) ? b : a; }

// ---- device terrain view ----------------------------------------------------
// Heights FastTerrainMap::z_data_[ix][iy] in fp32 (lossless for grid_map maps,
// whose layers are float) or fp64, stored as X-PAIRS: for 0 <= ix < nx-1,
//   zp[2*(ix*ny + iy) + {0,1}] = z[ix][iy], z[ix+1][iy]
// so the four corners of cell (ix, iy) are the two adjacent pairs at iy and
// iy+1: one 16-B (fp32) load from one cache line (15 lines in 16) instead of
// four 4-B gathers from two rows, at twice the rows' footprint (8 MB at
// 1024^2, fp32).  Measured against the alternatives (tools/diag.py, synth-
// rough-1024): x-major rows (4 MB, 4 loads) and cell quads (16 B per cell,
// 16 MB, 1 aligned load) are 7-8 % slower on the validate kernel and 8-24 %
// slower on lookups: the quads' footprint drops the L2 hit rate from 86 % to
// 39 %.  Every lookup's cell is clamped into range, so no other z is read.

template <class ZT>
struct TerrainView {
  const double *x, *y;           // coordinates (ascending)
  const ZT *z;                   // heights: x-pairs
  const double *dx, *dy, *dz;    // slope layers, x-major fp64, may be null
  int nx, ny;
  double x0, xN, y0, yN;         // x[0], x[nx-1], y[0], y[ny-1]
  double xNm, yNm;               // x[nx-2], y[ny-2]: the last cell's lower lines
  double inv_hx, inv_hy;         // 1 / mean spacing (bracket guess only)
  int one_x, one_y;              // host-verified: the guess is within one cell of the
                                 // bracket for every v (gbp_terrain_create), so a single
                                 // branch-free correction step is exact
  // host-verified affine coordinates (gbp_terrain_create): x[i] is bit-for-bit
  // ax + hx * (double)(i - bx) for every i (likewise y), e.g. x[i] = i * 0.02
  // (synthetic maps) or grid_map's reversed cell centres, so CM == 2 kernels
  // compute coordinates instead of reading them
  int affine;
  int bx, by;
  double ax, hx, ay, hy;
  // host-verified cell-area reciprocal (gbp_terrain_create): when nonzero, two
  // Newton steps from this seed give exactly 1.0 / ((x2-x1)*(y2-y1)) for every
  // pair of grid spacings of the terrain (recip_area)
  double rcp_seed;
  // the FRAGILE margin (GBP_OPT_FRAGILE_EPS): FRAGILE_EPS unless a caller asked
  // for a wider one (more host re-decisions, never a different result)
  double feps;
};

// Coordinate modes of the hot kernels (template CM): 0 = coordinate vectors
// read from global memory, 1 = staged in LDS (the pointers in the view point
// there), 2 = computed from the verified affine form.
template <int CM, int AX, class ZT>
__device__ __forceinline__ double coord(const TerrainView<ZT> &T, int i) {
  if constexpr (CM == 2) {
    return AX == 0 ? T.ax + T.hx * (double)(i - T.bx) : T.ay + T.hy * (double)(i - T.by);
  } else {
    return AX == 0 ? T.x[i] : T.y[i];
  }
}

// First i with d[i] <= v < d[i+1] (fast_terrain_map.cpp:101-117).  O(1): a
// guess from the mean spacing, then a fix-up against the actual coordinates,
// so the result equals the reference's linear scan for any ascending vector.
// No bracket: BR_LOW when v is NaN or below d[0] (the scan never reads past
// the end; the reference keeps index 0), BR_HIGH when v >= d[n-1] (the scan
// reads d[n]: UB).
constexpr int BR_LOW = -1;
constexpr int BR_HIGH = -2;

__device__ __forceinline__ int bracket_guess(int n, double d0, double inv, double v) {
  const int i = (int)((v - d0) * inv);
  return i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
}

__device__ __forceinline__ int bracket(const double *__restrict__ d, int n, double d0,
                                       double dN, double inv, int one, double v) {
  if (!(v >= d0 && v < dN)) return (v >= dN) ? BR_HIGH : BR_LOW;
  int i = bracket_guess(n, d0, inv, v);
  if (one) {
    i += (v >= d[i + 1] ? 1 : 0) - (v < d[i] ? 1 : 0);
  } else {
    while (i > 0 && v < d[i]) --i;
    while (i < n - 2 && v >= d[i + 1]) ++i;
  }
  return i;
}

// the four corners of cell (ix, iy), ix <= nx-2, iy <= ny-2, in Probe::q order
template <class ZT>
__device__ __forceinline__ void fetch_cell(const TerrainView<ZT> &T, int ix, int iy, ZT q[4]) {
  // x-pairs: zp[ix*ny + iy] = {z[ix][iy], z[ix+1][iy]}; the cell is 2 adjacent pairs
  typedef ZT pair4 __attribute__((ext_vector_type(4), aligned(2 * sizeof(ZT))));
  const pair4 c = *(const pair4 *)(T.z + 2 * ((size_t)ix * T.ny + iy));
  q[0] = c[0];
  q[2] = c[1];
  q[1] = c[2];
  q[3] = c[3];
}

// bracket() of axis AX of the view, coordinates per CM.  ONE: the caller has
// checked (wave-uniformly) that the view's one-step guess is exact on both
// axes; the bracket is then straight-line code — the guess from a point
// clamped into the domain (so the coordinate reads stay in range and a NaN
// never reaches the int conversion), one correction step, and the
// out-of-domain codes as selects — so the ten probes of a state check form
// one block the compiler schedules together (their coordinate reads and
// terrain gathers in flight at once) instead of ten branchy regions each
// waiting on its own reads.
// `cell` receives a valid cell index that the caller fetches from
// unconditionally: the bracket; without one, the cell at the domain edge the
// point lies beyond (0 below d[0] or for NaN — the cell the reference's
// heightIsNan tests — and n-2 at or above d[n-1]), so the cell's bounding
// coordinates are the lines a FRAGILE margin must be measured to.  The
// straight-line form's index is then used on every path, so the compiler
// cannot sink its computation (and the coordinate reads) back under a branch.
template <int CM, int AX, bool ONE = false, class ZT>
__device__ __forceinline__ int bracket_ax(const TerrainView<ZT> &T, double v, int &cell) {
  const double d0 = AX == 0 ? T.x0 : T.y0, dN = AX == 0 ? T.xN : T.yN;
  const int n = AX == 0 ? T.nx : T.ny;
  if constexpr (ONE) {
    const bool in = (v >= d0) & (v < dN);
    // the point clamped into [d[0], d[n-2]]: itself in the domain, d[0] below
    // it or for NaN (fmax returns the non-NaN operand), d[n-2] at or above
    // d[n-1] — whose brackets are the cells above (guess 0 / n-2, exact)
    const double vc = fmin(fmax(v, d0), AX == 0 ? T.xNm : T.yNm);
    int i = bracket_guess(n, d0, AX == 0 ? T.inv_hx : T.inv_hy, vc);
    i += (vc >= coord<CM, AX>(T, i + 1) ? 1 : 0) - (vc < coord<CM, AX>(T, i) ? 1 : 0);
    cell = i;
    return in ? i : (v >= dN ? BR_HIGH : BR_LOW);
  }
  const int r = bracket_ax<CM, AX, false>(T, v);
  cell = r >= 0 ? r : (r == BR_HIGH ? n - 2 : 0);
  return r;
}
template <int CM, int AX, bool ONE = false, class ZT>
__device__ __forceinline__ int bracket_ax(const TerrainView<ZT> &T, double v) {
  static_assert(!ONE, "the straight-line bracket returns its cell");
  const double d0 = AX == 0 ? T.x0 : T.y0, dN = AX == 0 ? T.xN : T.yN;
  const int n = AX == 0 ? T.nx : T.ny;
  if (!(v >= d0 && v < dN)) return (v >= dN) ? BR_HIGH : BR_LOW;
  int i = bracket_guess(n, d0, AX == 0 ? T.inv_hx : T.inv_hy, v);
  if (AX == 0 ? T.one_x : T.one_y) {
    i += (v >= coord<CM, AX>(T, i + 1) ? 1 : 0) - (v < coord<CM, AX>(T, i) ? 1 : 0);
  } else {
    while (i > 0 && v < coord<CM, AX>(T, i)) --i;
    while (i < n - 2 && v >= coord<CM, AX>(T, i + 1)) ++i;
  }
  return i;
}

template <class ZT>
__device__ __forceinline__ void load_quad(const TerrainView<ZT> &T, int ix, int iy, double &f11,
                                          double &f12, double &f21, double &f22) {
  ZT q[4];
  fetch_cell(T, ix, iy, q);
  f11 = (double)q[0];
  f12 = (double)q[1];
  f21 = (double)q[2];
  f22 = (double)q[3];
}

// FastTerrainMap::heightIsNan (fast_terrain_map.cpp:135-157): -1 = UB
// (BR_HIGH on an axis), else the reference's bool (BR_LOW -> index 0)
template <class ZT>
__device__ __forceinline__ int nan_at(const TerrainView<ZT> &T, double x, double y) {
  const int ix = bracket(T.x, T.nx, T.x0, T.xN, T.inv_hx, T.one_x, x);
  const int iy = bracket(T.y, T.ny, T.y0, T.yN, T.inv_hy, T.one_y, y);
  if (ix == BR_HIGH || iy == BR_HIGH) return -1;
  double f11, f12, f21, f22;
  load_quad(T, ix < 0 ? 0 : ix, iy < 0 ? 0 : iy, f11, f12, f21, f22);
  return (isnan(f11) || isnan(f12) || isnan(f21) || isnan(f22)) ? 1 : 0;
}

// 1.0 / d for a cell area d = (x2 - x1) * (y2 - y1) (fast_terrain_map.cpp:124):
// the IEEE quotient, or, when the host has checked bit-for-bit that it equals
// the quotient for every (x-spacing, y-spacing) pair of the terrain, two
// Newton steps from the terrain's uniform seed 1 / (mean area) — four FMAs
// instead of the scaled division sequence (v_rcp + v_div_scale/fmas/fixup).
// `seed` is wave-uniform, so the branch is too.
__host__ __device__ __forceinline__ double recip_newton(double d, double seed) {
  const double e0 = __builtin_fma(-d, seed, 1.0);
  const double y1 = __builtin_fma(seed, e0, seed);
  const double e1 = __builtin_fma(-d, y1, 1.0);
  return __builtin_fma(y1, e1, y1);
}
__device__ __forceinline__ double recip_area(double d, double seed) {
  return seed != 0.0 ? recip_newton(d, seed) : 1.0 / d;
}

// fast_terrain_map.cpp:124-126 (left-to-right evaluation, no contraction)
__device__ __forceinline__ double bilinear(double f11, double f12, double f21, double f22,
                                           double x1, double x2, double y1, double y2,
                                           double x, double y, double seed = 0.0) {
  return recip_area((x2 - x1) * (y2 - y1), seed) *
         (f11 * (x2 - x) * (y2 - y) + f21 * (x - x1) * (y2 - y) + f12 * (x2 - x) * (y - y1) +
          f22 * (x - x1) * (y - y1));
}

// FastTerrainMap::getGroundHeight (fast_terrain_map.cpp:94-132).  Returns
// false for UB (finite point without bracket).  NaN coordinates give NaN
// (whatever the uninitialised x1..y2 hold).  `near` is set when the point is
// within FRAGILE_EPS of a grid line.
template <class ZT>
__device__ __forceinline__ bool height_at(const TerrainView<ZT> &T, double x, double y,
                                          double &h, bool &near) {
  if (isnan(x) || isnan(y)) {
    h = __builtin_nan("");
    return true;
  }
  const int ix = bracket(T.x, T.nx, T.x0, T.xN, T.inv_hx, T.one_x, x);
  const int iy = bracket(T.y, T.ny, T.y0, T.yN, T.inv_hy, T.one_y, y);
  if (ix < 0 || iy < 0) return false;
  const double x1 = T.x[ix], x2 = T.x[ix + 1], y1 = T.y[iy], y2 = T.y[iy + 1];
  double f11, f12, f21, f22;
  load_quad(T, ix, iy, f11, f12, f21, f22);
  near = near || fabs(x - x1) < FRAGILE_EPS || fabs(x2 - x) < FRAGILE_EPS ||
         fabs(y - y1) < FRAGILE_EPS || fabs(y2 - y) < FRAGILE_EPS;
  h = bilinear(f11, f12, f21, f22, x1, x2, y1, y2, x, y, T.rcp_seed);
  return true;
}

// ---- batched lookups ------------------------------------------------------------
// A probe = one lookup point's bracket plus its four heights, fetched
// UNCONDITIONALLY from a clamped (always valid) cell so that every fetch of a
// state check can be in flight at once; the reference's sequential logic and
// early exits are then replayed on the fetched values (is_valid_state below).
template <class ZT>
struct Probe {
  int ix, iy;   // bracket codes: >= 0, BR_LOW or BR_HIGH
  int cx, cy;   // the fetched cell: the bracket, or 0 on an axis without one
  ZT q[4];      // z[cx][cy], z[cx][cy+1], z[cx+1][cy], z[cx+1][cy+1]
};

template <class ZT, int CM = 0, bool ONE = false>
__device__ __forceinline__ void probe(const TerrainView<ZT> &T, double x, double y, Probe<ZT> &p) {
  p.ix = bracket_ax<CM, 0, ONE>(T, x, p.cx);
  p.iy = bracket_ax<CM, 1, ONE>(T, y, p.cy);
  fetch_cell(T, p.cx, p.cy, p.q);
}

// heightIsNan on a probe: -1 = UB (BR_HIGH), else the reference's bool
// Branch-free (bitwise ors, a select): the cell's heights are then used on
// every path, so the compiler keeps the probe's fetch with the others instead
// of sinking it under the BR_HIGH test and waiting on it at once (the centre
// probe's gather was issued and waited for alone, before the rotation).
template <class ZT>
__device__ __forceinline__ int probe_nan(const Probe<ZT> &p) {
  const bool high = (p.ix == BR_HIGH) | (p.iy == BR_HIGH);
  const bool nan4 = (int)isnan(p.q[0]) | (int)isnan(p.q[1]) | (int)isnan(p.q[2]) | (int)isnan(p.q[3]);
  return high ? -1 : (nan4 ? 1 : 0);
}

// getGroundHeight on a probe (same contract as height_at)
template <class ZT, int CM = 0>
__device__ __forceinline__ bool probe_height(const TerrainView<ZT> &T, const Probe<ZT> &p,
                                             double x, double y, double &h, bool &near) {
  if (isnan(x) || isnan(y)) {
    h = __builtin_nan("");
    return true;
  }
  if (p.ix < 0 || p.iy < 0) return false;
  const double x1 = coord<CM, 0>(T, p.ix), x2 = coord<CM, 0>(T, p.ix + 1);
  const double y1 = coord<CM, 1>(T, p.iy), y2 = coord<CM, 1>(T, p.iy + 1);
  near = near || fabs(x - x1) < FRAGILE_EPS || fabs(x2 - x) < FRAGILE_EPS ||
         fabs(y - y1) < FRAGILE_EPS || fabs(y2 - y) < FRAGILE_EPS;
  h = bilinear((double)p.q[0], (double)p.q[1], (double)p.q[2], (double)p.q[3], x1, x2, y1, y2, x, y,
               T.rcp_seed);
  return true;
}

// fast_terrain_map.cpp:160-213
template <class ZT>
__device__ __forceinline__ bool surface_normal(const TerrainView<ZT> &T, double x, double y,
                                               double n[3]) {
  const int ix = bracket(T.x, T.nx, T.x0, T.xN, T.inv_hx, T.one_x, x);
  const int iy = bracket(T.y, T.ny, T.y0, T.yN, T.inv_hy, T.one_y, y);
  if (isnan(x) || isnan(y) || ix < 0 || iy < 0) {
    n[0] = n[1] = n[2] = __builtin_nan("");
    return isnan(x) || isnan(y);  // NaN coordinates: deterministic NaN, not UB
  }
  if (!T.dx) {
    n[0] = 0.0; n[1] = 0.0; n[2] = 1.0;
    return true;
  }
  double x1 = T.x[ix], x2 = T.x[ix + 1], y1 = T.y[iy], y2 = T.y[iy + 1];
  size_t b = (size_t)ix * T.ny + iy;
  const double *L[3] = {T.dx, T.dy, T.dz};
#pragma unroll
  for (int k = 0; k < 3; k++)
    n[k] = bilinear(L[k][b], L[k][b + 1], L[k][b + T.ny], L[k][b + T.ny + 1], x1, x2, y1, y2, x,
                    y, T.rcp_seed);
  return true;
}

// stance divisions x / (6 t_s), x / (2 t_s) (Markstein with a constant
// reciprocal was measured: no faster than the hardware-assisted sequence)
__device__ __forceinline__ double pdiv(double x, double d) {
  return x / d;
}
#define PDIV6(x) pdiv((x), 6.0 * t_s)
#define PDIV2(x) pdiv((x), 2.0 * t_s)
// ---- propagation --------------------------------------------------------------
// planning_utils.cpp:237-274
__device__ __forceinline__ void apply_stance(const double *s, const double *a, double t,
                                             double *o) {
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  o[0] = s[0] + s[3] * t + 0.5 * a_x_td * t * t + PDIV6((a_x_to - a_x_td) * (t * t * t));
  o[1] = s[1] + s[4] * t + 0.5 * a_y_td * t * t + PDIV6((a_y_to - a_y_td) * (t * t * t));
  o[2] = s[2] + s[5] * t + 0.5 * a_z_td * t * t + PDIV6((a_z_to - a_z_td) * (t * t * t));
  o[3] = s[3] + a_x_td * t + PDIV2((a_x_to - a_x_td) * t * t);
  o[4] = s[4] + a_y_td * t + PDIV2((a_y_to - a_y_td) * t * t);
  o[5] = s[5] + a_z_td * t + PDIV2((a_z_to - a_z_td) * t * t);
  o[6] = s[6] + s[7] * t + 0.5 * a_p_td * t * t + PDIV6((a_p_to - a_p_td) * (t * t * t));
  o[7] = s[7] + a_p_td * t + PDIV2((a_p_to - a_p_td) * t * t);
}

// planning_utils.cpp:282-306 (g is the literal 9.81)
__device__ __forceinline__ void apply_flight(const double *s, double t_f, double *o) {
  const double g = 9.81;
  o[0] = s[0] + s[3] * t_f;
  o[1] = s[1] + s[4] * t_f;
  o[2] = s[2] + s[5] * t_f - 0.5 * g * t_f * t_f;
  o[3] = s[3];
  o[4] = s[4];
  o[5] = s[5] - g * t_f;
  o[6] = s[6] + s[7] * t_f;
  o[7] = s[7];
}

// planning_utils.cpp:324-367
__device__ __forceinline__ void apply_stance_reverse(const double *s, const double *a, double t,
                                                     double *o) {
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  const double cx = s[3] - a_x_td * t_s - 0.5 * (a_x_to - a_x_td) * t_s;
  const double cy = s[4] - a_y_td * t_s - 0.5 * (a_y_to - a_y_td) * t_s;
  const double cz = s[5] - a_z_td * t_s - 0.5 * (a_z_to - a_z_td) * t_s;
  const double cp = s[7] - a_p_td * t_s - 0.5 * (a_p_to - a_p_td) * t_s;
  const double d1 = t_s - t, d2 = t_s * t_s - t * t, d3 = t_s * t_s * t_s - t * t * t;
  o[0] = s[0] - cx * d1 - 0.5 * a_x_td * d2 - PDIV6((a_x_to - a_x_td) * d3);
  o[1] = s[1] - cy * d1 - 0.5 * a_y_td * d2 - PDIV6((a_y_to - a_y_td) * d3);
  o[2] = s[2] - cz * d1 - 0.5 * a_z_td * d2 - PDIV6((a_z_to - a_z_td) * d3);
  o[3] = s[3] - a_x_td * d1 - PDIV2((a_x_to - a_x_td) * d2);
  o[4] = s[4] - a_y_td * d1 - PDIV2((a_y_to - a_y_td) * d2);
  o[5] = s[5] - a_z_td * d1 - PDIV2((a_z_to - a_z_td) * d2);
  o[7] = s[7] - a_p_td * d1 - PDIV2((a_p_to - a_p_td) * d2);
  o[6] = s[6] - cp * d1 - 0.5 * a_p_td * d2 - PDIV6((a_p_to - a_p_td) * d3);
}

// planning_utils.cpp:519-556
__device__ __forceinline__ bool is_valid_action(const double *a) {
  if ((a[6] <= 0) || (a[7] < 0)) return false;
  const double m = M_CONST, g = G_CONST, mu = MU;
  const double f_x_td = m * a[0], f_y_td = m * a[1], f_z_td = m * (a[2] + g);
  const double f_x_to = m * a[3], f_y_to = m * a[4], f_z_to = m * (a[5] + g);
  if ((sqrt(f_x_td * f_x_td + f_y_td * f_y_td + f_z_td * f_z_td) >= F_MAX) ||
      (sqrt(f_x_to * f_x_to + f_y_to * f_y_to + f_z_to * f_z_to) >= F_MAX) || (f_z_td < 0) ||
      (f_z_to < 0) || (a[8] >= F_MAX) || (a[9] >= F_MAX))
    return false;
  if ((sqrt(f_x_td * f_x_td + f_y_td * f_y_td) >= mu * f_z_td) ||
      (sqrt(f_x_to * f_x_to + f_y_to * f_y_to) >= mu * f_z_to))
    return false;
  return true;
}

// A 64-bit constant materialised AT ITS USE (two s_mov_b32 inside the loop
// body, an SGPR pair that lives for one instruction): left to itself the
// compiler hoists every polynomial coefficient out of the persistent loop and
// keeps it for the whole kernel, in VGPRs (with libm's atan2/sin/cos tables,
// ~80 of them: what held the validate kernel at 2 waves per SIMD) or, short
// of SGPRs, in VGPR spill lanes read back with v_readlane at every use.
template <uint64_t BITS>
__device__ __forceinline__ double kc() {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)(BITS & 0xFFFFFFFFu)));
  asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(BITS >> 32)));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
#define KC(v) kc<__builtin_bit_cast(uint64_t, (double)(v))>()

// isValidState's rotation (planning_utils.cpp:578-594) for a state that passed
// checks (2)-(3), i.e. |p| < P_MAX = 1 and speed = |(dx, dy)| <= V_MAX (or
// NaN), without libm, whose constant tables would stay resident for the whole
// persistent loop.  The reference forms these values with glibc's atan2 /
// cos / sin, which no device libm reproduces bit for bit either; decisions
// within FRAGILE_EPS of a threshold are therefore flagged GBP_F_FRAGILE and
// re-decided on the host with glibc (gbp_host_check.cpp):
//  * yaw: cos/sin(atan2(dy, dx)) = dx/|v|, dy/|v| (<= 2 ulp).  Below 1e-150
//    the components are first scaled by 2^600 (exact) so dx^2 + dy^2 cannot
//    underflow; |v| = 0 takes atan2's signed-zero results, atan2(+-0, +0) =
//    +-0 -> (1, +-0) and atan2(+-0, -0) = +-pi -> (-1, +-1.2246467991473532e-16)
//    (the correctly rounded cos/sin of the double nearest pi).  NaN propagates.
//  * pitch: Taylor series to p^19 / p^20 (truncation < 5e-20); NaN propagates.
// Lanes that already failed a check run the same code on values nobody reads.
__device__ __forceinline__ void rotation_trig_nolibm(double dx, double dy, double speed, double p,
                                                     double &cy, double &sy, double &cp,
                                                     double &sp) {
  cy = dx / speed;
  sy = dy / speed;
  if (speed < 1e-150) {  // rare; false for NaN (the quotients are NaN, as atan2 is)
    if (speed == 0) {
      const bool west = signbit(dx);
      cy = west ? -1.0 : 1.0;
      sy = west ? copysign(1.2246467991473532e-16, dy) : dy;
    } else {
      const double xs = dx * 0x1p600, ys = dy * 0x1p600;
      const double r = sqrt(xs * xs + ys * ys);
      cy = xs / r;
      sy = ys / r;
    }
  }
  if (p == 0) {  // sin(+-0) = +-0, cos(+-0) = 1 exactly, as glibc
    sp = p;
    cp = 1.0;
    return;
  }
  const double z = p * p;
  double ps = KC(-1.0 / 121645100408832000.0);              // -1/19!
  ps = __builtin_fma(ps, z, KC(1.0 / 355687428096000.0));   //  1/17!
  ps = __builtin_fma(ps, z, KC(-1.0 / 1307674368000.0));    // -1/15!
  ps = __builtin_fma(ps, z, KC(1.0 / 6227020800.0));        //  1/13!
  ps = __builtin_fma(ps, z, KC(-1.0 / 39916800.0));         // -1/11!
  ps = __builtin_fma(ps, z, KC(1.0 / 362880.0));            //  1/9!
  ps = __builtin_fma(ps, z, KC(-1.0 / 5040.0));             // -1/7!
  ps = __builtin_fma(ps, z, KC(1.0 / 120.0));               //  1/5!
  ps = __builtin_fma(ps, z, KC(-1.0 / 6.0));                // -1/3!
  sp = __builtin_fma(p * z, ps, p);
  double pc = KC(1.0 / 2432902008176640000.0);              //  1/20!
  pc = __builtin_fma(pc, z, KC(-1.0 / 6402373705728000.0)); // -1/18!
  pc = __builtin_fma(pc, z, KC(1.0 / 20922789888000.0));    //  1/16!
  pc = __builtin_fma(pc, z, KC(-1.0 / 87178291200.0));      // -1/14!
  pc = __builtin_fma(pc, z, KC(1.0 / 479001600.0));         //  1/12!
  pc = __builtin_fma(pc, z, KC(-1.0 / 3628800.0));          // -1/10!
  pc = __builtin_fma(pc, z, KC(1.0 / 40320.0));             //  1/8!
  pc = __builtin_fma(pc, z, KC(-1.0 / 720.0));              // -1/6!
  pc = __builtin_fma(pc, z, KC(1.0 / 24.0));                //  1/4!
  pc = __builtin_fma(pc, z, -0.5);                          // -1/2!
  cp = __builtin_fma(z, pc, 1.0);
}

// ---- state validity: planning_utils.cpp:562-635 ------------------------------
// Out-of-domain convention: a reached lookup with no bracket makes
// the state invalid; GBP_F_OOD marks the cases where the reference's decision
// depends on its UB read.  G/V follow the reference's executed calls.
struct Acc {
  uint32_t G, V, flags;
};

// getGroundHeight on a probe, evaluated unconditionally (branch-free form):
// the bilinear value of the clamped cell, `ok` = the reference's call would not
// be UB, `near` = the point is within FRAGILE_EPS of a line bounding its cell
// (bracket_ax): an interior grid line, or the map edge an out-of-domain point
// lies beyond or an in-domain point lies next to — where a last-ulp difference
// of the point moves it into another cell (another height, another NaN test)
// or across the domain edge (defined <-> OOD)
template <class ZT, int CM>
__device__ __forceinline__ double probe_height_bf(const TerrainView<ZT> &T, const Probe<ZT> &p,
                                                  double x, double y, double eps, bool &ok,
                                                  bool &near) {
  const bool nanxy = isnan(x) || isnan(y);
  const bool br = p.ix >= 0 && p.iy >= 0;  // else the value below is not used
  const double x1 = coord<CM, 0>(T, p.cx), x2 = coord<CM, 0>(T, p.cx + 1);
  const double y1 = coord<CM, 1>(T, p.cy), y2 = coord<CM, 1>(T, p.cy + 1);
  ok = br || nanxy;
  near = !nanxy &&
         (fabs(x - x1) < eps || fabs(x2 - x) < eps || fabs(y - y1) < eps || fabs(y2 - y) < eps);
  const double h = bilinear((double)p.q[0], (double)p.q[1], (double)p.q[2], (double)p.q[3], x1, x2,
                            y1, y2, x, y, T.rcp_seed);
  return nanxy ? __builtin_nan("") : h;
}

// isValidState as ONE straight-line pass: every lookup, height and test is
// evaluated for every lane, and the reference's sequence of early returns is
// replayed as a predicate `alive` (a test only counts, sets flags or rejects
// while every earlier test has passed).  Lanes of a wave hold unrelated
// states, so the early-return form executes nearly every branch per wave
// anyway and pays the exec-mask bookkeeping on top; here the wave issues one
// path.  Same values, same decisions, same G/V and flags as the reference's
// executed calls.
template <class ZT, int CM = 0, bool ONE = false>
__device__ bool is_valid_state(const TerrainView<ZT> &T, const double *s, int phase, Acc &acc) {
  if (acc.V >= GBP_MAX_SAMPLES) {  // engine guard: the reference loop would not terminate
    acc.flags |= GBP_F_LIMIT;
    return false;
  }
  acc.V++;
  const double eps = T.feps, hmin = H_MIN, hmax = H_MAX, hl = 0.5 * ROBOT_L, hw = 0.5 * ROBOT_W;
  const bool outside = (s[0] < T.x0) || (s[0] > T.xN) || (s[1] < T.y0) || (s[1] > T.yN);
  const double speed = sqrt(s[3] * s[3] + s[4] * s[4]);
  // (4) rotation :578-594, formed first so that the centre's gather is issued
  // with the nine others (one round trip per state check, not two)
  double cy, sy, cp, sp;
  rotation_trig_nolibm(s[3], s[4], speed, s[6], cy, sy, cp, sp);
  Probe<ZT> pc;
  probe<ZT, CM, ONE>(T, s[0], s[1], pc);
  // A state heading along +x with zero pitch (dy = +-0, dx > 0, p = +-0: every
  // start / goal state of the reference node, global_body_planner.cpp:219-264)
  // has exactly glibc's trig values: atan2(+-0, dx) = +-0 -> (1, +-0), and
  // dx / |v| = 1 since sqrt(dx*dx) == |dx| in binary64.  Its lookup points
  // and heights are then glibc's bit for bit, so no decision can differ and
  // nothing is FRAGILE.
  const double feps = (s[4] == 0 && s[3] > 0 && s[6] == 0) ? 0.0 : eps;
  const double R_11 = cy * cp, R_12 = -sy, R_13 = cy * sp;
  const double R_21 = sy * cp, R_22 = cy, R_23 = sy * sp;
  const double R_31 = -sp, R_32 = 0, R_33 = cp;
  const double z_body = -ROBOT_H;
  Probe<ZT> pl[4], pk[4], pu;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double x_body = (k < 2) ? -hl : hl;
    const double y_body = (k & 1) ? hw : -hw;
    const double x_leg = s[0] + R_11 * x_body + R_12 * y_body;
    const double y_leg = s[1] + R_21 * x_body + R_22 * y_body;
    probe<ZT, CM, ONE>(T, x_leg, y_leg, pl[k]);
    probe<ZT, CM, ONE>(T, x_leg + R_13 * z_body, y_leg + R_23 * z_body, pk[k]);
  }
  const double ux = s[0] + R_13 * z_body, uy = s[1] + R_23 * z_body;
  probe<ZT, CM, ONE>(T, ux, uy, pu);
  uint32_t fl = 0;
  // (1) heightIsNan(centre) :564 (x or y >= the last coordinate: UB, rejected
  //     by (2) unless exactly equal)
  const int r = probe_nan(pc);
  if (r < 0 && !outside) fl |= GBP_F_OOD;
  if (r > 0) fl |= GBP_F_NAN;
  // (2) bounds + |pitch| :568-571, (3) horizontal speed :574
  bool alive = r == 0 && !(outside || (fabs(s[6]) >= P_MAX)) && !(speed > V_MAX);
  uint32_t G = 0;
  // (5) four corners :601-627, x_body outer, y_body inner, in reference order
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double x_body = (k < 2) ? -hl : hl;
    const double y_body = (k & 1) ? hw : -hw;
    const double x_leg = s[0] + R_11 * x_body + R_12 * y_body;
    const double y_leg = s[1] + R_21 * x_body + R_22 * y_body;
    const double z_leg = s[2] + R_31 * x_body + R_32 * y_body;
    const double x_corner = x_leg + R_13 * z_body;
    const double y_corner = y_leg + R_23 * z_body;
    const double z_corner = z_leg + R_33 * z_body;
    const int rl = probe_nan(pl[k]);  // heightIsNan(leg) :614
    bool okl, okc, nl, nc;
    const double gl = probe_height_bf<ZT, CM>(T, pl[k], x_leg, y_leg, feps, okl, nl);
    const double gc = probe_height_bf<ZT, CM>(T, pk[k], x_corner, y_corner, feps, okc, nc);
    // a leg near a line bounding its cell is FRAGILE from its heightIsNan on:
    // glibc's leg may sit in the neighbouring cell (NaN <-> finite) or across
    // the map edge (OOD <-> in domain) as well as give another height
    if (alive && nl) fl |= GBP_F_FRAGILE;
    if (alive && rl < 0) fl |= GBP_F_OOD;
    if (alive && rl > 0) fl |= GBP_F_NAN;
    alive = alive && rl == 0;
    G += alive ? 2u : 0u;  // both heights computed before the test :618-619
    if (alive && !okl) fl |= GBP_F_OOD;
    alive = alive && okl;
    if (alive && nc) fl |= GBP_F_FRAGILE;
    if (alive && !okc) fl |= GBP_F_OOD;
    alive = alive && okc;
    const double leg_height = z_leg - gl;
    const double corner_height = z_corner - gc;
    if (alive && (fabs(corner_height - hmin) < feps ||
                  (phase == GBP_STANCE && fabs(leg_height - hmax) < feps)))
      fl |= GBP_F_FRAGILE;
    alive = alive && !((corner_height < hmin) || ((phase == GBP_STANCE) && (leg_height > hmax)));
  }
  // (6) underside centre :630-632
  G += alive ? 1u : 0u;
  bool oku, nu;
  const double gu = probe_height_bf<ZT, CM>(T, pu, ux, uy, feps, oku, nu);
  if (alive && nu) fl |= GBP_F_FRAGILE;
  if (alive && !oku) fl |= GBP_F_OOD;
  alive = alive && oku;
  const double height = (s[2] + R_33 * z_body) - gu;
  if (alive && fabs(height - hmin) < feps) fl |= GBP_F_FRAGILE;
  alive = alive && !(height < hmin);
  acc.G += G;
  acc.flags |= fl;
  return alive;
}

__device__ __forceinline__ uint32_t stage_bits(uint32_t k) { return k << GBP_F_STAGE_SHIFT; }

// ---- pair checks, one lane per attempt (the "direct" form) ------------------
// planning_utils.cpp:713-753 (plain) and :651-712 (adaptive)
template <class ZT, bool ADAPTIVE>
__device__ bool pair_forward(const TerrainView<ZT> &T, const double *s, const double *a,
                             double *s_new, double &t_new, Acc &acc, uint32_t &f) {
  const double t_s = a[6], t_f = a[7];
  double sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_FWD_STANCE);
  for (double t = 0; t <= t_s; t += (ADAPTIVE ? time_step : KINEMATICS_RES)) {
    apply_stance(s, a, t, sc);
    if (!is_valid_state(T, sc, GBP_STANCE, acc)) {
      if (acc.flags & GBP_F_LIMIT) return false;
      if (!ADAPTIVE || (KINEMATICS_RES - 0.01 <= time_step && time_step <= KINEMATICS_RES + 0.01)) {
        apply_stance(s, a, (1.0 - BACKUP_RATIO) * t, s_new);
        f |= GBP_F_SNEW_SET;
        return false;
      }
      time_step = KINEMATICS_RES;
      t = t_pre_success;
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) s_new[k] = sc[k];
      t_new = t;
      f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      if (ADAPTIVE) {
        time_step += KINEMATICS_RES;
        t_pre_success = t;
      }
    }
  }
  double s_takeoff[8];
  apply_stance(s, a, a[6], s_takeoff);
  time_step = KINEMATICS_RES;
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_FWD_FLIGHT);
  for (double t = 0; t < t_f; t += (ADAPTIVE ? time_step : KINEMATICS_RES)) {
    apply_flight(s_takeoff, t, sc);
    if (!is_valid_state(T, sc, GBP_FLIGHT, acc)) return false;
    if (ADAPTIVE) time_step += KINEMATICS_RES;
  }
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_FWD_LAND);
  apply_flight(s_takeoff, t_f, sc);
  if (!is_valid_state(T, sc, GBP_STANCE, acc)) return false;
#pragma unroll
  for (int k = 0; k < 8; k++) s_new[k] = sc[k];
  t_new = t_s + t_f;
  f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return true;
}

// planning_utils.cpp:837-876 (plain) and :774-836 (adaptive)
template <class ZT, bool ADAPTIVE>
__device__ bool pair_reverse(const TerrainView<ZT> &T, const double *s, const double *a,
                             double *s_new, double &t_new, Acc &acc, uint32_t &f) {
  const double t_s = a[6], t_f = a[7];
  double sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_REV_FLIGHT);
  for (double t = 0; t < t_f; t += (ADAPTIVE ? time_step : KINEMATICS_RES)) {
    apply_flight(s, -t, sc);
    if (!is_valid_state(T, sc, GBP_FLIGHT, acc)) return false;
    if (ADAPTIVE) time_step += KINEMATICS_RES;
  }
  double s_takeoff[8];
  apply_flight(s, -t_f, s_takeoff);
  time_step = KINEMATICS_RES;
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_REV_STANCE);
  for (double t = t_s; t >= 0; t -= (ADAPTIVE ? time_step : KINEMATICS_RES)) {
    apply_stance_reverse(s_takeoff, a, t, sc);
    if (!is_valid_state(T, sc, GBP_STANCE, acc)) {
      if (acc.flags & GBP_F_LIMIT) return false;
      if (!ADAPTIVE || (KINEMATICS_RES - 0.01 <= time_step && time_step <= KINEMATICS_RES + 0.01)) {
        apply_stance(s, a, t + BACKUP_RATIO * (t_s - t), s_new);  // forward stance, as written (:857)
        f |= GBP_F_SNEW_SET;
        return false;
      }
      time_step = KINEMATICS_RES;
      t = t_pre_success;
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) s_new[k] = sc[k];
      t_new = t_s - t;
      f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      if (ADAPTIVE) {
        time_step += KINEMATICS_RES;
        t_pre_success = t;
      }
    }
  }
  f = (f & ~GBP_F_STAGE_MASK) | stage_bits(GBP_STAGE_REV_START);
  apply_stance_reverse(s_takeoff, a, 0, sc);
  if (!is_valid_state(T, sc, GBP_STANCE, acc)) return false;
#pragma unroll
  for (int k = 0; k < 8; k++) s_new[k] = sc[k];
  t_new = t_s;
  f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return true;
}

// ---- distances: planning_utils.cpp:106-127 -------------------------------------
__device__ __forceinline__ double state_distance(const double *q1, const double *q2) {
  double sum = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) sum = sum + 1.0 * (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return sqrt(sum);
}

__device__ __forceinline__ double pose_distance(const double *q1, const double *q2) {
  double sum = 0;  // planning_utils.cpp:106-115
#pragma unroll
  for (int i = 0; i < 3; i++) sum = sum + (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return sqrt(sum);
}

// stateYawDistance (planning_utils.h:133-145) on the two states' yaws, which
// the caller forms with glibc's atan2(q[4], q[3]) as the reference does (no
// device atan2 reproduces glibc's bits); std::min / std::max as selects
__device__ __forceinline__ double yaw_distance(double yaw1, double yaw2) {
  const double yaw_min = (yaw2 < yaw1) ? yaw2 : yaw1;
  const double yaw_max = (yaw1 < yaw2) ? yaw2 : yaw1;
  const double a = yaw_max - yaw_min, b = yaw_min + 2 * MY_PI - yaw_max;
  return (b < a) ? b : a;
}

// ---- Philox4x32-10 counter RNG (Salmon et al., SC'11) -------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c[0]), lo0 = 0xD2511F53u * c[0];
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]), lo1 = 0xCD9E8D57u * c[2];
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

// two uniforms in [0,1) for (seed, stream_id, purpose, index, draw)
__device__ __forceinline__ void uniform2(uint64_t seed, uint64_t stream_id, uint32_t purpose,
                                         int64_t index, uint32_t draw, double &u0, double &u1) {
  uint32_t c[4] = {draw, (uint32_t)(uint64_t)index, (uint32_t)((uint64_t)index >> 32),
                   (uint32_t)stream_id ^ (purpose << 24)};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(stream_id >> 32));
  const uint64_t w0 = ((uint64_t)c[1] << 32) | c[0];
  const uint64_t w1 = ((uint64_t)c[3] << 32) | c[2];
  u0 = (double)(w0 >> 11) * 0x1p-53;
  u1 = (double)(w1 >> 11) * 0x1p-53;
}

// ---- the samplers' transcendentals -------------------------------------------
// The reference's draws (rand(), clock-seeded engines) are not reproducible
// (SURVEY H11), so the engine defines its own streams and with them the log /
// sin / cos / acos / atan2 that shape the uniforms.  The device libm and glibc
// differ in the last bits; these routines use only +, -, *, /, sqrt, floor and
// frexp (correctly rounded or exact in binary64), no contraction, a fixed
// Horner order — the CPU restatement under oracle/ restates them, so the
// host and the device draw bit-identical targets and candidate actions and a
// whole planner run can be replayed on the CPU bit for bit.  A few ulp of
// accuracy (series past 1e-17 relative): the sampled distributions are the
// reference's.
constexpr double RM_SIN[9] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7,
                                       -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
                                       -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                                       -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49,
                                       -0x1.2f49b46814157p-57};
constexpr double RM_COS[9] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5,
                                       -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
                                       -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29,
                                       -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45,
                                       -0x1.6827863b97d97p-53};
constexpr double RM_LOG[11] = {0x1.5555555555555p-1, 0x1.999999999999ap-2,
                                        0x1.2492492492492p-2, 0x1.c71c71c71c71cp-3,
                                        0x1.745d1745d1746p-3, 0x1.3b13b13b13b14p-3,
                                        0x1.1111111111111p-3, 0x1.e1e1e1e1e1e1ep-4,
                                        0x1.af286bca1af28p-4, 0x1.8618618618618p-4,
                                        0x1.642c8590b2164p-4};
constexpr double RM_ATAN[12] = {-0x1.5555555555555p-2, 0x1.999999999999ap-3,
                                         -0x1.2492492492492p-3, 0x1.c71c71c71c71cp-4,
                                         -0x1.745d1745d1746p-4, 0x1.3b13b13b13b14p-4,
                                         -0x1.1111111111111p-4, 0x1.e1e1e1e1e1e1ep-5,
                                         -0x1.af286bca1af28p-5, 0x1.8618618618618p-5,
                                         -0x1.642c8590b2164p-5, 0x1.47ae147ae147bp-5};
constexpr double RM_INVPIO2 = 0x1.45f306dc9c883p-1;
constexpr double RM_PIO2_1 = 0x1.921fb54400000p+0, RM_PIO2_2 = 0x1.0b4611a600000p-34,
                 RM_PIO2_2T = 0x1.3198a2e037073p-69;
constexpr double RM_PIO2_HI = 0x1.921fb54442d18p+0, RM_PIO2_LO = 0x1.1a62633145c07p-54;
constexpr double RM_PI_HI = 0x1.921fb54442d18p+1, RM_PI_LO = 0x1.1a62633145c07p-53;
constexpr double RM_LN2_HI = 0x1.62e42fee00000p-1, RM_LN2_LO = 0x1.a39ef35793c76p-33;

// ln x, x > 0 finite: x = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(f)
__device__ __forceinline__ double rm_log(double x) {
  int e;
  double m = frexp(x, &e);
  if (m < 0x1.6a09e667f3bcdp-1) {
    m = m * 2.0;
    e = e - 1;
  }
  const double f = (m - 1.0) / (m + 1.0);
  const double w = f * f;
  double p = RM_LOG[10];
#pragma unroll
  for (int k = 9; k >= 0; k--) p = RM_LOG[k] + w * p;
  const double l = 2.0 * f + f * w * p;
  const double de = (double)e;
  return de * RM_LN2_HI + (l + de * RM_LN2_LO);
}

// sin x, cos x for |x| < 2^20: x = k pi/2 + r (Cody-Waite, three parts)
__device__ __forceinline__ void rm_sincos(double x, double &s, double &c) {
  const double kf = floor(x * RM_INVPIO2 + 0.5);
  const double r = ((x - kf * RM_PIO2_1) - kf * RM_PIO2_2) - kf * RM_PIO2_2T;
  const double z = r * r;
  double ps = RM_SIN[8], pc = RM_COS[8];
#pragma unroll
  for (int k = 7; k >= 0; k--) {
    ps = RM_SIN[k] + z * ps;
    pc = RM_COS[k] + z * pc;
  }
  const double sr = r + r * z * ps;
  const double cr = 1.0 + z * pc;
  const int q = (int)kf & 3;
  const double a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;  // sin / cos of r + (q&1) pi/2, unsigned
  s = (q == 0 || q == 1) ? a : -a;
  c = (q == 0 || q == 3) ? b : -b;
}

// atan t, t in [0, 1]: two halvings atan t = 2 atan(t / (1 + sqrt(1 + t^2))),
// then the series on [0, tan(pi/16)]
__device__ __forceinline__ double rm_atan01(double t) {
  t = t / (1.0 + sqrt(1.0 + t * t));
  t = t / (1.0 + sqrt(1.0 + t * t));
  const double v = t * t;
  double p = RM_ATAN[11];
#pragma unroll
  for (int k = 10; k >= 0; k--) p = RM_ATAN[k] + v * p;
  return 4.0 * (t + t * v * p);
}

// atan2 with glibc's signed-zero / axis conventions
__device__ __forceinline__ double rm_atan2(double y, double x) {
  if (isnan(x) || isnan(y)) return x + y;
  const double ax = fabs(x), ay = fabs(y);
  double a;
  if (ay == 0.0) {
    a = signbit(x) ? RM_PI_HI : 0.0;
  } else if (ax == 0.0) {
    a = RM_PIO2_HI;
  } else {
    if (ay <= ax)
      a = rm_atan01(ay / ax);
    else
      a = RM_PIO2_HI - (rm_atan01(ax / ay) - RM_PIO2_LO);
    if (signbit(x)) a = RM_PI_HI - (a - RM_PI_LO);
  }
  return copysign(a, y);
}

__device__ __forceinline__ double rm_acos(double c) {
  return rm_atan2(sqrt((1.0 - c) * (1.0 + c)), c);
}

__device__ __forceinline__ void box_muller(double u1, double u2, double &z0, double &z1) {
  const double r = sqrt(-2.0 * rm_log(1.0 - u1));
  const double th = 6.283185307179586 * u2;
  double s, c;
  rm_sincos(th, s, c);
  z0 = r * c;
  z1 = r * s;
}

// v (sin theta cos phi, sin theta sin phi, cos theta), theta = acos(cos_theta)
// (planner_class.cpp:61-73)
__device__ __forceinline__ void speed_vector(double v, double cos_theta, double phi, double *q) {
  const double theta = rm_acos(cos_theta);
  double st, ct, sp, cp;
  rm_sincos(theta, st, ct);
  rm_sincos(phi, sp, cp);
  q[3] = v * st * cp;
  q[4] = v * st * sp;
  q[5] = v * ct;
}

// planning_utils.cpp:198-231 (Eigen cross / norm / I + [v]x + [v]x^2 (1-c)/s^2)
__device__ __forceinline__ void rotate_grf(const double *n, const double *f, double *out) {
  const double v0 = n[1] * 1.0 - n[2] * 0.0;
  const double v1 = n[2] * 0.0 - n[0] * 1.0;
  const double v2 = n[0] * 0.0 - n[1] * 0.0;
  const double s = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  const double c = n[0] * 0.0 + n[1] * 0.0 + n[2] * 1.0;
  if (s < 0.000001) {
    out[0] = f[0]; out[1] = f[1]; out[2] = f[2];
    return;
  }
  const double K[3][3] = {{0, -v2, v1}, {v2, 0, -v0}, {-v1, v0, 0}};
  double R[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      const double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
      R[i][j] = (i == j ? 1.0 : 0.0) + K[i][j] + kk * (1 - c) / (s * s);
    }
#pragma unroll
  for (int i = 0; i < 3; i++) out[i] = R[i][0] * f[0] + R[i][1] * f[1] + R[i][2] * f[2];
}

// planning_utils.cpp:392-442, the reference's rand()/RAND_MAX replaced by
// counter-addressed uniforms (draws 0..4 of (stream_id, index)).
__device__ __forceinline__ void sample_action(const double *nrm, uint64_t seed, uint64_t stream_id,
                                              int64_t index, double *a) {
  double u[10];
#pragma unroll
  for (uint32_t d = 0; d < 5; d++) uniform2(seed, stream_id, PURPOSE_ACTION, index, d, u[2 * d], u[2 * d + 1]);
  const double f_z_td = F_MAX * u[0];
  const double f_z_to = F_MAX * u[1];
  const double f_td[3] = {2 * MU * f_z_td * u[2] - MU * f_z_td, 2 * MU * f_z_td * u[4] - MU * f_z_td,
                          f_z_td};
  const double f_to[3] = {2 * MU * f_z_to * u[3] - MU * f_z_to, 2 * MU * f_z_to * u[5] - MU * f_z_to,
                          f_z_to};
  double r_td[3], r_to[3];
  rotate_grf(nrm, f_td, r_td);
  rotate_grf(nrm, f_to, r_to);
  a[0] = r_td[0] / M_CONST;
  a[1] = r_td[1] / M_CONST;
  a[2] = r_td[2] / M_CONST - G_CONST;
  a[3] = r_to[0] / M_CONST;
  a[4] = r_to[1] / M_CONST;
  a[5] = r_to[2] / M_CONST - G_CONST;
  a[6] = 0.3;
  a[7] = (T_F_MAX - T_F_MIN) * u[6] + T_F_MIN;
  double z0, z1;
  box_muller(u[8], u[9], z0, z1);
  a[8] = std_max(std_min(z0 * (ANG_ACC_MAX / 4.0) + 0.0, ANG_ACC_MAX), -ANG_ACC_MAX);
  a[9] = std_max(std_min(z1 * (ANG_ACC_MAX / 4.0) + 0.0, ANG_ACC_MAX), -ANG_ACC_MAX);
}

// planner_class.cpp:38-76, one try k of index i (draws 4k .. 4k+3)
template <class ZT>
__device__ __forceinline__ void sample_state_try(const TerrainView<ZT> &T, uint64_t seed,
                                                 uint64_t stream_id, int64_t index, int k,
                                                 double *q) {
  const double z_min_rel = H_MIN + ROBOT_H, z_max_rel = H_MAX + ROBOT_H;
  const double mean = 0.5 * (z_max_rel + z_min_rel);
  const double sd = (z_max_rel - z_min_rel) * (1.0 / (2 * 3.0));
  double u00, u01, u10, u11, u20, u21, u30, u31;
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 0, u00, u01);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 1, u10, u11);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 2, u20, u21);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 3, u30, u31);
  double z0, z1;
  box_muller(u10, u11, z0, z1);
  const double hz = z0 * sd + mean;
  q[0] = (T.xN - T.x0) * u00 + T.x0;
  q[1] = (T.yN - T.y0) * u01 + T.y0;
  double g;
  bool near = false;
  if (!height_at(T, q[0], q[1], g, near)) g = __builtin_nan("");
  q[2] = std_max(std_min(hz, z_max_rel), z_min_rel) + g;
  const double phi = (2.0 * MY_PI) * u20;
  const double cos_theta = 2.0 * u21 - 1.0;
  const double v = u30 * V_MAX;
  speed_vector(v, cos_theta, phi, q);
  q[6] = 2 * P_MAX * u31 - P_MAX;
  q[7] = 0.0;
}

// ---- direction-biased sampling (gbp.h gbp_sampling) -----------------------------
// The coin of a draw: the reference's `(double) rand() / RAND_MAX <= threshold`
// (planner_class.cpp:27-29, planning_utils.cpp:381-383) as a uniform of its own
// purpose, so either branch consumes the same counter-addressed draws.
constexpr uint32_t PURPOSE_COIN = 3u;
__device__ __forceinline__ bool coin(uint64_t seed, uint64_t stream_id, int64_t index,
                                     uint32_t draw, double p) {
  double c0, c1;
  uniform2(seed, stream_id, PURPOSE_COIN, index, draw, c0, c1);
  return c0 <= p;
}

// getRandomActionDirection (planning_utils.cpp:443-515): sample_action's draws
// (f_z td/to, f_x td/to, f_y td/to, t_f, the normal pair), each tangential
// force on the side of the velocity change s_from -> s_to: [0, mu f_z] where
// the component grows, else [-mu f_z, 0]
__device__ __forceinline__ void sample_action_direction(const double *nrm, const double *s_from,
                                                        const double *s_to, uint64_t seed,
                                                        uint64_t stream_id, int64_t index,
                                                        double *a) {
  double u[10];
#pragma unroll
  for (uint32_t d = 0; d < 5; d++) uniform2(seed, stream_id, PURPOSE_ACTION, index, d, u[2 * d], u[2 * d + 1]);
  const bool dx_inc = s_to[3] > s_from[3], dy_inc = s_to[4] > s_from[4];
  const double f_z_td = F_MAX * u[0];
  const double f_z_to = F_MAX * u[1];
  const double ff_td = MU * f_z_td, ff_to = MU * f_z_to;
  const double f_x_td = dx_inc ? ff_td * u[2] : ff_td * u[2] - ff_td;
  const double f_x_to = dx_inc ? ff_to * u[3] : ff_to * u[3] - ff_to;
  const double f_y_td = dy_inc ? ff_td * u[4] : ff_td * u[4] - ff_td;
  const double f_y_to = dy_inc ? ff_to * u[5] : ff_to * u[5] - ff_to;
  const double f_td[3] = {f_x_td, f_y_td, f_z_td}, f_to[3] = {f_x_to, f_y_to, f_z_to};
  double r_td[3], r_to[3];
  rotate_grf(nrm, f_td, r_td);
  rotate_grf(nrm, f_to, r_to);
  a[0] = r_td[0] / M_CONST;
  a[1] = r_td[1] / M_CONST;
  a[2] = r_td[2] / M_CONST - G_CONST;
  a[3] = r_to[0] / M_CONST;
  a[4] = r_to[1] / M_CONST;
  a[5] = r_to[2] / M_CONST - G_CONST;
  a[6] = 0.3;
  a[7] = (T_F_MAX - T_F_MIN) * u[6] + T_F_MIN;
  double z0, z1;
  box_muller(u[8], u[9], z0, z1);
  a[8] = std_max(std_min(z0 * (ANG_ACC_MAX / 4.0) + 0.0, ANG_ACC_MAX), -ANG_ACC_MAX);
  a[9] = std_max(std_min(z1 * (ANG_ACC_MAX / 4.0) + 0.0, ANG_ACC_MAX), -ANG_ACC_MAX);
}

// getRandomAction(surf_norm, direction, flag, p, s, s_near) (planning_utils.cpp:379-391)
__device__ __forceinline__ void sample_action_cfg(const double *nrm, const gbp_sampling &cfg,
                                                  int direction, const double *s,
                                                  const double *s_near, uint64_t seed,
                                                  uint64_t stream_id, int64_t index, double *a) {
  if (cfg.action_flag && coin(seed, stream_id, index, 0, cfg.action_p)) {
    if (direction == GBP_FORWARD)
      sample_action_direction(nrm, s_near, s, seed, stream_id, index, a);
    else
      sample_action_direction(nrm, s, s_near, seed, stream_id, index, a);
    return;
  }
  sample_action(nrm, seed, stream_id, index, a);
}

// PlannerClass::randomStateDirection (planner_class.cpp:82-148), try k of
// index i: sample_state_try's draws, x and y over the rectangle spanned by
// s_from and s_to, the heading atan2(to - from) when speed_direction
template <class ZT>
__device__ __forceinline__ void sample_state_direction_try(const TerrainView<ZT> &T,
                                                           const double *s_from, const double *s_to,
                                                           int speed_direction, uint64_t seed,
                                                           uint64_t stream_id, int64_t index, int k,
                                                           double *q) {
  const double x_min = std_min(s_from[0], s_to[0]), x_max = std_max(s_from[0], s_to[0]);
  const double y_min = std_min(s_from[1], s_to[1]), y_max = std_max(s_from[1], s_to[1]);
  const double z_min_rel = H_MIN + ROBOT_H, z_max_rel = H_MAX + ROBOT_H;
  const double mean = 0.5 * (z_max_rel + z_min_rel);
  const double sd = (z_max_rel - z_min_rel) * (1.0 / (2 * 3.0));
  double u00, u01, u10, u11, u20, u21, u30, u31;
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 0, u00, u01);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 1, u10, u11);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 2, u20, u21);
  uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 3, u30, u31);
  double z0, z1;
  box_muller(u10, u11, z0, z1);
  const double hz = z0 * sd + mean;
  q[0] = (x_max - x_min) * u00 + x_min;
  q[1] = (y_max - y_min) * u01 + y_min;
  double g;
  bool near = false;
  if (!height_at(T, q[0], q[1], g, near)) g = __builtin_nan("");
  q[2] = std_max(std_min(hz, z_max_rel), z_min_rel) + g;
  const double phi = speed_direction ? rm_atan2(s_to[1] - s_from[1], s_to[0] - s_from[0])
                                     : (2.0 * MY_PI) * u20;
  const double cos_theta = 2.0 * u21 - 1.0;
  const double v = u30 * V_MAX;
  speed_vector(v, cos_theta, phi, q);
  q[6] = 2 * P_MAX * u31 - P_MAX;
  q[7] = 0.0;
}

// PlannerClass::randomState(terrain, flag, p, speed_direction_flag, s_from, s_to)
// (planner_class.cpp:22-35), try k: the coin is draw k of its purpose
template <class ZT>
__device__ __forceinline__ void sample_state_cfg_try(const TerrainView<ZT> &T, const gbp_sampling &cfg,
                                                     const double *s_from, const double *s_to,
                                                     uint64_t seed, uint64_t stream_id,
                                                     int64_t index, int k, double *q) {
  if (cfg.state_flag && coin(seed, stream_id, index, (uint32_t)k, cfg.state_p))
    sample_state_direction_try(T, s_from, s_to, cfg.state_speed_direction, seed, stream_id, index,
                               k, q);
  else
    sample_state_try(T, seed, stream_id, index, k, q);
}

}  // namespace gbp
