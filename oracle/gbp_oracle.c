/*
 * gbp_oracle.c — CPU restatement of the global_body_planner hot path.
 * TEST INFRASTRUCTURE ONLY (see gbp_oracle.h).  Every function cites the
 * reference file:line it restates; expressions keep the reference's
 * left-to-right evaluation order and are compiled with -ffp-contract=off.
 */
#include "gbp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- constants: include/global_body_planner/planning_utils.h:21-66 ------ */
#define H_MAX 0.4
#define H_MIN 0.075
#define V_MAX 2.0
#define V_NOM 0.75
#define P_MAX 1.0
#define ANG_ACC_MAX 7.0
#define ROBOT_L 0.3
#define ROBOT_W 0.3
#define ROBOT_H 0.05
#define M_CONST 13.0
#define G_CONST 9.81
#define F_MAX 637.0
#define MU 1.0
#define T_F_MAX 0.5
#define T_F_MIN 0.0
#define KINEMATICS_RES 0.05
#define BACKUP_RATIO 0.5
#define NUM_GEN_STATES 6
#define GOAL_BOUNDS 0.5
#define MY_PI 3.14159
#define FRAGILE_EPS 1e-12

#define PURPOSE_STATE 1u
#define PURPOSE_ACTION 2u

/* std::min / std::max semantics (NaN behaviour included) */
static inline double std_min(double a, double b) { return (b < a) ? b : a; }
static inline double std_max(double a, double b) { return (a < b) ? b : a; }

static int g_scan_mode = 0;
void orc_set_scan_mode(int mode) { g_scan_mode = mode; }
int orc_get_scan_mode(void) { return g_scan_mode; }

/* ---- bracket search: fast_terrain_map.cpp:101-117 ----------------------
 * The reference scans i < size for d[i] <= v && v < d[i+1] (first match) and
 * leaves the index at its default 0 when nothing matches.  Outcomes:
 *   i >= 0          a bracket;
 *   BR_LOW  (-1)    v is NaN or v < d[0]: no match, and the short-circuit of
 *                   `d[i] <= v` never reads d[size]: well defined, index 0
 *                   (heightIsNan then tests cell 0; getGroundHeight's x1/x2
 *                   stay uninitialised -> UB unless v is NaN, which makes the
 *                   height NaN whatever they hold);
 *   BR_HIGH (-2)    v >= d[size-1]: the last step reads d[size] -> UB. */
#define BR_LOW (-1)
#define BR_HIGH (-2)
static int bracket(const double *d, int n, double v) {
  if (g_scan_mode == 0) {
    for (int i = 0; i < n - 1; i++)
      if (d[i] <= v && v < d[i + 1]) return i;
  } else if (d[0] <= v && v < d[n - 1]) {
    int lo = 0, hi = n - 1; /* d[lo] <= v < d[hi] */
    while (hi - lo > 1) {
      int mid = lo + (hi - lo) / 2;
      if (d[mid] <= v) lo = mid; else hi = mid;
    }
    return lo;
  }
  return (d[n - 1] <= v) ? BR_HIGH : BR_LOW;
}

/* bilinear blend, fast_terrain_map.cpp:120-126 (same expression for :191-211) */
static double bilinear(const double *f, int ny, int ix, int iy, double x1, double x2,
                       double y1, double y2, double x, double y) {
  double fx1y1 = f[(long)ix * ny + iy];
  double fx1y2 = f[(long)ix * ny + iy + 1];
  double fx2y1 = f[(long)(ix + 1) * ny + iy];
  double fx2y2 = f[(long)(ix + 1) * ny + iy + 1];
  return 1.0 / ((x2 - x1) * (y2 - y1)) *
         (fx1y1 * (x2 - x) * (y2 - y) + fx2y1 * (x - x1) * (y2 - y) +
          fx1y2 * (x2 - x) * (y - y1) + fx2y2 * (x - x1) * (y - y1));
}

/* fast_terrain_map.cpp:94-132.  NaN coordinate -> NaN (deterministic);
 * any other missing bracket -> *ood = 1 (UB), NaN returned. */
double orc_ground_height(const orc_terrain *T, double x, double y, int *ood) {
  int ix = bracket(T->x, T->nx, x), iy = bracket(T->y, T->ny, y);
  if (ood) *ood = 0;
  if (isnan(x) || isnan(y)) return NAN;
  if (ix < 0 || iy < 0) { if (ood) *ood = 1; return NAN; }
  return bilinear(T->z, T->ny, ix, iy, T->x[ix], T->x[ix + 1], T->y[iy], T->y[iy + 1], x, y);
}

static int cell_has_nan(const orc_terrain *T, int ix, int iy) {
  const double *z = T->z;
  long ny = T->ny;
  return isnan(z[ix * ny + iy]) || isnan(z[ix * ny + iy + 1]) || isnan(z[(ix + 1) * ny + iy]) ||
         isnan(z[(ix + 1) * ny + iy + 1]);
}

/* fast_terrain_map.cpp:135-157.  BR_HIGH on either axis -> *ood = 1 (UB),
 * returns 1; BR_LOW -> index 0 on that axis (the reference default). */
int orc_height_is_nan(const orc_terrain *T, double x, double y, int *ood) {
  int ix = bracket(T->x, T->nx, x), iy = bracket(T->y, T->ny, y);
  if (ood) *ood = 0;
  if (ix == BR_HIGH || iy == BR_HIGH) { if (ood) *ood = 1; return 1; }
  return cell_has_nan(T, ix < 0 ? 0 : ix, iy < 0 ? 0 : iy);
}

/* fast_terrain_map.cpp:160-213 (same bracket rules as getGroundHeight) */
void orc_surface_normal(const orc_terrain *T, double x, double y, double n[3], int *ood) {
  int ix = bracket(T->x, T->nx, x), iy = bracket(T->y, T->ny, y);
  if (ood) *ood = 0;
  if (isnan(x) || isnan(y) || ix < 0 || iy < 0) {
    if (ood && !(isnan(x) || isnan(y))) *ood = 1;
    n[0] = n[1] = n[2] = NAN;
    return;
  }
  if (!T->dx) { n[0] = 0.0; n[1] = 0.0; n[2] = 1.0; return; }
  double x1 = T->x[ix], x2 = T->x[ix + 1], y1 = T->y[iy], y2 = T->y[iy + 1];
  n[0] = bilinear(T->dx, T->ny, ix, iy, x1, x2, y1, y2, x, y);
  n[1] = bilinear(T->dy, T->ny, ix, iy, x1, x2, y1, y2, x, y);
  n[2] = bilinear(T->dz, T->ny, ix, iy, x1, x2, y1, y2, x, y);
}

/* ---- propagation -------------------------------------------------------- */
/* planning_utils.cpp:237-274 */
void orc_apply_stance(const double *s, const double *a, double t, double *o) {
  double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  double x_td = s[0], y_td = s[1], z_td = s[2], dx_td = s[3], dy_td = s[4], dz_td = s[5];
  double p_td = s[6], dp_td = s[7];
  double r[8];
  r[0] = x_td + dx_td * t + 0.5 * a_x_td * t * t + (a_x_to - a_x_td) * (t * t * t) / (6.0 * t_s);
  r[1] = y_td + dy_td * t + 0.5 * a_y_td * t * t + (a_y_to - a_y_td) * (t * t * t) / (6.0 * t_s);
  r[2] = z_td + dz_td * t + 0.5 * a_z_td * t * t + (a_z_to - a_z_td) * (t * t * t) / (6.0 * t_s);
  r[3] = dx_td + a_x_td * t + (a_x_to - a_x_td) * t * t / (2.0 * t_s);
  r[4] = dy_td + a_y_td * t + (a_y_to - a_y_td) * t * t / (2.0 * t_s);
  r[5] = dz_td + a_z_td * t + (a_z_to - a_z_td) * t * t / (2.0 * t_s);
  r[6] = p_td + dp_td * t + 0.5 * a_p_td * t * t + (a_p_to - a_p_td) * (t * t * t) / (6.0 * t_s);
  r[7] = dp_td + a_p_td * t + (a_p_to - a_p_td) * t * t / (2.0 * t_s);
  memcpy(o, r, sizeof r);
}

/* planning_utils.cpp:282-306 (g is the literal 9.81, :283) */
void orc_apply_flight(const double *s, double t_f, double *o) {
  double g = 9.81;
  double r[8];
  r[0] = s[0] + s[3] * t_f;
  r[1] = s[1] + s[4] * t_f;
  r[2] = s[2] + s[5] * t_f - 0.5 * g * t_f * t_f;
  r[3] = s[3];
  r[4] = s[4];
  r[5] = s[5] - g * t_f;
  r[6] = s[6] + s[7] * t_f;
  r[7] = s[7];
  memcpy(o, r, sizeof r);
}

/* planning_utils.cpp:324-367 */
void orc_apply_stance_reverse(const double *s, const double *a, double t, double *o) {
  double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  double x_to = s[0], y_to = s[1], z_to = s[2], dx_to = s[3], dy_to = s[4], dz_to = s[5];
  double p_to = s[6], dp_to = s[7];
  double cx = dx_to - a_x_td * t_s - 0.5 * (a_x_to - a_x_td) * t_s;
  double cy = dy_to - a_y_td * t_s - 0.5 * (a_y_to - a_y_td) * t_s;
  double cz = dz_to - a_z_td * t_s - 0.5 * (a_z_to - a_z_td) * t_s;
  double cp = dp_to - a_p_td * t_s - 0.5 * (a_p_to - a_p_td) * t_s;
  double r[8];
  r[0] = x_to - cx * (t_s - t) - 0.5 * a_x_td * (t_s * t_s - t * t) -
         (a_x_to - a_x_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[1] = y_to - cy * (t_s - t) - 0.5 * a_y_td * (t_s * t_s - t * t) -
         (a_y_to - a_y_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[2] = z_to - cz * (t_s - t) - 0.5 * a_z_td * (t_s * t_s - t * t) -
         (a_z_to - a_z_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[3] = dx_to - a_x_td * (t_s - t) - (a_x_to - a_x_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[4] = dy_to - a_y_td * (t_s - t) - (a_y_to - a_y_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[5] = dz_to - a_z_td * (t_s - t) - (a_z_to - a_z_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[7] = dp_to - a_p_td * (t_s - t) - (a_p_to - a_p_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[6] = p_to - cp * (t_s - t) - 0.5 * a_p_td * (t_s * t_s - t * t) -
         (a_p_to - a_p_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  memcpy(o, r, sizeof r);
}

/* planning_utils.cpp:519-556 */
int orc_is_valid_action(const double *a) {
  if ((a[6] <= 0) || (a[7] < 0)) return 0;
  double m = M_CONST, g = G_CONST, mu = MU;
  double f_x_td = m * a[0], f_y_td = m * a[1], f_z_td = m * (a[2] + g);
  double f_x_to = m * a[3], f_y_to = m * a[4], f_z_to = m * (a[5] + g);
  double a_p_td = a[8], a_p_to = a[9];
  if ((sqrt(f_x_td * f_x_td + f_y_td * f_y_td + f_z_td * f_z_td) >= F_MAX) ||
      (sqrt(f_x_to * f_x_to + f_y_to * f_y_to + f_z_to * f_z_to) >= F_MAX) || (f_z_td < 0) ||
      (f_z_to < 0) || (a_p_td >= F_MAX) || (a_p_to >= F_MAX))
    return 0;
  if ((sqrt(f_x_td * f_x_td + f_y_td * f_y_td) >= mu * f_z_td) ||
      (sqrt(f_x_to * f_x_to + f_y_to * f_y_to) >= mu * f_z_to))
    return 0;
  return 1;
}

/* Does a trig-dependent lookup coordinate sit within FRAGILE_EPS of a line
 * bounding its cell, so that a last-ulp trig difference could move it into
 * another cell (another height, another heightIsNan cell: NaN <-> finite) or
 * across the map edge (defined <-> OOD)?  The cell of a point with no bracket
 * is the one at the edge it lies beyond: 0 below d[0] (the cell the
 * reference's heightIsNan tests), n-2 at or above d[n-1]. */
static int near_cell_line(const double *d, int n, int i, double v) {
  int c = i >= 0 ? i : (i == BR_HIGH ? n - 2 : 0);
  return fabs(v - d[c]) < FRAGILE_EPS || fabs(d[c + 1] - v) < FRAGILE_EPS;
}

static int near_point(const orc_terrain *T, double x, double y) {
  if (isnan(x) || isnan(y)) return 0; /* NaN heights whatever the trig */
  return near_cell_line(T->x, T->nx, bracket(T->x, T->nx, x), x) ||
         near_cell_line(T->y, T->ny, bracket(T->y, T->ny, y), y);
}

static double cell_height(const orc_terrain *T, int ix, int iy, double x, double y) {
  return bilinear(T->z, T->ny, ix, iy, T->x[ix], T->x[ix + 1], T->y[iy], T->y[iy + 1], x, y);
}

/* getGroundHeight inside isValidState: 0 = UB (no bracket, finite coords),
 * 1 = value in *h (NaN for NaN coordinates) */
static int height_at(const orc_terrain *T, double x, double y, double *h, orc_stats *st) {
  if (isnan(x) || isnan(y)) { *h = NAN; return 1; }
  if (near_point(T, x, y)) st->flags |= GBP_F_FRAGILE;
  int ix = bracket(T->x, T->nx, x), iy = bracket(T->y, T->ny, y);
  if (ix < 0 || iy < 0) return 0;
  *h = cell_height(T, ix, iy, x, y);
  return 1;
}

/* heightIsNan inside isValidState: -1 = UB, else the reference's bool */
static int nan_at(const orc_terrain *T, double x, double y) {
  int ix = bracket(T->x, T->nx, x), iy = bracket(T->y, T->ny, y);
  if (ix == BR_HIGH || iy == BR_HIGH) return -1;
  return cell_has_nan(T, ix < 0 ? 0 : ix, iy < 0 ? 0 : iy);
}

/* planning_utils.cpp:562-635.  Out-of-domain convention: where
 * the reference's result depends on an undefined read (a lookup point with
 * no bracket and finite coordinates), the state is invalid and GBP_F_OOD is
 * set when that UB could change the decision.  Every well-defined case
 * (NaN coordinates, points below the first coordinate in heightIsNan) is
 * restated exactly. */
int orc_is_valid_state(const orc_terrain *T, const double *s, int phase, orc_stats *st) {
  if (st->V >= GBP_MAX_SAMPLES) { st->flags |= GBP_F_LIMIT; return 0; } /* engine guard */
  st->V++;
  const double x0 = T->x[0], xN = T->x[T->nx - 1], y0 = T->y[0], yN = T->y[T->ny - 1];
  /* (1) heightIsNan(centre) :564 */
  int r = nan_at(T, s[0], s[1]);
  if (r < 0) {
    /* x or y >= the last coordinate: rejected by (2) unless exactly equal */
    int in_closed = !(s[0] < x0 || s[0] > xN || s[1] < y0 || s[1] > yN);
    if (in_closed) st->flags |= GBP_F_OOD;
    return 0;
  }
  if (r) { st->flags |= GBP_F_NAN; return 0; }
  /* (2) bounds + pitch :568-571 (abs() resolves to the double overload) */
  if ((s[0] < x0) || (s[0] > xN) || (s[1] < y0) || (s[1] > yN) || (fabs(s[6]) >= P_MAX)) return 0;
  /* (3) horizontal speed :574 */
  if (sqrt(s[3] * s[3] + s[4] * s[4]) > V_MAX) return 0;
  /* (4) rotation :578-594 */
  double yaw = atan2(s[4], s[3]);
  double cy = cos(yaw), sy = sin(yaw);
  double pitch = s[6];
  double cp = cos(pitch), sp = sin(pitch);
  double R_11 = cy * cp, R_12 = -sy, R_13 = cy * sp;
  double R_21 = sy * cp, R_22 = cy, R_23 = sy * sp;
  double R_31 = -sp, R_32 = 0, R_33 = cp;
  const double test_x[2] = {-0.5 * ROBOT_L, 0.5 * ROBOT_L};
  const double test_y[2] = {-0.5 * ROBOT_W, 0.5 * ROBOT_W};
  double z_body = -ROBOT_H;
  /* (5) four corners :601-627 */
  for (int bx = 0; bx < 2; bx++) {
    for (int by = 0; by < 2; by++) {
      double x_body = test_x[bx], y_body = test_y[by];
      double x_leg = s[0] + R_11 * x_body + R_12 * y_body;
      double y_leg = s[1] + R_21 * x_body + R_22 * y_body;
      double z_leg = s[2] + R_31 * x_body + R_32 * y_body;
      double x_corner = x_leg + R_13 * z_body;
      double y_corner = y_leg + R_23 * z_body;
      double z_corner = z_leg + R_33 * z_body;
      /* heightIsNan(leg) :614; FRAGILE from here on when the leg is near a
       * line bounding its cell (NaN-cell boundaries and the map edge too) */
      if (near_point(T, x_leg, y_leg)) st->flags |= GBP_F_FRAGILE;
      int rl = nan_at(T, x_leg, y_leg);
      if (rl < 0) { st->flags |= GBP_F_OOD; return 0; }
      if (rl) { st->flags |= GBP_F_NAN; return 0; }
      /* both heights before the test :618-619 */
      st->G += 2;
      double gl, gc;
      if (!height_at(T, x_leg, y_leg, &gl, st)) { st->flags |= GBP_F_OOD; return 0; }
      if (!height_at(T, x_corner, y_corner, &gc, st)) { st->flags |= GBP_F_OOD; return 0; }
      double leg_height = z_leg - gl;
      double corner_height = z_corner - gc;
      if (fabs(corner_height - H_MIN) < FRAGILE_EPS ||
          (phase == GBP_STANCE && fabs(leg_height - H_MAX) < FRAGILE_EPS))
        st->flags |= GBP_F_FRAGILE;
      /* :624 */
      if ((corner_height < H_MIN) || ((phase == GBP_STANCE) && (leg_height > H_MAX))) return 0;
    }
  }
  /* (6) underside centre :630-632 */
  st->G++;
  double gu;
  if (!height_at(T, s[0] + R_13 * z_body, s[1] + R_23 * z_body, &gu, st)) {
    st->flags |= GBP_F_OOD;
    return 0;
  }
  double height = (s[2] + R_33 * z_body) - gu;
  if (fabs(height - H_MIN) < FRAGILE_EPS) st->flags |= GBP_F_FRAGILE;
  if (height < H_MIN) return 0;
  return 1;
}

#define STAGE(f, k) ((f) = ((f) & ~GBP_F_STAGE_MASK) | ((uint32_t)(k) << GBP_F_STAGE_SHIFT))

/* planning_utils.cpp:713-753 */
static int pair_fwd(const orc_terrain *T, const double *s, const double *a, double *s_new,
                    double *t_new, orc_stats *st, uint32_t *f) {
  double t_s = a[6], t_f = a[7], sc[8];
  STAGE(*f, GBP_STAGE_FWD_STANCE);
  for (double t = 0; t <= t_s; t += KINEMATICS_RES) {
    orc_apply_stance(s, a, t, sc);
    if (orc_is_valid_state(T, sc, GBP_STANCE, st) == 0) {
      if (st->flags & GBP_F_LIMIT) return 0;
      orc_apply_stance(s, a, (1.0 - BACKUP_RATIO) * t, s_new);
      *f |= GBP_F_SNEW_SET;
      return 0;
    }
    memcpy(s_new, sc, sizeof sc);
    *t_new = t;
    *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  }
  double s_takeoff[8];
  orc_apply_stance(s, a, a[6], s_takeoff);
  STAGE(*f, GBP_STAGE_FWD_FLIGHT);
  for (double t = 0; t < t_f; t += KINEMATICS_RES) {
    orc_apply_flight(s_takeoff, t, sc);
    if (orc_is_valid_state(T, sc, GBP_FLIGHT, st) == 0) return 0;
  }
  STAGE(*f, GBP_STAGE_FWD_LAND);
  double s_land[8];
  orc_apply_flight(s_takeoff, t_f, s_land);
  if (orc_is_valid_state(T, s_land, GBP_STANCE, st) == 0) return 0;
  memcpy(s_new, s_land, sizeof s_land);
  *t_new = t_s + t_f;
  *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return 1;
}

/* planning_utils.cpp:651-712 */
static int pair_fwd_adaptive(const orc_terrain *T, const double *s, const double *a,
                             double *s_new, double *t_new, orc_stats *st, uint32_t *f) {
  double t_s = a[6], t_f = a[7], sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  STAGE(*f, GBP_STAGE_FWD_STANCE);
  for (double t = 0; t <= t_s; t += time_step) {
    orc_apply_stance(s, a, t, sc);
    if (orc_is_valid_state(T, sc, GBP_STANCE, st) == 0) {
      if (st->flags & GBP_F_LIMIT) return 0;
      if (KINEMATICS_RES - 0.01 <= time_step && time_step <= KINEMATICS_RES + 0.01) {
        orc_apply_stance(s, a, (1.0 - BACKUP_RATIO) * t, s_new);
        *f |= GBP_F_SNEW_SET;
        return 0;
      } else {
        time_step = KINEMATICS_RES;
        t = t_pre_success;
      }
    } else {
      memcpy(s_new, sc, sizeof sc);
      *t_new = t;
      *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      time_step += KINEMATICS_RES;
      t_pre_success = t;
    }
  }
  double s_takeoff[8];
  orc_apply_stance(s, a, a[6], s_takeoff);
  time_step = KINEMATICS_RES;
  t_pre_success = 0;
  STAGE(*f, GBP_STAGE_FWD_FLIGHT);
  for (double t = 0; t < t_f; t += time_step) {
    orc_apply_flight(s_takeoff, t, sc);
    if (orc_is_valid_state(T, sc, GBP_FLIGHT, st) == 0) return 0;
    time_step += KINEMATICS_RES;
    t_pre_success = t;
  }
  (void)t_pre_success;
  STAGE(*f, GBP_STAGE_FWD_LAND);
  double s_land[8];
  orc_apply_flight(s_takeoff, t_f, s_land);
  if (orc_is_valid_state(T, s_land, GBP_STANCE, st) == 0) return 0;
  memcpy(s_new, s_land, sizeof s_land);
  *t_new = t_s + t_f;
  *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return 1;
}

/* planning_utils.cpp:837-876 */
static int pair_rev(const orc_terrain *T, const double *s, const double *a, double *s_new,
                    double *t_new, orc_stats *st, uint32_t *f) {
  double t_s = a[6], t_f = a[7], sc[8];
  STAGE(*f, GBP_STAGE_REV_FLIGHT);
  for (double t = 0; t < t_f; t += KINEMATICS_RES) {
    orc_apply_flight(s, -t, sc);
    if (orc_is_valid_state(T, sc, GBP_FLIGHT, st) == 0) return 0;
  }
  double s_takeoff[8];
  orc_apply_flight(s, -t_f, s_takeoff);
  STAGE(*f, GBP_STAGE_REV_STANCE);
  for (double t = t_s; t >= 0; t -= KINEMATICS_RES) {
    orc_apply_stance_reverse(s_takeoff, a, t, sc);
    if (orc_is_valid_state(T, sc, GBP_STANCE, st) == 0) {
      if (st->flags & GBP_F_LIMIT) return 0;
      /* a FORWARD stance applied to the end state, as written (:857) */
      orc_apply_stance(s, a, t + BACKUP_RATIO * (t_s - t), s_new);
      *f |= GBP_F_SNEW_SET;
      return 0;
    }
    memcpy(s_new, sc, sizeof sc);
    *t_new = t_s - t;
    *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  }
  STAGE(*f, GBP_STAGE_REV_START);
  double s_start[8];
  orc_apply_stance_reverse(s_takeoff, a, 0, s_start);
  if (orc_is_valid_state(T, s_start, GBP_STANCE, st) == 0) return 0;
  memcpy(s_new, s_start, sizeof s_start);
  *t_new = t_s;
  *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return 1;
}

/* planning_utils.cpp:774-836 */
static int pair_rev_adaptive(const orc_terrain *T, const double *s, const double *a,
                             double *s_new, double *t_new, orc_stats *st, uint32_t *f) {
  double t_s = a[6], t_f = a[7], sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  STAGE(*f, GBP_STAGE_REV_FLIGHT);
  for (double t = 0; t < t_f; t += time_step) {
    orc_apply_flight(s, -t, sc);
    if (orc_is_valid_state(T, sc, GBP_FLIGHT, st) == 0) return 0;
    time_step += KINEMATICS_RES;
    t_pre_success = t;
  }
  double s_takeoff[8];
  orc_apply_flight(s, -t_f, s_takeoff);
  time_step = KINEMATICS_RES;
  t_pre_success = 0;
  STAGE(*f, GBP_STAGE_REV_STANCE);
  for (double t = t_s; t >= 0; t -= time_step) {
    orc_apply_stance_reverse(s_takeoff, a, t, sc);
    if (orc_is_valid_state(T, sc, GBP_STANCE, st) == 0) {
      if (st->flags & GBP_F_LIMIT) return 0;
      if (KINEMATICS_RES - 0.01 <= time_step && time_step <= KINEMATICS_RES + 0.01) {
        orc_apply_stance(s, a, t + BACKUP_RATIO * (t_s - t), s_new);
        *f |= GBP_F_SNEW_SET;
        return 0;
      } else {
        time_step = KINEMATICS_RES;
        t = t_pre_success;
      }
    } else {
      memcpy(s_new, sc, sizeof sc);
      *t_new = t_s - t;
      *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      time_step += KINEMATICS_RES;
      t_pre_success = t;
    }
  }
  STAGE(*f, GBP_STAGE_REV_START);
  double s_start[8];
  orc_apply_stance_reverse(s_takeoff, a, 0, s_start);
  if (orc_is_valid_state(T, s_start, GBP_STANCE, st) == 0) return 0;
  memcpy(s_new, s_start, sizeof s_start);
  *t_new = t_s;
  *f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return 1;
}

int orc_is_valid_pair(const orc_terrain *T, const double *s, const double *a, int direction,
                      int adaptive, double *s_new, double *t_new, uint32_t *flags,
                      uint32_t *counts) {
  orc_stats st = {0, 0, 0};
  uint32_t f = 0;
  int v;
  if (direction == GBP_FORWARD)
    v = adaptive ? pair_fwd_adaptive(T, s, a, s_new, t_new, &st, &f)
                 : pair_fwd(T, s, a, s_new, t_new, &st, &f);
  else
    v = adaptive ? pair_rev_adaptive(T, s, a, s_new, t_new, &st, &f)
                 : pair_rev(T, s, a, s_new, t_new, &st, &f);
  f |= st.flags | (v ? GBP_F_VALID : 0u);
  if (flags) *flags = f;
  if (counts) *counts = (st.G & 0xFFFFu) | (st.V << 16);
  return v;
}

/* ---- distances: planning_utils.cpp:106-132, planning_utils.h:133-145 ---- */
double orc_pose_distance(const double *q1, const double *q2) {
  double sum = 0;
  for (int i = 0; i < 3; i++) sum = sum + (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return sqrt(sum);
}

double orc_state_distance(const double *q1, const double *q2) {
  double sum = 0;
  for (int i = 0; i < 8; i++) sum = sum + 1.0 * (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return sqrt(sum);
}

double orc_state_yaw_distance(const double *q1, const double *q2) {
  double yaw1 = atan2(q1[4], q1[3]);
  double yaw2 = atan2(q2[4], q2[3]);
  double yaw_min = std_min(yaw1, yaw2);
  double yaw_max = std_max(yaw1, yaw2);
  return std_min(yaw_max - yaw_min, yaw_min + 2 * MY_PI - yaw_max);
}

/* planner_class.cpp:185-200 */
int orc_nearest(const double *verts, int n_vert, const double *q, double *dist) {
  int nearest = 0;
  double best = INFINITY;
  for (int v = 0; v < n_vert; v++) {
    double c = orc_state_distance(q, verts + (long)v * 8);
    if (c < best) { best = c; nearest = v; }
  }
  if (dist) *dist = best;
  return nearest;
}

/* rrt.cpp:20-70 + :84-101 */
int orc_extend(const orc_terrain *T, const double *s_near, const double *target,
               const double *actions, int direction, int adaptive, double *s_new,
               double *a_new, int *chosen, uint32_t *counts) {
  double best_so_far = orc_state_distance(s_near, target);
  uint32_t G = 0, V = 0;
  double s_test[8];
  double t_new;
  int found = -1;
  for (int j = 0; j < NUM_GEN_STATES; ++j) {
    uint32_t f, c;
    int v = orc_is_valid_pair(T, s_near, actions + 10 * j, direction, adaptive, s_test, &t_new,
                              &f, &c);
    G += GBP_COUNT_G(c);
    V += GBP_COUNT_V(c);
    if (v) { found = j; break; }
  }
  if (counts) *counts = (G & 0xFFFFu) | (V << 16);
  if (chosen) *chosen = found;
  if (found >= 0) {
    double current_dist = orc_state_distance(s_test, target);
    if (current_dist < best_so_far) {
      best_so_far = current_dist;
      memcpy(s_new, s_test, sizeof s_test);
      memcpy(a_new, actions + 10 * found, 10 * sizeof(double));
    }
  }
  if (best_so_far == orc_state_distance(s_near, target)) return GBP_TRAPPED;
  return (orc_state_distance(s_new, target) <= GOAL_BOUNDS) ? GBP_REACHED : GBP_ADVANCED;
}

/* rrt_connect.cpp:53-63: the cubic-Hermite stance action from s_start to
 * s_goal in t_s (t_f = 0) */
static void connect_action(const double *s_start, const double *s_goal, double t_s, double *a) {
  double x_td = s_start[0], y_td = s_start[1], z_td = s_start[2];
  double dx_td = s_start[3], dy_td = s_start[4], dz_td = s_start[5];
  double x_to = s_goal[0], y_to = s_goal[1], z_to = s_goal[2];
  double dx_to = s_goal[3], dy_to = s_goal[4], dz_to = s_goal[5];
  double p_td = s_start[6], dp_td = s_start[7], p_to = s_goal[6], dp_to = s_goal[7];
  a[0] = -(2.0 * (3.0 * x_td - 3.0 * x_to + 2.0 * dx_td * t_s + dx_to * t_s)) / (t_s * t_s);
  a[1] = -(2.0 * (3.0 * y_td - 3.0 * y_to + 2.0 * dy_td * t_s + dy_to * t_s)) / (t_s * t_s);
  a[2] = -(2.0 * (3.0 * z_td - 3.0 * z_to + 2.0 * dz_td * t_s + dz_to * t_s)) / (t_s * t_s);
  a[3] = (2.0 * (3.0 * x_td - 3.0 * x_to + dx_td * t_s + 2.0 * dx_to * t_s)) / (t_s * t_s);
  a[4] = (2.0 * (3.0 * y_td - 3.0 * y_to + dy_td * t_s + 2.0 * dy_to * t_s)) / (t_s * t_s);
  a[5] = (2.0 * (3.0 * z_td - 3.0 * z_to + dz_td * t_s + 2.0 * dz_to * t_s)) / (t_s * t_s);
  a[6] = t_s;
  a[7] = 0;
  a[8] = -(2.0 * (3.0 * p_td - 3.0 * p_to + 2.0 * dp_td * t_s + dp_to * t_s)) / (t_s * t_s);
  a[9] = (2.0 * (3.0 * p_td - 3.0 * p_to + dp_td * t_s + 2.0 * dp_to * t_s)) / (t_s * t_s);
}

/* rrt_connect.cpp:20-84 (recursive attemptConnect) */
typedef struct {
  int capped;     /* the recursion reached GBP_CONNECT_MAX_DEPTH */
  int64_t checks; /* pair checks run (the engine's attempts_checked) */
} ac_stats;

static int attempt_connect_ts(const orc_terrain *T, const double *s_existing, const double *s,
                              double t_s, double *s_new, double *a_new, int direction,
                              int adaptive, int depth, ac_stats *acs) {
  /* engine convention (gbp.h GBP_CONNECT_MAX_DEPTH): the reference recursion
   * is unbounded; levels 0 .. MAX are evaluated, a connection still open then
   * is TRAPPED (and counted) */
  if (depth > GBP_CONNECT_MAX_DEPTH) {
    if (acs) acs->capped = 1;
    return GBP_TRAPPED;
  }
  if (t_s <= KINEMATICS_RES) return GBP_TRAPPED;
  const double *s_start = (direction == GBP_FORWARD) ? s_existing : s;
  const double *s_goal = (direction == GBP_FORWARD) ? s : s_existing;
  double t_new = NAN; /* reference: uninitialised */
  double a[10];
  connect_action(s_start, s_goal, t_s, a);
  memcpy(a_new, a, sizeof a);
  if (orc_is_valid_action(a_new)) {
    uint32_t f;
    if (acs) acs->checks++;
    int ok = (direction == GBP_FORWARD)
                 ? orc_is_valid_pair(T, s_start, a_new, GBP_FORWARD, adaptive, s_new, &t_new, &f, 0)
                 : orc_is_valid_pair(T, s_goal, a_new, GBP_REVERSE, adaptive, s_new, &t_new, &f, 0);
    if (ok) return GBP_REACHED;
    /* The reference recurses with t_new / s_new even when the failed check
     * never assigned them (uninitialised locals: UB).
     * Convention shared with the engine: that case is TRAPPED. */
    if (!(f & GBP_F_TNEW_SET) || !(f & GBP_F_SNEW_SET)) return GBP_TRAPPED;
    double s_mid[8];
    memcpy(s_mid, s_new, sizeof s_mid);
    if (attempt_connect_ts(T, s_existing, s_mid, t_new, s_new, a_new, direction, adaptive,
                           depth + 1, acs) == GBP_TRAPPED)
      return GBP_TRAPPED;
    return GBP_ADVANCED;
  }
  return GBP_TRAPPED;
}

int orc_attempt_connect(const orc_terrain *T, const double *s_existing, const double *s,
                        double t_s, double *s_new, double *a_new, int direction, int adaptive) {
  if (!(t_s > 0)) t_s = orc_pose_distance(s, s_existing) / V_NOM; /* rrt_connect.cpp:89 */
  return attempt_connect_ts(T, s_existing, s, t_s, s_new, a_new, direction, adaptive, 0, 0);
}

/* ---- batch helpers ------------------------------------------------------ */
#ifdef _OPENMP
#define OMP_FOR _Pragma("omp parallel for schedule(dynamic, 256) num_threads(nthreads)")
#else
#define OMP_FOR
#endif

void orc_validate_pairs(const orc_terrain *T, int64_t n, const double *s, const double *a,
                        const uint8_t *direction, int direction_all, int adaptive,
                        uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                        uint32_t *counts, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    double sn[8], tn;
    uint32_t f, c;
    int dir = direction ? direction[i] : direction_all;
    int v = orc_is_valid_pair(T, s + 8 * i, a + 10 * i, dir, adaptive, sn, &tn, &f, &c);
    if (valid) valid[i] = (uint8_t)v;
    if (s_new && (f & GBP_F_SNEW_SET)) memcpy(s_new + 8 * i, sn, sizeof sn);
    if (t_new && (f & GBP_F_TNEW_SET)) t_new[i] = tn;
    if (flags) flags[i] = f;
    if (counts) counts[i] = c;
  }
}

void orc_valid_states(const orc_terrain *T, int64_t n, const double *states,
                      const uint8_t *phase, int phase_all, uint8_t *valid, uint32_t *flags,
                      uint32_t *counts, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    orc_stats st = {0, 0, 0};
    int v = orc_is_valid_state(T, states + 8 * i, phase ? phase[i] : phase_all, &st);
    if (valid) valid[i] = (uint8_t)v;
    if (flags) flags[i] = st.flags | (v ? GBP_F_VALID : 0u);
    if (counts) counts[i] = (st.G & 0xFFFFu) | (st.V << 16);
  }
}

void orc_height_batch(const orc_terrain *T, int64_t n, const double *xy, double *h,
                      uint8_t *is_nan, uint8_t *ood, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    int o1 = 0, o2 = 0;
    double v = orc_ground_height(T, xy[2 * i], xy[2 * i + 1], &o1);
    int nn = orc_height_is_nan(T, xy[2 * i], xy[2 * i + 1], &o2);
    if (h) h[i] = v;
    if (is_nan) is_nan[i] = (uint8_t)nn;
    if (ood) ood[i] = (uint8_t)(o1 | o2);
  }
}

void orc_normal_batch(const orc_terrain *T, int64_t n, const double *xy, double *nrm,
                      uint8_t *ood, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    int o = 0;
    orc_surface_normal(T, xy[2 * i], xy[2 * i + 1], nrm + 3 * i, &o);
    if (ood) ood[i] = (uint8_t)o;
  }
}

void orc_extend_batch(const orc_terrain *T, int64_t n, const double *s_near,
                      const double *target, const double *actions, const uint8_t *direction,
                      int direction_all, int adaptive, int32_t *result, int32_t *chosen,
                      double *s_new, double *a_new, uint32_t *counts, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    double sn[8], an[10];
    int ch;
    uint32_t c;
    int dir = direction ? direction[i] : direction_all;
    int r = orc_extend(T, s_near + 8 * i, target + 8 * i, actions + 60 * i, dir, adaptive, sn,
                       an, &ch, &c);
    if (result) result[i] = r;
    if (chosen) chosen[i] = ch;
    if (r != GBP_TRAPPED) {
      if (s_new) memcpy(s_new + 8 * i, sn, sizeof sn);
      if (a_new) memcpy(a_new + 10 * i, an, sizeof an);
    }
    if (counts) counts[i] = c;
  }
}

void orc_nearest_batch(int64_t n_q, const double *q, int n_vert, const double *verts,
                       int32_t *idx, double *dist, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n_q; i++) {
    double d;
    int k = orc_nearest(verts, n_vert, q + 8 * i, &d);
    if (idx) idx[i] = k;
    if (dist) dist[i] = d;
  }
}

/* ---- the iteration order of GraphClass::vertices ----------------------------
 * graph_class.h:155 keeps the vertices in a std::unordered_map<int, State>
 * filled by operator[] with keys 0, 1, 2, ... (graph_class.cpp:28-31, :141-145;
 * a tree is never erased from), and neighborhoodDist / getNearestNeighbor walk
 * it begin() to end() (planner_class.cpp:176-179, :190-198).  libstdc++ (GCC
 * 11.4, this image's g++; the third-party arithmetic SURVEY §8(c) names) keeps
 * one singly linked list: a key whose bucket is empty is linked at the FRONT,
 * and a rehash relinks the nodes in list order, each at the front of the new
 * list — it reverses the list.  With int keys hashed to themselves and the load
 * factor <= 1 every key below the bucket count has a bucket of its own, so the
 * order of keys 0..n-1 is
 *     order(n) = [n-1, n-2, ..., r] ++ reverse(order(r))
 * where r is the last rehash point <= n-1: the element counts at which
 * _Prime_rehash_policy::_M_need_rehash grows the table (the first insertion
 * into the single-bucket empty map, then every time the size reaches the
 * bucket count; bucket counts from __prime_list, growth factor 2).  The points
 * below were read from libstdc++'s own policy object and are checked against a
 * real std::unordered_map by tests/test_um_order.py. */
static const int64_t UM_REHASH[] = {
    0,        13,       29,        59,        127,       257,       541,
    1109,     2357,     5087,      10273,     20753,     42043,     85229,
    172933,   351061,   712697,    1447153,   2938679,   5967347,   12117689,
    24607243, 49969847, 101473717, 206062531, 418451333, 849749479, 1725587117};
#define UM_NREHASH ((int)(sizeof UM_REHASH / sizeof UM_REHASH[0]))

/* index of the last rehash point <= n - 1 (n >= 1) */
static int um_epoch(int64_t n) {
  int m = 0;
  while (m + 1 < UM_NREHASH && UM_REHASH[m + 1] <= n - 1) m++;
  return m;
}

/* position of key k (0 <= k < n) when a map holding keys 0..n-1 is iterated */
int64_t orc_um_rank(int64_t k, int64_t n) {
  /* rank(k, n) = n-1-k in the front run, else n-1-rank(k, r): k's place in
   * reverse(order(r)), which fills the last r places */
  int64_t acc = 0, sign = 1;
  for (;;) {
    const int64_t r = UM_REHASH[um_epoch(n)];
    if (k >= r) return acc + sign * (n - 1 - k);
    acc += sign * (n - 1);
    sign = -sign;
    n = r;
  }
}

/* the segments of order(n): key ranges [lo, hi) walked descending (desc = 1)
 * or ascending, in iteration order; returns their count (<= UM_NREHASH) */
static int um_segments(int64_t n, int64_t *lo, int64_t *hi, int *desc) {
  if (n <= 0) return 0;
  const int m = um_epoch(n);
  int c = 0;
  /* order(n) = desc[R_m, n) ++ desc[R_{m-2}, R_{m-1}) ++ ... ++ asc[R_{m-3}, R_{m-2}) ++ asc[R_{m-1}, R_m) */
  for (int j = m; j >= 0; j -= 2) {
    lo[c] = UM_REHASH[j];
    hi[c] = j == m ? n : UM_REHASH[j + 1];
    desc[c++] = 1;
  }
  for (int j = (m - 1) & 1; j <= m - 1; j += 2) {
    lo[c] = UM_REHASH[j];
    hi[c] = UM_REHASH[j + 1];
    desc[c++] = 0;
  }
  return c;
}

/* the keys 0..n-1 in iteration order */
void orc_um_order(int64_t n, int32_t *out) {
  int64_t lo[2 * UM_NREHASH], hi[2 * UM_NREHASH];
  int desc[2 * UM_NREHASH];
  const int ns = um_segments(n, lo, hi, desc);
  int64_t p = 0;
  for (int s = 0; s < ns; s++) {
    if (desc[s])
      for (int64_t k = hi[s] - 1; k >= lo[s]; k--) out[p++] = (int32_t)k;
    else
      for (int64_t k = lo[s]; k < hi[s]; k++) out[p++] = (int32_t)k;
  }
}

/* PlannerClass::neighborhoodDist (planner_class.cpp:173-182): the vertices
 * 0..n_vert-1 with 0 < stateDistance <= dist, in the map's iteration order
 * (order = 0) or ascending index (order = 1, the engine's form before round 6,
 * kept for the tests that show the two differ) */
void orc_neighbors_batch(int64_t n_q, const double *q, int n_vert, const double *verts,
                         double radius, int max_out, int32_t *out, int32_t *count, int nthreads) {
  orc_neighbors_batch_ordered(n_q, q, n_vert, verts, radius, max_out, out, count, 0, nthreads);
}

void orc_neighbors_batch_ordered(int64_t n_q, const double *q, int n_vert, const double *verts,
                                 double radius, int max_out, int32_t *out, int32_t *count,
                                 int order, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  int64_t lo[2 * UM_NREHASH], hi[2 * UM_NREHASH];
  int desc[2 * UM_NREHASH];
  int ns = 1;
  if (order == 0) {
    ns = um_segments(n_vert, lo, hi, desc);
  } else {
    lo[0] = 0;
    hi[0] = n_vert;
    desc[0] = 0;
  }
  OMP_FOR
  for (int64_t i = 0; i < n_q; i++) {
    int c = 0;
    for (int s = 0; s < ns; s++) {
      const int64_t len = hi[s] - lo[s];
      for (int64_t t = 0; t < len; t++) {
        const int64_t v = desc[s] ? hi[s] - 1 - t : lo[s] + t;
        if ((orc_state_distance(q + 8 * i, verts + v * 8) <= radius) &&
            orc_state_distance(q + 8 * i, verts + v * 8) > 0) {
          if (c < max_out) out[i * (int64_t)max_out + c] = (int32_t)v;
          c++;
        }
      }
    }
    count[i] = c;
  }
}

/* PlannerClass::neighborhoodN (planner_class.cpp:151-171): the reference
 * pushes every (stateDistance, index) into a min-heap of std::pair<double, int>
 * (std::greater) and pops min(N, size): ascending distance, equal distances by
 * ascending index.  Restated as a full sort of the keys (NaN distances ordered
 * after every number, ascending index among them).  out[n_q][n_nearest], -1 /
 * NaN past the tree's size. */
typedef struct {
  double key, d;
  int i;
} knn_entry;

static int knn_cmp(const void *pa, const void *pb) {
  const knn_entry *a = (const knn_entry *)pa, *b = (const knn_entry *)pb;
  if (a->key < b->key) return -1;
  if (b->key < a->key) return 1;
  return (a->i > b->i) - (a->i < b->i);
}

/* planning_utils.h:146-155: stateDistance(q1, q2, cost_add_yaw_flag, lw, yw) */
double orc_state_distance_yaw(const double *q1, const double *q2, int flag, double lw, double yw) {
  if (flag) return orc_pose_distance(q1, q2) * lw + orc_state_yaw_distance(q1, q2) * yw;
  return orc_state_distance(q1, q2);
}

/* neighborhoodN, the key stateDistance(q, v, flag, lw, yw) (planner_class.cpp:157-158) */
void orc_knn_yaw_batch(int64_t n_q, const double *q, int n_vert, const double *verts, int n_nearest,
                       int flag, double lw, double yw, int32_t *out, double *dist, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n_q; i++) {
    knn_entry *e = (knn_entry *)malloc(sizeof(knn_entry) * (size_t)(n_vert > 0 ? n_vert : 1));
    for (int v = 0; v < n_vert; v++) {
      double d = orc_state_distance_yaw(q + 8 * i, verts + (long)v * 8, flag, lw, yw);
      e[v].d = d;
      e[v].key = isnan(d) ? INFINITY : d;
      e[v].i = v;
    }
    qsort(e, (size_t)n_vert, sizeof(knn_entry), knn_cmp);
    for (int k = 0; k < n_nearest; k++) {
      out[i * n_nearest + k] = k < n_vert ? e[k].i : -1;
      if (dist) dist[i * n_nearest + k] = k < n_vert ? e[k].d : NAN;
    }
    free(e);
  }
}

void orc_knn_batch(int64_t n_q, const double *q, int n_vert, const double *verts, int n_nearest,
                   int32_t *out, double *dist, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n_q; i++) {
    knn_entry *e = (knn_entry *)malloc(sizeof(knn_entry) * (size_t)(n_vert > 0 ? n_vert : 1));
    for (int v = 0; v < n_vert; v++) {
      double d = orc_state_distance(q + 8 * i, verts + (long)v * 8);
      e[v].d = d;
      e[v].key = isnan(d) ? INFINITY : d;
      e[v].i = v;
    }
    qsort(e, (size_t)n_vert, sizeof(knn_entry), knn_cmp);
    for (int k = 0; k < n_nearest; k++) {
      out[i * n_nearest + k] = k < n_vert ? e[k].i : -1;
      if (dist) dist[i * n_nearest + k] = k < n_vert ? e[k].d : NAN;
    }
    free(e);
  }
}

/* ---- Philox4x32-10 (Salmon et al., SC'11) ------------------------------- */
static inline void mulhilo32(uint32_t a, uint32_t b, uint32_t *hi, uint32_t *lo) {
  uint64_t p = (uint64_t)a * b;
  *hi = (uint32_t)(p >> 32);
  *lo = (uint32_t)p;
}

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; r++) {
    uint32_t hi0, lo0, hi1, lo1;
    mulhilo32(0xD2511F53u, c0, &hi0, &lo0);
    mulhilo32(0xCD9E8D57u, c2, &hi1, &lo1);
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

void orc_uniform2(uint64_t seed, uint64_t stream_id, uint32_t purpose, int64_t index,
                  uint32_t draw, double u[2]) {
  uint32_t ctr[4] = {draw, (uint32_t)(uint64_t)index, (uint32_t)((uint64_t)index >> 32),
                     (uint32_t)stream_id ^ (purpose << 24)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32) ^ (uint32_t)(stream_id >> 32)};
  uint32_t o[4];
  orc_philox4x32_10(ctr, key, o);
  uint64_t w0 = ((uint64_t)o[1] << 32) | o[0];
  uint64_t w1 = ((uint64_t)o[3] << 32) | o[2];
  u[0] = (double)(w0 >> 11) * 0x1p-53;
  u[1] = (double)(w1 >> 11) * 0x1p-53;
}

/* ---- the samplers' transcendentals (restates gbp_device.h rm_*) -------------
 * The reference draws from rand() and clock-seeded engines: its
 * samples are not reproducible, so the engine defines its own streams, and
 * with them the log / sin / cos / acos / atan2 that turn uniforms into
 * samples.  glibc and the device libm differ in the last bits, so both sides
 * use these routines: +, -, *, /, sqrt, floor, frexp only (all correctly
 * rounded or exact in IEEE binary64), no contraction, fixed Horner order —
 * host and device then draw bit-identical targets and candidate actions, and
 * a planner run is reproducible bit for bit off the device.  Accuracy: a few
 * ulp (Taylor / atanh series past 1e-17 relative), which leaves the
 * distributions the reference samples unchanged. */
static const double RM_SIN[9] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7,
                                 -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
                                 -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33,
                                 -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49,
                                 -0x1.2f49b46814157p-57};
static const double RM_COS[9] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5,
                                 -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
                                 -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29,
                                 -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45,
                                 -0x1.6827863b97d97p-53};
static const double RM_LOG[11] = {0x1.5555555555555p-1, 0x1.999999999999ap-2, 0x1.2492492492492p-2,
                                  0x1.c71c71c71c71cp-3, 0x1.745d1745d1746p-3, 0x1.3b13b13b13b14p-3,
                                  0x1.1111111111111p-3, 0x1.e1e1e1e1e1e1ep-4, 0x1.af286bca1af28p-4,
                                  0x1.8618618618618p-4, 0x1.642c8590b2164p-4};
static const double RM_ATAN[12] = {-0x1.5555555555555p-2, 0x1.999999999999ap-3,
                                   -0x1.2492492492492p-3, 0x1.c71c71c71c71cp-4,
                                   -0x1.745d1745d1746p-4, 0x1.3b13b13b13b14p-4,
                                   -0x1.1111111111111p-4, 0x1.e1e1e1e1e1e1ep-5,
                                   -0x1.af286bca1af28p-5, 0x1.8618618618618p-5,
                                   -0x1.642c8590b2164p-5, 0x1.47ae147ae147bp-5};
#define RM_INVPIO2 0x1.45f306dc9c883p-1
#define RM_PIO2_1 0x1.921fb54400000p+0
#define RM_PIO2_2 0x1.0b4611a600000p-34
#define RM_PIO2_2T 0x1.3198a2e037073p-69
#define RM_PIO2_HI 0x1.921fb54442d18p+0
#define RM_PIO2_LO 0x1.1a62633145c07p-54
#define RM_PI_HI 0x1.921fb54442d18p+1
#define RM_PI_LO 0x1.1a62633145c07p-53
#define RM_LN2_HI 0x1.62e42fee00000p-1
#define RM_LN2_LO 0x1.a39ef35793c76p-33

/* ln x, x > 0 finite: x = m 2^e, m in [sqrt(1/2), sqrt(2)), ln m = 2 atanh(f) */
static double rm_log(double x) {
  int e;
  double m = frexp(x, &e);
  if (m < 0x1.6a09e667f3bcdp-1) {
    m = m * 2.0;
    e = e - 1;
  }
  double f = (m - 1.0) / (m + 1.0);
  double w = f * f;
  double p = RM_LOG[10];
  for (int k = 9; k >= 0; k--) p = RM_LOG[k] + w * p;
  double l = 2.0 * f + f * w * p;
  double de = (double)e;
  return de * RM_LN2_HI + (l + de * RM_LN2_LO);
}

/* sin x, cos x for |x| < 2^20: x = k pi/2 + r (Cody-Waite, three parts) */
static void rm_sincos(double x, double *s, double *c) {
  double kf = floor(x * RM_INVPIO2 + 0.5);
  double r = ((x - kf * RM_PIO2_1) - kf * RM_PIO2_2) - kf * RM_PIO2_2T;
  double z = r * r;
  double ps = RM_SIN[8], pc = RM_COS[8];
  for (int k = 7; k >= 0; k--) {
    ps = RM_SIN[k] + z * ps;
    pc = RM_COS[k] + z * pc;
  }
  double sr = r + r * z * ps;
  double cr = 1.0 + z * pc;
  switch ((int)kf & 3) {
    case 0: *s = sr; *c = cr; break;
    case 1: *s = cr; *c = -sr; break;
    case 2: *s = -sr; *c = -cr; break;
    default: *s = -cr; *c = sr; break;
  }
}

/* atan t, t in [0, 1]: two halvings atan t = 2 atan(t / (1 + sqrt(1 + t^2))),
 * then the series on [0, tan(pi/16)] */
static double rm_atan01(double t) {
  t = t / (1.0 + sqrt(1.0 + t * t));
  t = t / (1.0 + sqrt(1.0 + t * t));
  double v = t * t;
  double p = RM_ATAN[11];
  for (int k = 10; k >= 0; k--) p = RM_ATAN[k] + v * p;
  return 4.0 * (t + t * v * p);
}

/* atan2 with glibc's signed-zero / axis conventions */
static double rm_atan2(double y, double x) {
  if (isnan(x) || isnan(y)) return x + y;
  double ax = fabs(x), ay = fabs(y), a;
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

/* acos c, c in [-1, 1] */
static double rm_acos(double c) { return rm_atan2(sqrt((1.0 - c) * (1.0 + c)), c); }

/* Box-Muller pair (the reference's libstdc++ polar method yields a pair too:
 * a[9] is its cached second value) */
static void box_muller(double u1, double u2, double *z0, double *z1) {
  double r = sqrt(-2.0 * rm_log(1.0 - u1));
  double th = 6.283185307179586 * u2;
  double s, c;
  rm_sincos(th, &s, &c);
  *z0 = r * c;
  *z1 = r * s;
}

/* v (sin theta cos phi, sin theta sin phi, cos theta), theta = acos(cos_theta)
 * (planner_class.cpp:61-73) */
static void speed_vector(double v, double cos_theta, double phi, double *q) {
  double theta = rm_acos(cos_theta);
  double st, ct, sp, cp;
  rm_sincos(theta, &st, &ct);
  rm_sincos(phi, &sp, &cp);
  q[3] = v * st * cp;
  q[4] = v * st * sp;
  q[5] = v * ct;
}

/* exported for the CPU tests of the routines (accuracy vs glibc) */
void orc_rmath(int fn, int64_t n, const double *x, const double *y, double *out) {
  for (int64_t i = 0; i < n; i++) {
    double s, c;
    switch (fn) {
      case 0: out[i] = rm_log(x[i]); break;
      case 1: rm_sincos(x[i], &s, &c); out[2 * i] = s; out[2 * i + 1] = c; break;
      case 2: out[i] = rm_atan2(y[i], x[i]); break;
      default: out[i] = rm_acos(x[i]); break;
    }
  }
}

/* planner_class.cpp:38-76 */
int orc_sample_state(const orc_terrain *T, uint64_t seed, uint64_t stream_id, int64_t index,
                     int require_phase, int max_tries, double *q) {
  double x_min = T->x[0], x_max = T->x[T->nx - 1];
  double y_min = T->y[0], y_max = T->y[T->ny - 1];
  double z_min_rel = H_MIN + ROBOT_H, z_max_rel = H_MAX + ROBOT_H;
  double mean = 0.5 * (z_max_rel + z_min_rel);
  double sd = (z_max_rel - z_min_rel) * (1.0 / (2 * 3.0));
  if (max_tries <= 0) max_tries = 1;
  for (int k = 0; k < max_tries; k++) {
    double u0[2], u1[2], u2[2], u3[2];
    orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 0, u0);
    orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 1, u1);
    orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 2, u2);
    orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 4u * k + 3, u3);
    double z0, z1;
    box_muller(u1[0], u1[1], &z0, &z1);
    double hz = z0 * sd + mean;
    q[0] = (x_max - x_min) * u0[0] + x_min;
    q[1] = (y_max - y_min) * u0[1] + y_min;
    q[2] = std_max(std_min(hz, z_max_rel), z_min_rel) + orc_ground_height(T, q[0], q[1], 0);
    double phi = (2.0 * MY_PI) * u2[0];
    double cos_theta = 2.0 * u2[1] - 1.0;
    double v = u3[0] * V_MAX;
    speed_vector(v, cos_theta, phi, q);
    q[6] = 2 * P_MAX * u3[1] - P_MAX;
    q[7] = 0.0;
    if (require_phase < 0) return k + 1;
    orc_stats st = {0, 0, 0};
    if (orc_is_valid_state(T, q, require_phase, &st)) return k + 1;
  }
  return -1;
}

/* planning_utils.cpp:198-231 */
void orc_rotate_grf(const double *n, const double *f, double *out) {
  double v0 = n[1] * 1.0 - n[2] * 0.0;
  double v1 = n[2] * 0.0 - n[0] * 1.0;
  double v2 = n[0] * 0.0 - n[1] * 0.0;
  double s = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
  double c = n[0] * 0.0 + n[1] * 0.0 + n[2] * 1.0;
  if (s < 0.000001) {
    out[0] = f[0]; out[1] = f[1]; out[2] = f[2];
    return;
  }
  double K[3][3] = {{0, -v2, v1}, {v2, 0, -v0}, {-v1, v0, 0}};
  double R[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
      R[i][j] = (i == j ? 1.0 : 0.0) + K[i][j] + kk * (1 - c) / (s * s);
    }
  for (int i = 0; i < 3; i++) out[i] = R[i][0] * f[0] + R[i][1] * f[1] + R[i][2] * f[2];
}

/* planning_utils.cpp:392-442 */
void orc_sample_action(const double *nrm, uint64_t seed, uint64_t stream_id, int64_t index,
                       double *a) {
  double u[5][2];
  for (uint32_t d = 0; d < 5; d++) orc_uniform2(seed, stream_id, PURPOSE_ACTION, index, d, u[d]);
  double f_z_td = F_MAX * u[0][0];
  double f_z_to = F_MAX * u[0][1];
  double f_x_td = 2 * MU * f_z_td * u[1][0] - MU * f_z_td;
  double f_x_to = 2 * MU * f_z_to * u[1][1] - MU * f_z_to;
  double f_y_td = 2 * MU * f_z_td * u[2][0] - MU * f_z_td;
  double f_y_to = 2 * MU * f_z_to * u[2][1] - MU * f_z_to;
  double f_td[3] = {f_x_td, f_y_td, f_z_td}, f_to[3] = {f_x_to, f_y_to, f_z_to};
  double r_td[3], r_to[3];
  orc_rotate_grf(nrm, f_td, r_td);
  orc_rotate_grf(nrm, f_to, r_to);
  double t_s = 0.3;
  double t_f = (T_F_MAX - T_F_MIN) * u[3][0] + T_F_MIN;
  a[0] = r_td[0] / M_CONST;
  a[1] = r_td[1] / M_CONST;
  a[2] = r_td[2] / M_CONST - G_CONST;
  a[3] = r_to[0] / M_CONST;
  a[4] = r_to[1] / M_CONST;
  a[5] = r_to[2] / M_CONST - G_CONST;
  a[6] = t_s;
  a[7] = t_f;
  double z0, z1;
  box_muller(u[4][0], u[4][1], &z0, &z1);
  double n0 = z0 * (ANG_ACC_MAX / 4.0) + 0.0, n1 = z1 * (ANG_ACC_MAX / 4.0) + 0.0;
  a[8] = std_max(std_min(n0, ANG_ACC_MAX), -ANG_ACC_MAX);
  a[9] = std_max(std_min(n1, ANG_ACC_MAX), -ANG_ACC_MAX);
}

/* ---- direction-biased sampling ----------------------------------------------
 * The reference's coin `(double) rand() / RAND_MAX <= threshold`
 * (planner_class.cpp:27-29, planning_utils.cpp:381-383) is the engine's
 * uniform of purpose PURPOSE_COIN (index, draw = try / 0). */
#define PURPOSE_COIN 3u
static int coin(uint64_t seed, uint64_t stream_id, int64_t index, uint32_t draw, double p) {
  double c[2];
  orc_uniform2(seed, stream_id, PURPOSE_COIN, index, draw, c);
  return c[0] <= p;
}

/* planning_utils.cpp:443-515 (the draws of orc_sample_action, the tangential
 * forces on the side of the velocity change s_from -> s_to) */
static void sample_action_direction(const double *nrm, const double *s_from, const double *s_to,
                                    uint64_t seed, uint64_t stream_id, int64_t index, double *a) {
  double u[5][2];
  for (uint32_t d = 0; d < 5; d++) orc_uniform2(seed, stream_id, PURPOSE_ACTION, index, d, u[d]);
  int dx_increase_flag = s_to[3] > s_from[3];
  int dy_increase_flag = s_to[4] > s_from[4];
  double f_z_td = F_MAX * u[0][0];
  double f_z_to = F_MAX * u[0][1];
  double f_friction_td = MU * f_z_td;
  double f_friction_to = MU * f_z_to;
  double f_x_td, f_x_to, f_y_td, f_y_to;
  if (dx_increase_flag) {
    f_x_td = f_friction_td * u[1][0];
    f_x_to = f_friction_to * u[1][1];
  } else {
    f_x_td = f_friction_td * u[1][0] - f_friction_td;
    f_x_to = f_friction_to * u[1][1] - f_friction_to;
  }
  if (dy_increase_flag) {
    f_y_td = f_friction_td * u[2][0];
    f_y_to = f_friction_to * u[2][1];
  } else {
    f_y_td = f_friction_td * u[2][0] - f_friction_td;
    f_y_to = f_friction_to * u[2][1] - f_friction_to;
  }
  double f_td[3] = {f_x_td, f_y_td, f_z_td}, f_to[3] = {f_x_to, f_y_to, f_z_to};
  double r_td[3], r_to[3];
  orc_rotate_grf(nrm, f_td, r_td);
  orc_rotate_grf(nrm, f_to, r_to);
  a[0] = r_td[0] / M_CONST;
  a[1] = r_td[1] / M_CONST;
  a[2] = r_td[2] / M_CONST - G_CONST;
  a[3] = r_to[0] / M_CONST;
  a[4] = r_to[1] / M_CONST;
  a[5] = r_to[2] / M_CONST - G_CONST;
  a[6] = 0.3;
  a[7] = (T_F_MAX - T_F_MIN) * u[3][0] + T_F_MIN;
  double z0, z1;
  box_muller(u[4][0], u[4][1], &z0, &z1);
  double n0 = z0 * (ANG_ACC_MAX / 4.0) + 0.0, n1 = z1 * (ANG_ACC_MAX / 4.0) + 0.0;
  a[8] = std_max(std_min(n0, ANG_ACC_MAX), -ANG_ACC_MAX);
  a[9] = std_max(std_min(n1, ANG_ACC_MAX), -ANG_ACC_MAX);
}

/* planning_utils.cpp:379-391 */
static void sample_action_any(const double *nrm, int direction, int flag, double p,
                              const double *s, const double *s_near, uint64_t seed,
                              uint64_t stream_id, int64_t index, double *a) {
  if (flag && coin(seed, stream_id, index, 0, p)) {
    if (direction == GBP_FORWARD)
      sample_action_direction(nrm, s_near, s, seed, stream_id, index, a);
    else
      sample_action_direction(nrm, s, s_near, seed, stream_id, index, a);
  } else {
    orc_sample_action(nrm, seed, stream_id, index, a);
  }
}

/* planner_class.cpp:82-148, one try (draws 0..3 of the index) */
static void sample_state_direction(const orc_terrain *T, const double *s_from, const double *s_to,
                                   int speed_direction_flag, uint64_t seed, uint64_t stream_id,
                                   int64_t index, double *q) {
  double x_min = std_min(s_from[0], s_to[0]);
  double x_max = std_max(s_from[0], s_to[0]);
  double y_min = std_min(s_from[1], s_to[1]);
  double y_max = std_max(s_from[1], s_to[1]);
  double z_min_rel = H_MIN + ROBOT_H, z_max_rel = H_MAX + ROBOT_H;
  double mean = 0.5 * (z_max_rel + z_min_rel);
  double sd = (z_max_rel - z_min_rel) * (1.0 / (2 * 3.0));
  double u0[2], u1[2], u2[2], u3[2];
  orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 0, u0);
  orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 1, u1);
  orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 2, u2);
  orc_uniform2(seed, stream_id, PURPOSE_STATE, index, 3, u3);
  double z0, z1;
  box_muller(u1[0], u1[1], &z0, &z1);
  double hz = z0 * sd + mean;
  q[0] = (x_max - x_min) * u0[0] + x_min;
  q[1] = (y_max - y_min) * u0[1] + y_min;
  q[2] = std_max(std_min(hz, z_max_rel), z_min_rel) + orc_ground_height(T, q[0], q[1], 0);
  double phi;
  if (speed_direction_flag) {
    double delta_x = s_to[0] - s_from[0];
    double delta_y = s_to[1] - s_from[1];
    phi = rm_atan2(delta_y, delta_x);
  } else {
    phi = (2.0 * MY_PI) * u2[0];
  }
  double cos_theta = 2.0 * u2[1] - 1.0;
  double v = u3[0] * V_MAX;
  speed_vector(v, cos_theta, phi, q);
  q[6] = 2 * P_MAX * u3[1] - P_MAX;
  q[7] = 0.0;
}

void orc_sample_states_dir(const orc_terrain *T, int64_t n, uint64_t seed, uint64_t stream_id,
                           int64_t index_base, int state_flag, double state_p, int speed_direction,
                           const double *s_from, const double *s_to, double *states, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    const int64_t idx = index_base + i;
    if (state_flag && coin(seed, stream_id, idx, 0, state_p)) /* planner_class.cpp:22-35 */
      sample_state_direction(T, s_from, s_to, speed_direction, seed, stream_id, idx, states + 8 * i);
    else
      orc_sample_state(T, seed, stream_id, idx, -1, 1, states + 8 * i);
  }
}

void orc_sample_actions_dir(int64_t n, const double *normals, const double *s,
                            const double *s_near, const uint8_t *direction, int direction_all,
                            int action_flag, double action_p, uint64_t seed, uint64_t stream_id,
                            int64_t index_base, double *actions, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++)
    sample_action_any(normals + 3 * i, direction ? direction[i] : direction_all, action_flag,
                      action_p, s + 8 * i, s_near + 8 * i, seed, stream_id, index_base + i,
                      actions + 10 * i);
}

void orc_sample_states(const orc_terrain *T, int64_t n, uint64_t seed, uint64_t stream_id,
                       int64_t index_base, int require_phase, int max_tries, double *states,
                       int32_t *tries, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++) {
    int k = orc_sample_state(T, seed, stream_id, index_base + i, require_phase, max_tries,
                             states + 8 * i);
    if (tries) tries[i] = k;
  }
}

void orc_sample_actions(int64_t n, const double *normals, uint64_t seed, uint64_t stream_id,
                        int64_t index_base, double *actions, int nthreads) {
  if (nthreads <= 0) nthreads = 1;
  OMP_FOR
  for (int64_t i = 0; i < n; i++)
    orc_sample_action(normals + 3 * i, seed, stream_id, index_base + i, actions + 10 * i);
}

/* ==== the planner loop ========================================================
 * The batch-synchronous RRT-Connect the engine runs (include/gbp_planner.h
 * buildRRTConnectBatched / buildRRTConnectDevice) restated on the CPU: each
 * half-iteration h extends tree h % 2 (Ta FORWARD, Tb REVERSE) toward B random
 * targets against the tree as it stands when the half starts, appends the
 * successors in target order, then connects each new vertex to the other tree
 * (again against that tree's snapshot) and appends the connections in order.
 * B = 1 is the reference's runRRTConnect (rrt_connect.cpp:230-314) on the
 * engine's counter-based streams.  Every draw, decision and tree update
 * below is the oracle's own (the functions above), nothing is read from the
 * engine. */
#define EXTD_STREAM 0x45585444ull /* newConfig's candidates: (extend index) * 8 + j */

static void tree_put(orc_tree *t, const double *v, const double *a, int parent, double g,
                     double y) {
  int i = t->n++;
  memcpy(t->v + 8 * (int64_t)i, v, 8 * sizeof(double));
  if (a) memcpy(t->a + 10 * (int64_t)i, a, 10 * sizeof(double));
  else memset(t->a + 10 * (int64_t)i, 0, 10 * sizeof(double));
  t->parent[i] = parent;
  t->g[i] = g;
  t->y[i] = y;
  if (t->child) {
    t->child[i] = -1;
    t->sibling[i] = -1;
  }
}

/* graph_class.cpp:36-42 (the successor list kept as first-child / next-sibling) */
static void tree_add_edge(orc_tree *t, int p, int c) {
  const double *vp = t->v + 8 * (int64_t)p, *vc = t->v + 8 * (int64_t)c;
  t->parent[c] = p;
  if (t->child) {
    t->sibling[c] = t->child[p];
    t->child[p] = c;
  }
  t->g[c] = t->g[p] + orc_pose_distance(vp, vc);
  t->y[c] = t->y[p] + orc_state_yaw_distance(vp, vc);
}

/* graph_class.cpp:44-58 */
static void tree_remove_edge(orc_tree *t, int p, int c) {
  if (t->parent[c] == p) t->parent[c] = -1;
  int *link = &t->child[p];
  while (*link >= 0 && *link != c) link = &t->sibling[*link];
  if (*link == c) *link = t->sibling[c];
}

/* RRT* insertion statistics (orc_star_stats; diagnostics only): insertions,
 * neighbours, max neighbours, rewires, subtree vertices updated by rewires,
 * largest such subtree, summed subtree depths, deepest subtree */
static int64_t g_star_stats[8];
static int64_t g_gy_nodes, g_gy_depth;

void orc_star_stats(int64_t out[8], int reset) {
  for (int i = 0; i < 8; i++) {
    if (out) out[i] = g_star_stats[i];
    if (reset) g_star_stats[i] = 0;
  }
}

/* graph_class.cpp:131-138 (recursive over the successors) */
static void tree_update_gy_d(orc_tree *t, int idx, double g, double y, int64_t depth) {
  t->g[idx] = g;
  t->y[idx] = y;
  g_gy_nodes++;
  if (depth > g_gy_depth) g_gy_depth = depth;
  for (int c = t->child ? t->child[idx] : -1; c >= 0; c = t->sibling[c]) {
    const double *vi = t->v + 8 * (int64_t)idx, *vc = t->v + 8 * (int64_t)c;
    tree_update_gy_d(t, c, t->g[idx] + orc_pose_distance(vi, vc),
                     t->y[idx] + orc_state_yaw_distance(vi, vc), depth + 1);
  }
}

static void tree_update_gy(orc_tree *t, int idx, double g, double y) {
  tree_update_gy_d(t, idx, g, y, 0);
}

/* attemptConnect's depth-0 decision only (callers that test == REACHED,
 * rrt_star_connect.cpp:36, :59): REACHED iff t_s > KINEMATICS_RES, the
 * cubic-Hermite action is valid and its pair check passes (rrt_connect.cpp:20-70);
 * a_new receives the action */
static int connect_reached(const orc_terrain *T, const double *s_existing, const double *s,
                           double t_s, int direction, int adaptive, double *a_new,
                           int64_t *checks) {
  if (t_s <= KINEMATICS_RES) return 0;
  const double *s_start = (direction == GBP_FORWARD) ? s_existing : s;
  const double *s_goal = (direction == GBP_FORWARD) ? s : s_existing;
  connect_action(s_start, s_goal, t_s, a_new);
  if (!orc_is_valid_action(a_new)) return 0;
  (*checks)++;
  double sn[8], tn;
  uint32_t f;
  return (direction == GBP_FORWARD)
             ? orc_is_valid_pair(T, s_start, a_new, GBP_FORWARD, adaptive, sn, &tn, &f, 0)
             : orc_is_valid_pair(T, s_goal, a_new, GBP_REVERSE, adaptive, sn, &tn, &f, 0);
}

/* rrt_star_connect.cpp:18-66 for the vertex `idx` just added to t (its
 * nearest `nn`, newConfig's action a_new): choose-parent among the vertices
 * within `delta` — neighborhoodDist (planner_class.cpp:173-182) over the map
 * that now holds keys 0..idx (addVertex at :22 precedes it), in the map's
 * iteration order (order 0; 1 = ascending index) — then rewire them through
 * it.  Both loops are order-dependent: a choose-parent tie goes to the first
 * neighbour, and a rewire lowers the g of a whole subtree that a later
 * neighbour's test (:59) then reads. */
static void star_insert(const orc_terrain *T, orc_tree *t, int idx, int nn, const double *a_new,
                        double delta, int direction, int adaptive, int order, orc_plan_out *out) {
  const double *s_new = t->v + 8 * (int64_t)idx;
  const double *s_nearest = t->v + 8 * (int64_t)nn;
  int nb_n = 0;
  int *nb = (int *)malloc(sizeof(int) * (size_t)(idx > 0 ? idx : 1));
  {
    int32_t cnt = 0;
    /* the key idx itself is at distance 0 and never listed */
    orc_neighbors_batch_ordered(1, s_new, idx + 1, t->v, delta, idx > 0 ? idx : 1, nb, &cnt, order, 1);
    nb_n = cnt;
  }
  out->connects += 2 * (int64_t)nb_n; /* a choose-parent and a rewire connect per neighbour */
  g_star_stats[0]++;
  g_star_stats[1] += nb_n;
  if (nb_n > g_star_stats[2]) g_star_stats[2] = nb_n;
  int s_min = nn;
  double a_sel[10], a_c[10];
  memcpy(a_sel, a_new, sizeof a_sel);
  double g_s_new = t->g[nn] + orc_pose_distance(s_new, s_nearest);
  double y_s_new = t->y[nn] + orc_state_yaw_distance(s_new, s_nearest);
  for (int i = 0; i < nb_n; i++) {
    const int j = nb[i];
    const double *s_near = t->v + 8 * (int64_t)j;
    if (connect_reached(T, s_near, s_new, orc_pose_distance(s_new, s_near) / V_NOM, direction,
                        adaptive, a_c, &out->attempts)) {
      double g_s_near = t->g[j] + orc_pose_distance(s_near, s_new);
      double y_s_near = t->y[j] + orc_state_yaw_distance(s_near, s_new);
      if (g_s_near < g_s_new) {
        memcpy(a_sel, a_c, sizeof a_sel);
        s_min = j;
        g_s_new = g_s_near;
        y_s_new = y_s_near;
      }
    }
  }
  tree_add_edge(t, s_min, idx);
  tree_update_gy(t, idx, g_s_new, y_s_new);
  memcpy(t->a + 10 * (int64_t)idx, a_sel, sizeof a_sel);
  for (int i = 0; i < nb_n; i++) {
    const int j = nb[i];
    const double *s_near = t->v + 8 * (int64_t)j;
    /* the engine checks every neighbour's rewire connect in one batch, the
     * parent's included (it only counts toward attempts) */
    int reached = connect_reached(T, s_new, s_near, orc_pose_distance(s_near, s_new) / V_NOM,
                                  direction, adaptive, a_c, &out->attempts);
    if (j == s_min) continue;
    if (reached &&
        (t->g[j] > (t->g[idx] + orc_pose_distance(s_near, s_new)))) {
      tree_remove_edge(t, t->parent[j], j);
      tree_add_edge(t, idx, j);
      g_gy_nodes = g_gy_depth = 0;
      tree_update_gy(t, j, t->g[idx] + orc_pose_distance(s_near, s_new),
                     t->y[idx] + orc_state_yaw_distance(s_near, s_new));
      g_star_stats[4] += g_gy_nodes;
      if (g_gy_nodes > g_star_stats[5]) g_star_stats[5] = g_gy_nodes;
      g_star_stats[6] += g_gy_depth;
      if (g_gy_depth > g_star_stats[7]) g_star_stats[7] = g_gy_depth;
      g_star_stats[3]++;
      memcpy(t->a + 10 * (int64_t)j, a_c, sizeof a_c);
      out->rewires++;
    }
  }
  free(nb);
}

/* vertices 0..n-1 of an RRT* tree given by parents alone (any tree rooted at
 * 0): successor lists, then g / y from the root down (every updateGYValue
 * keeps g[c] == g[parent] + poseDistance, graph_class.cpp:131-138, so these
 * are the bits the grown tree holds); -1 if it is not one tree rooted at 0 */
static int tree_derive_star(orc_tree *t, int n) {
  if (!t->child || n < 1 || t->parent[0] != -1) return -1;
  for (int i = 0; i < n; i++) t->child[i] = t->sibling[i] = -1;
  for (int i = 1; i < n; i++) {
    const int p = t->parent[i];
    if (p < 0 || p >= n || p == i) return -1;
    t->sibling[i] = t->child[p];
    t->child[p] = i;
  }
  t->g[0] = t->y[0] = 0.0;
  int *queue = (int *)malloc(sizeof(int) * (size_t)n);
  int qh = 0, qt = 0;
  queue[qt++] = 0;
  while (qh < qt) {
    const int p = queue[qh++];
    const double *vp = t->v + 8 * (int64_t)p;
    for (int c = t->child[p]; c >= 0; c = t->sibling[c]) {
      if (qt >= n) break;
      const double *vc = t->v + 8 * (int64_t)c;
      t->g[c] = t->g[p] + orc_pose_distance(vp, vc);
      t->y[c] = t->y[p] + orc_state_yaw_distance(vp, vc);
      queue[qt++] = c;
    }
  }
  free(queue);
  return qt == n ? 0 : -1;
}

int orc_star_insert_one(const orc_terrain *T, orc_tree *t, int idx, int nn, const double *a_new,
                        double delta, int direction, int adaptive, int order, int64_t *rewires) {
  if (!t || idx < 1 || idx >= t->cap || nn < 0 || nn >= idx) return -1;
  if (tree_derive_star(t, idx) != 0) return -1;
  t->n = idx + 1;
  t->parent[idx] = -1;
  t->child[idx] = t->sibling[idx] = -1;
  orc_plan_out out;
  memset(&out, 0, sizeof out);
  star_insert(T, t, idx, nn, a_new, delta, direction, adaptive, order, &out);
  if (rewires) *rewires = out.rewires;
  return 0;
}

int orc_plan(const orc_terrain *T, const double *start, const double *goal,
             const orc_plan_cfg *cfg, orc_tree *tr, orc_plan_out *out) {
  const int B = cfg->batch;
  const int star = cfg->star;
  if (B < 1 || !tr || !out) return -1;
  memset(out, 0, sizeof *out);
  out->meet_a = out->meet_b = -1;
  const int64_t h0 = cfg->warm ? cfg->first_half : 0;
  for (int k = 0; k < 2; k++) {
    if (cfg->warm && tr[k].n > 0) {
      /* a continuation: the given vertices in order, each joined to its parent
       * (graph_class.cpp:36-42: g / y from the parent's) */
      orc_tree *t = &tr[k];
      if (t->parent[0] != -1) return -1;
      t->g[0] = t->y[0] = 0.0;
      for (int i = 0; i < t->n; i++)
        if (t->child) t->child[i] = t->sibling[i] = -1;
      if (!star) {
        for (int i = 1; i < t->n; i++) {
          if (t->parent[i] < 0 || t->parent[i] >= i) return -1;
          tree_add_edge(t, t->parent[i], i);
        }
        continue;
      }
      /* RRT*: rewiring gives vertices parents added after them */
      if (tree_derive_star(t, t->n) != 0) return -1;
      continue;
    }
    tr[k].n = 0;
    tree_put(&tr[k], k == 0 ? start : goal, 0, -1, 0.0, 0.0);
  }
  const uint64_t stream[2] = {cfg->stream_a, cfg->stream_b};
  /* tree k's draws before half h0: (h >> 1) * B at half h of tree k */
  int64_t draws[2] = {((h0 + 1) >> 1) * (int64_t)B, (h0 >> 1) * (int64_t)B};
  int64_t ext = cfg->extend_base;
  double *cand = (double *)malloc(sizeof(double) * 8 * (size_t)B);
  double *tgt = (double *)malloc(sizeof(double) * 8 * (size_t)B);
  int *added = (int *)malloc(sizeof(int) * (size_t)B);
  int *nearest = (int *)malloc(sizeof(int) * (size_t)B);
  double *a_ext = (double *)malloc(sizeof(double) * 10 * (size_t)B);
  /* per-item results of the parallel passes (each item reads only the
   * half's snapshot of the trees; insertion stays sequential, in order) */
  int nthreads = cfg->nthreads > 0 ? cfg->nthreads : 1;
  int *it_nn = (int *)malloc(sizeof(int) * (size_t)B);
  int *it_r = (int *)malloc(sizeof(int) * (size_t)B);
  int64_t *it_chk = (int64_t *)malloc(sizeof(int64_t) * (size_t)B);
  int *it_cap = (int *)malloc(sizeof(int) * (size_t)B);
  double *it_sn = (double *)malloc(sizeof(double) * 8 * (size_t)B);
  double *it_an = (double *)malloc(sizeof(double) * 10 * (size_t)B);
  uint8_t *it_ok = (uint8_t *)malloc((size_t)B);
  double *shared = 0; /* RRT*: (a, b) vertex pairs whose connect REACHED */
  int64_t n_shared = 0, cap_shared = 0;
  double cost_so_far = INFINITY;
  int rc = 0;
  for (int64_t h = h0; cfg->max_halves <= 0 || h < h0 + cfg->max_halves; h++) {
    const int k = (int)(h & 1);
    orc_tree *Tt = &tr[k], *O = &tr[k ^ 1];
    const int dir = k == 0 ? GBP_FORWARD : GBP_REVERSE;
    const int cdir = k == 0 ? GBP_REVERSE : GBP_FORWARD;
    /* targets: randomState + isValidState(STANCE) (rrt_connect.cpp:248-254,
     * :283-289); s_from / s_to as the trees stand when the half starts */
    if (star) {
      for (int i = 0; i < B; i++)
        orc_sample_state(T, cfg->seed, stream[k], draws[k] + i, -1, 1, cand + 8 * i);
    } else {
      const double *last = Tt->v + 8 * (int64_t)(Tt->n - 1), *root = O->v;
      orc_sample_states_dir(T, B, cfg->seed, stream[k], draws[k], cfg->state_flag, cfg->state_p,
                            cfg->state_speed_direction, dir == GBP_FORWARD ? last : root,
                            dir == GBP_FORWARD ? root : last, cand, nthreads);
    }
    draws[k] += B;
    OMP_FOR
    for (int i = 0; i < B; i++) {
      orc_stats st = {0, 0, 0};
      it_ok[i] = (uint8_t)orc_is_valid_state(T, cand + 8 * i, GBP_STANCE, &st);
    }
    int nt = 0;
    for (int i = 0; i < B; i++)
      if (it_ok[i]) memcpy(tgt + 8 * nt++, cand + 8 * i, 64);
    out->targets += nt;
    out->extends += nt;
    /* extend every target against the snapshot (rrt.cpp:77-102, planner_class.cpp:185-200) */
    const int n0 = Tt->n;
    if (Tt->n + nt > Tt->cap) { rc = -2; break; }
    int n_added = 0;
    OMP_FOR
    for (int i = 0; i < nt; i++) {
      const double *q = tgt + 8 * i;
      const int nn = orc_nearest(Tt->v, n0, q, 0);
      const double *s_near = Tt->v + 8 * (int64_t)nn;
      double nrm[3], acts[60];
      int ood = 0, ch;
      uint32_t cnt;
      orc_surface_normal(T, q[0], q[1], nrm, &ood);
      for (int j = 0; j < NUM_GEN_STATES; j++)
        sample_action_any(nrm, dir, cfg->action_flag, cfg->action_p, q, s_near, cfg->seed,
                          EXTD_STREAM, (ext + i) * 8 + j, acts + 10 * j);
      it_r[i] = orc_extend(T, s_near, q, acts, dir, cfg->adaptive, it_sn + 8 * (int64_t)i,
                           it_an + 10 * (int64_t)i, &ch, &cnt);
      it_nn[i] = nn;
      it_chk[i] = ch >= 0 ? ch + 1 : NUM_GEN_STATES;
    }
    for (int i = 0; i < nt; i++) {  /* in target order */
      const int nn = it_nn[i];
      const double *s_near = Tt->v + 8 * (int64_t)nn;
      const double *sn = it_sn + 8 * (int64_t)i, *an = it_an + 10 * (int64_t)i;
      out->attempts += it_chk[i];
      if (it_r[i] == GBP_TRAPPED) continue;
      const int idx = Tt->n;
      tree_put(Tt, sn, an, -1, 0.0, 0.0);
      if (!star) { /* rrt.cpp:86-92 */
        tree_add_edge(Tt, nn, idx);
        tree_update_gy(Tt, idx, Tt->g[nn] + orc_pose_distance(s_near, sn),
                       Tt->y[nn] + orc_state_yaw_distance(s_near, sn));
      }
      added[n_added] = idx;
      nearest[n_added] = nn;
      memcpy(a_ext + 10 * n_added, an, 10 * sizeof(double));
      n_added++;
    }
    ext += nt;
    if (star) {
      for (int i = 0; i < n_added; i++)
        star_insert(T, Tt, added[i], nearest[i], a_ext + 10 * i, cfg->star_delta, dir, cfg->adaptive,
                    cfg->star_order, out);
    }
    /* connect each new vertex to the other tree (rrt_connect.cpp:98-120) */
    const int m0 = O->n;
    if (O->n + n_added > O->cap) { rc = -2; break; }
    int meet = 0;
    OMP_FOR
    for (int i = 0; i < n_added; i++) {
      const double *q = Tt->v + 8 * (int64_t)added[i];
      const int nn = orc_nearest(O->v, m0, q, 0);
      const double *s_ex = O->v + 8 * (int64_t)nn;
      double *sn = it_sn + 8 * (int64_t)i, *an = it_an + 10 * (int64_t)i;
      memset(sn, 0, 8 * sizeof(double));
      memset(an, 0, 10 * sizeof(double));
      ac_stats acs = {0, 0};
      it_r[i] = attempt_connect_ts(T, s_ex, q, orc_pose_distance(q, s_ex) / V_NOM, sn, an, cdir,
                                   cfg->adaptive, 0, &acs);
      it_nn[i] = nn;
      it_chk[i] = acs.checks;
      it_cap[i] = acs.capped;
    }
    for (int i = 0; i < n_added; i++) {  /* in order of the new vertices */
      const int nn = it_nn[i], r = it_r[i];
      const double *s_ex = O->v + 8 * (int64_t)nn;
      const double *sn = it_sn + 8 * (int64_t)i, *an = it_an + 10 * (int64_t)i;
      out->connects++;
      out->depth_capped += it_cap[i];
      out->attempts += it_chk[i];
      if (r == GBP_TRAPPED) continue;
      const int idx = O->n;
      tree_put(O, sn, an, -1, 0.0, 0.0);
      tree_add_edge(O, nn, idx);
      tree_update_gy(O, idx, O->g[nn] + orc_pose_distance(s_ex, sn),
                     O->y[nn] + orc_state_yaw_distance(s_ex, sn));
      if (r != GBP_REACHED) continue;
      const int va = k == 0 ? added[i] : idx, vb = k == 0 ? idx : added[i];
      if (!meet && out->meet_a < 0) {
        out->meet_a = va;
        out->meet_b = vb;
        out->meet_half = h;
      }
      meet = 1;
      if (star) {
        if (n_shared == cap_shared) {
          cap_shared = cap_shared ? 2 * cap_shared : 64;
          shared = (double *)realloc(shared, sizeof(double) * 2 * (size_t)cap_shared);
        }
        shared[2 * n_shared] = va;
        shared[2 * n_shared + 1] = vb;
        n_shared++;
        out->solutions++;
      }
    }
    out->halves = h + 1 - h0;
    if (star) {
      /* the cheapest connection so far with the current g values, ranked after
       * each pair of halves (include/gbp_planner.h buildRRTStarConnectBatched) */
      if (k == 1) {
        for (int64_t i = 0; i < n_shared; i++) {
          const int sa = (int)shared[2 * i], sb = (int)shared[2 * i + 1];
          const double c = tr[0].g[sa] + tr[1].g[sb];
          if (c < cost_so_far) {
            cost_so_far = c;
            out->best_a = sa;
            out->best_b = sb;
          }
        }
      }
      continue;
    }
    if (meet) {
      out->found = 1;
      break;
    }
  }
  out->ext_counter = ext;
  out->draws_a = draws[0];
  out->draws_b = draws[1];
  if (star) {
    out->found = n_shared > 0;
    out->best_cost = cost_so_far;
  } else if (out->found) {
    out->path_length = tr[0].g[out->meet_a] + tr[1].g[out->meet_b];
    out->path_yaw = tr[0].y[out->meet_a] + tr[1].y[out->meet_b];
  }
  free(cand);
  free(tgt);
  free(added);
  free(nearest);
  free(a_ext);
  free(shared);
  free(it_nn);
  free(it_r);
  free(it_chk);
  free(it_cap);
  free(it_sn);
  free(it_an);
  free(it_ok);
  return rc;
}

/* std::array<double, 8> == (element-wise double ==) */
static int state_equal(const double *a, const double *b) {
  for (int k = 0; k < 8; k++)
    if (!(a[k] == b[k])) return 0;
  return 1;
}

/* rrt_connect.cpp:139-227: greedy shortcutting from the start — connect s to
 * the farthest later state that attemptConnect(FORWARD) REACHES; when none
 * does, step to the next state with its original action and add to
 * path_cost_ but not to path_length_ (the reference's quirk, :202-215).
 * Returns the new number of states (<= n). */
int orc_post_process_path(const orc_terrain *T, int n, const double *states,
                          const double *actions, int adaptive, double *out_states,
                          double *out_actions, double *path_length, double *path_yaw,
                          double *path_cost) {
  double s[8], s_goal[8], a_new[10] = {0};
  memcpy(s, states, sizeof s);
  memcpy(s_goal, states + 8 * (int64_t)(n - 1), sizeof s_goal);
  int m = 1;
  memcpy(out_states, s, sizeof s);
  double len = 0, yaw = 0, cost = 0;
  while (!state_equal(s, s_goal)) {
    int last = n - 1; /* s_next = state_sequence_copy.back() */
    int old = -1;
    for (;;) {
      const double *s_next = states + 8 * (int64_t)last;
      double dummy[8] = {0};
      const int r = orc_attempt_connect(T, s, s_next, 0.0, dummy, a_new, GBP_FORWARD, adaptive);
      if (r == GBP_REACHED || state_equal(s, s_next)) break;
      old = last;
      last--;
    }
    const double *s_next = states + 8 * (int64_t)last;
    if (!state_equal(s, s_next)) {
      memcpy(out_states + 8 * (int64_t)m, s_next, 64);
      memcpy(out_actions + 10 * (int64_t)(m - 1), a_new, 80);
      m++;
      const double dl = orc_pose_distance(s, s_next), dy = orc_state_yaw_distance(s, s_next);
      len += dl;
      yaw += dy;
      cost += dl;
      memcpy(s, s_next, sizeof s);
    } else {
      const double *s_old = states + 8 * (int64_t)old;
      memcpy(out_states + 8 * (int64_t)m, s_old, 64);
      memcpy(out_actions + 10 * (int64_t)(m - 1), actions + 10 * (int64_t)(old - 1), 80);
      m++;
      const double dl = orc_pose_distance(s, s_old);
      cost += dl;
      memcpy(s, s_old, sizeof s);
    }
  }
  if (path_length) *path_length = len;
  if (path_yaw) *path_yaw = yaw;
  if (path_cost) *path_cost = cost;
  return m;
}
