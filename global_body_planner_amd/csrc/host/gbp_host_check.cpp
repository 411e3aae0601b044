// gbp_host_check.cpp — glibc re-decision of FRAGILE attempts (see the header).
// Built with g++ -O2 -ffp-contract=off: the reference's x86-64 arithmetic, the
// reference's libm.  Every function follows the reference source line by line;
// the only departures are the engine conventions every engine path shares
// (gbp.h): an undefined out-of-map lookup makes the state invalid (GBP_F_OOD),
// a check is stopped after GBP_MAX_SAMPLES states (GBP_F_LIMIT).
#include "gbp_host_check.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "gbp.h"

namespace gbp_host {
namespace {

// planning_utils.h:21-66
constexpr double H_MAX = 0.4, H_MIN = 0.075, V_MAX = 2.0, P_MAX = 1.0;
constexpr double ROBOT_L = 0.3, ROBOT_W = 0.3, ROBOT_H = 0.05;
constexpr double KINEMATICS_RES = 0.05, BACKUP_RATIO = 0.5;

constexpr int NO_BRACKET_LOW = -1;   // v < d[0] or NaN: the scan never matches, index 0
constexpr int NO_BRACKET_HIGH = -2;  // v >= d[n-1]: the scan reads d[n] (undefined)

// fast_terrain_map.cpp:101-117: the first i with d[i] <= v < d[i+1]; for an
// ascending vector that is the last i with d[i] <= v, if v < d[n-1]
int bracket(const std::vector<double> &d, double v) {
  const int n = (int)d.size();
  if (!(v >= d[0])) return NO_BRACKET_LOW;
  if (v >= d[n - 1]) return NO_BRACKET_HIGH;
  return (int)(std::upper_bound(d.begin(), d.end(), v) - d.begin()) - 1;
}

double zc(const Terrain &T, int ix, int iy) { return T.z[(size_t)ix * T.ny + iy]; }

// fast_terrain_map.cpp:135-157; -1 = undefined (a scan read past the end)
int height_is_nan(const Terrain &T, double x, double y) {
  const int ix = bracket(T.x, x), iy = bracket(T.y, y);
  if (ix == NO_BRACKET_HIGH || iy == NO_BRACKET_HIGH) return -1;
  const int cx = ix < 0 ? 0 : ix, cy = iy < 0 ? 0 : iy;
  return (std::isnan(zc(T, cx, cy)) || std::isnan(zc(T, cx, cy + 1)) ||
          std::isnan(zc(T, cx + 1, cy)) || std::isnan(zc(T, cx + 1, cy + 1)))
             ? 1
             : 0;
}

// fast_terrain_map.cpp:94-132; false = undefined (finite point with no bracket)
bool ground_height(const Terrain &T, double x, double y, double &h) {
  if (std::isnan(x) || std::isnan(y)) {  // every term is NaN whatever x1..y2 hold
    h = NAN;
    return true;
  }
  const int ix = bracket(T.x, x), iy = bracket(T.y, y);
  if (ix < 0 || iy < 0) return false;
  const double x1 = T.x[ix], x2 = T.x[ix + 1], y1 = T.y[iy], y2 = T.y[iy + 1];
  const double fx1y1 = zc(T, ix, iy), fx1y2 = zc(T, ix, iy + 1);
  const double fx2y1 = zc(T, ix + 1, iy), fx2y2 = zc(T, ix + 1, iy + 1);
  h = 1.0 / ((x2 - x1) * (y2 - y1)) *
      (fx1y1 * (x2 - x) * (y2 - y) + fx2y1 * (x - x1) * (y2 - y) + fx1y2 * (x2 - x) * (y - y1) +
       fx2y2 * (x - x1) * (y - y1));
  return true;
}

// planning_utils.cpp:237-274
void apply_stance(const double *s, const double *a, double t, double *o) {
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  double r[8];
  r[0] = s[0] + s[3] * t + 0.5 * a_x_td * t * t + (a_x_to - a_x_td) * (t * t * t) / (6.0 * t_s);
  r[1] = s[1] + s[4] * t + 0.5 * a_y_td * t * t + (a_y_to - a_y_td) * (t * t * t) / (6.0 * t_s);
  r[2] = s[2] + s[5] * t + 0.5 * a_z_td * t * t + (a_z_to - a_z_td) * (t * t * t) / (6.0 * t_s);
  r[3] = s[3] + a_x_td * t + (a_x_to - a_x_td) * t * t / (2.0 * t_s);
  r[4] = s[4] + a_y_td * t + (a_y_to - a_y_td) * t * t / (2.0 * t_s);
  r[5] = s[5] + a_z_td * t + (a_z_to - a_z_td) * t * t / (2.0 * t_s);
  r[6] = s[6] + s[7] * t + 0.5 * a_p_td * t * t + (a_p_to - a_p_td) * (t * t * t) / (6.0 * t_s);
  r[7] = s[7] + a_p_td * t + (a_p_to - a_p_td) * t * t / (2.0 * t_s);
  std::memcpy(o, r, sizeof r);
}

// planning_utils.cpp:282-306 (the literal 9.81)
void apply_flight(const double *s, double t_f, double *o) {
  const double g = 9.81;
  double r[8];
  r[0] = s[0] + s[3] * t_f;
  r[1] = s[1] + s[4] * t_f;
  r[2] = s[2] + s[5] * t_f - 0.5 * g * t_f * t_f;
  r[3] = s[3];
  r[4] = s[4];
  r[5] = s[5] - g * t_f;
  r[6] = s[6] + s[7] * t_f;
  r[7] = s[7];
  std::memcpy(o, r, sizeof r);
}

// planning_utils.cpp:324-367 (s_new[7] before s_new[6], as written)
void apply_stance_reverse(const double *s, const double *a, double t, double *o) {
  const double a_x_td = a[0], a_y_td = a[1], a_z_td = a[2];
  const double a_x_to = a[3], a_y_to = a[4], a_z_to = a[5];
  const double t_s = a[6], a_p_td = a[8], a_p_to = a[9];
  const double x_to = s[0], y_to = s[1], z_to = s[2], dx_to = s[3], dy_to = s[4], dz_to = s[5];
  const double p_to = s[6], dp_to = s[7];
  const double c_x = dx_to - a_x_td * t_s - 0.5 * (a_x_to - a_x_td) * t_s;
  const double c_y = dy_to - a_y_td * t_s - 0.5 * (a_y_to - a_y_td) * t_s;
  const double c_z = dz_to - a_z_td * t_s - 0.5 * (a_z_to - a_z_td) * t_s;
  const double c_p = dp_to - a_p_td * t_s - 0.5 * (a_p_to - a_p_td) * t_s;
  double r[8];
  r[0] = x_to - c_x * (t_s - t) - 0.5 * a_x_td * (t_s * t_s - t * t) -
         (a_x_to - a_x_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[1] = y_to - c_y * (t_s - t) - 0.5 * a_y_td * (t_s * t_s - t * t) -
         (a_y_to - a_y_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[2] = z_to - c_z * (t_s - t) - 0.5 * a_z_td * (t_s * t_s - t * t) -
         (a_z_to - a_z_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  r[3] = dx_to - a_x_td * (t_s - t) - (a_x_to - a_x_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[4] = dy_to - a_y_td * (t_s - t) - (a_y_to - a_y_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[5] = dz_to - a_z_td * (t_s - t) - (a_z_to - a_z_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[7] = dp_to - a_p_td * (t_s - t) - (a_p_to - a_p_td) * (t_s * t_s - t * t) / (2.0 * t_s);
  r[6] = p_to - c_p * (t_s - t) - 0.5 * a_p_td * (t_s * t_s - t * t) -
         (a_p_to - a_p_td) * (t_s * t_s * t_s - t * t * t) / (6.0 * t_s);
  std::memcpy(o, r, sizeof r);
}

void set_stage(uint32_t &f, uint32_t k) {
  f = (f & ~GBP_F_STAGE_MASK) | (k << GBP_F_STAGE_SHIFT);
}

void assign(double *dst, const double *src) { std::memcpy(dst, src, 8 * sizeof(double)); }

bool small_step(double time_step) {  // planning_utils.cpp:662 / :795
  return KINEMATICS_RES - 0.01 <= time_step && time_step <= KINEMATICS_RES + 0.01;
}

// planning_utils.cpp:651-753: the plain loop is the adaptive one with the step
// pinned to KINEMATICS_RES (time_step never grows, every failure backs up)
bool pair_forward(const Terrain &T, const double *s, const double *a, bool adaptive,
                  double *s_new, double *t_new, Acc &acc, uint32_t &f) {
  const double t_s = a[6], t_f = a[7];
  double sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  set_stage(f, GBP_STAGE_FWD_STANCE);
  for (double t = 0; t <= t_s; t += time_step) {
    apply_stance(s, a, t, sc);
    if (!is_valid_state(T, sc, GBP_STANCE, acc)) {
      if (acc.flags & GBP_F_LIMIT) return false;
      if (!adaptive || small_step(time_step)) {
        apply_stance(s, a, (1.0 - BACKUP_RATIO) * t, s_new);
        f |= GBP_F_SNEW_SET;
        return false;
      }
      time_step = KINEMATICS_RES;
      t = t_pre_success;
    } else {
      assign(s_new, sc);
      *t_new = t;
      f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      if (adaptive) {
        time_step += KINEMATICS_RES;
        t_pre_success = t;
      }
    }
  }
  double s_takeoff[8];
  apply_stance(s, a, a[6], s_takeoff);
  time_step = KINEMATICS_RES;
  set_stage(f, GBP_STAGE_FWD_FLIGHT);
  for (double t = 0; t < t_f; t += time_step) {
    apply_flight(s_takeoff, t, sc);
    if (!is_valid_state(T, sc, GBP_FLIGHT, acc)) return false;
    if (adaptive) time_step += KINEMATICS_RES;
  }
  set_stage(f, GBP_STAGE_FWD_LAND);
  apply_flight(s_takeoff, t_f, sc);
  if (!is_valid_state(T, sc, GBP_STANCE, acc)) return false;
  assign(s_new, sc);
  *t_new = t_s + t_f;
  f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return true;
}

// planning_utils.cpp:774-876
bool pair_reverse(const Terrain &T, const double *s, const double *a, bool adaptive,
                  double *s_new, double *t_new, Acc &acc, uint32_t &f) {
  const double t_s = a[6], t_f = a[7];
  double sc[8];
  double time_step = KINEMATICS_RES, t_pre_success = 0;
  set_stage(f, GBP_STAGE_REV_FLIGHT);
  for (double t = 0; t < t_f; t += time_step) {
    apply_flight(s, -t, sc);
    if (!is_valid_state(T, sc, GBP_FLIGHT, acc)) return false;
    if (adaptive) time_step += KINEMATICS_RES;
  }
  double s_takeoff[8];
  apply_flight(s, -t_f, s_takeoff);
  time_step = KINEMATICS_RES;
  set_stage(f, GBP_STAGE_REV_STANCE);
  for (double t = t_s; t >= 0; t -= time_step) {
    apply_stance_reverse(s_takeoff, a, t, sc);
    if (!is_valid_state(T, sc, GBP_STANCE, acc)) {
      if (acc.flags & GBP_F_LIMIT) return false;
      if (!adaptive || small_step(time_step)) {
        apply_stance(s, a, t + BACKUP_RATIO * (t_s - t), s_new);  // forward stance, as written (:857)
        f |= GBP_F_SNEW_SET;
        return false;
      }
      time_step = KINEMATICS_RES;
      t = t_pre_success;
    } else {
      assign(s_new, sc);
      *t_new = t_s - t;
      f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
      if (adaptive) {
        time_step += KINEMATICS_RES;
        t_pre_success = t;
      }
    }
  }
  set_stage(f, GBP_STAGE_REV_START);
  apply_stance_reverse(s_takeoff, a, 0, sc);
  if (!is_valid_state(T, sc, GBP_STANCE, acc)) return false;
  assign(s_new, sc);
  *t_new = t_s;
  f |= GBP_F_SNEW_SET | GBP_F_TNEW_SET;
  return true;
}

}  // namespace

bool is_valid_state(const Terrain &T, const double s[8], int phase, Acc &acc) {
  if (acc.V >= GBP_MAX_SAMPLES) {  // engine guard (gbp.h GBP_F_LIMIT)
    acc.flags |= GBP_F_LIMIT;
    return false;
  }
  acc.V++;
  const double x0 = T.x.front(), xN = T.x.back(), y0 = T.y.front(), yN = T.y.back();
  // :564 heightIsNan(centre); an undefined read matters only where (2) passes
  const int r = height_is_nan(T, s[0], s[1]);
  if (r < 0) {
    if (!(s[0] < x0 || s[0] > xN || s[1] < y0 || s[1] > yN)) acc.flags |= GBP_F_OOD;
    return false;
  }
  if (r) {
    acc.flags |= GBP_F_NAN;
    return false;
  }
  // :568-571 (abs resolves to the double overload)
  if ((s[0] < x0) || (s[0] > xN) || (s[1] < y0) || (s[1] > yN) || (std::fabs(s[6]) >= P_MAX))
    return false;
  // :574
  if (std::sqrt(s[3] * s[3] + s[4] * s[4]) > V_MAX) return false;
  // :578-594
  const double yaw = std::atan2(s[4], s[3]);
  const double cy = std::cos(yaw);
  const double sy = std::sin(yaw);
  const double pitch = s[6];
  const double cp = std::cos(pitch);
  const double sp = std::sin(pitch);
  const double R_11 = cy * cp, R_12 = -sy, R_13 = cy * sp;
  const double R_21 = sy * cp, R_22 = cy, R_23 = sy * sp;
  const double R_31 = -sp, R_32 = 0, R_33 = cp;
  const double test_x[2] = {-0.5 * ROBOT_L, 0.5 * ROBOT_L};
  const double test_y[2] = {-0.5 * ROBOT_W, 0.5 * ROBOT_W};
  const double z_body = -ROBOT_H;
  // :601-627
  for (double x_body : test_x) {
    for (double y_body : test_y) {
      const double x_leg = s[0] + R_11 * x_body + R_12 * y_body;
      const double y_leg = s[1] + R_21 * x_body + R_22 * y_body;
      const double z_leg = s[2] + R_31 * x_body + R_32 * y_body;
      const double x_corner = x_leg + R_13 * z_body;
      const double y_corner = y_leg + R_23 * z_body;
      const double z_corner = z_leg + R_33 * z_body;
      const int rl = height_is_nan(T, x_leg, y_leg);
      if (rl < 0) {
        acc.flags |= GBP_F_OOD;
        return false;
      }
      if (rl) {
        acc.flags |= GBP_F_NAN;
        return false;
      }
      acc.G += 2;  // both heights are computed before the test (:618-619)
      double gl, gc;
      if (!ground_height(T, x_leg, y_leg, gl) || !ground_height(T, x_corner, y_corner, gc)) {
        acc.flags |= GBP_F_OOD;
        return false;
      }
      const double leg_height = z_leg - gl;
      const double corner_height = z_corner - gc;
      if ((corner_height < H_MIN) || ((phase == GBP_STANCE) && (leg_height > H_MAX))) return false;
    }
  }
  // :630-632
  acc.G++;
  double gu;
  if (!ground_height(T, s[0] + R_13 * z_body, s[1] + R_23 * z_body, gu)) {
    acc.flags |= GBP_F_OOD;
    return false;
  }
  const double height = (s[2] + R_33 * z_body) - gu;
  if (height < H_MIN) return false;
  return true;
}

bool pair_check(const Terrain &T, const double s[8], const double a[10], int direction,
                int adaptive, double s_new[8], double *t_new, uint32_t *flags, uint32_t *counts) {
  Acc acc;
  uint32_t f = 0;
  const bool v = direction == GBP_FORWARD
                     ? pair_forward(T, s, a, adaptive != 0, s_new, t_new, acc, f)
                     : pair_reverse(T, s, a, adaptive != 0, s_new, t_new, acc, f);
  f |= acc.flags | (v ? GBP_F_VALID : 0u);
  if (flags) *flags = f;
  if (counts) *counts = (acc.G & 0xFFFFu) | (acc.V << 16);
  return v;
}

double state_distance(const double *q1, const double *q2) {  // planning_utils.cpp:116-127
  double sum = 0;
  for (int i = 0; i < 8; i++) sum = sum + 1.0 * (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return std::sqrt(sum);
}

double pose_distance(const double *q1, const double *q2) {  // planning_utils.cpp:106-115
  double sum = 0;
  for (int i = 0; i < 3; i++) sum = sum + (q2[i] - q1[i]) * (q2[i] - q1[i]);
  return std::sqrt(sum);
}

bool is_valid_action(const double a[10]) {  // planning_utils.cpp:519-556
  if ((a[6] <= 0) || (a[7] < 0)) return false;
  const double m = 13, g = 9.81, mu = 1.0, f_max = 637;  // M_CONST, G_CONST, MU, F_MAX
  const double f_x_td = m * a[0], f_y_td = m * a[1], f_z_td = m * (a[2] + g);
  const double f_x_to = m * a[3], f_y_to = m * a[4], f_z_to = m * (a[5] + g);
  if ((std::sqrt(f_x_td * f_x_td + f_y_td * f_y_td + f_z_td * f_z_td) >= f_max) ||
      (std::sqrt(f_x_to * f_x_to + f_y_to * f_y_to + f_z_to * f_z_to) >= f_max) || (f_z_td < 0) ||
      (f_z_to < 0) || (a[8] >= f_max) || (a[9] >= f_max))
    return false;
  if ((std::sqrt(f_x_td * f_x_td + f_y_td * f_y_td) >= mu * f_z_td) ||
      (std::sqrt(f_x_to * f_x_to + f_y_to * f_y_to) >= mu * f_z_to))
    return false;
  return true;
}

void connect_action(const double *s_start, const double *s_goal, double t_s, double a[10]) {
  const double x_td = s_start[0], y_td = s_start[1], z_td = s_start[2];  // rrt_connect.cpp:33-51
  const double dx_td = s_start[3], dy_td = s_start[4], dz_td = s_start[5];
  const double x_to = s_goal[0], y_to = s_goal[1], z_to = s_goal[2];
  const double dx_to = s_goal[3], dy_to = s_goal[4], dz_to = s_goal[5];
  const double p_td = s_start[6], dp_td = s_start[7], p_to = s_goal[6], dp_to = s_goal[7];
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

int attempt_connect(const Terrain &T, const double *s_existing, const double *s0, double t_s,
                    double s_new[8], double a_new[10], int direction, int adaptive, int max_depth,
                    uint32_t *flags) {
  double s[8];
  std::memcpy(s, s0, sizeof s);
  uint32_t fl = 0;
  int result = GBP_TRAPPED;
  for (int depth = 0;; depth++) {
    if (depth > max_depth) {  // engine convention: the reference recursion is unbounded
      fl |= GBP_F_DEPTH_CAPPED;
      break;
    }
    if (t_s <= KINEMATICS_RES) break;  // :23-24
    const double *s_start = direction == GBP_FORWARD ? s_existing : s;
    const double *s_goal = direction == GBP_FORWARD ? s : s_existing;
    connect_action(s_start, s_goal, t_s, a_new);
    if (!is_valid_action(a_new)) break;  // :66, :83
    double sn[8], tn = 0;
    uint32_t f = 0;
    const bool ok = pair_check(T, direction == GBP_FORWARD ? s_start : s_goal, a_new, direction,
                               adaptive, sn, &tn, &f, nullptr);
    fl |= f & (GBP_F_OOD | GBP_F_NAN | GBP_F_LIMIT);
    if (f & GBP_F_SNEW_SET) std::memcpy(s_new, sn, sizeof sn);
    if (ok) {
      result = depth == 0 ? GBP_REACHED : GBP_ADVANCED;  // :74-75, :79-80
      break;
    }
    // :77 recurse toward the returned state; unassigned t_new / s_new: TRAPPED
    if (!(f & GBP_F_TNEW_SET) || !(f & GBP_F_SNEW_SET)) break;
    std::memcpy(s, sn, sizeof s);
    t_s = tn;
  }
  if (flags) *flags = fl;
  return result;
}

}  // namespace gbp_host

// the reference's yaw of a state with glibc (planning_utils.h:135-136), for the
// device's yaw-weighted k-nearest (gbp_knn_yaw_batch_dev takes the yaws)
extern "C" __attribute__((visibility("default"))) double gbp_host_yaw(const double *s) {
  return std::atan2(s[4], s[3]);
}
