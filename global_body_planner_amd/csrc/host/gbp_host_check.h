// gbp_host_check.h — host re-decision of FRAGILE attempts (internal to libgbp).
//
// The validity kernels form the body rotation of isValidState without libm
// (gbp_device.h rotation_trig_nolibm), so a decision whose margin is below
// FRAGILE_EPS could differ from the reference's glibc atan2 / cos / sin by an
// ulp.  Those attempts are flagged GBP_F_FRAGILE and re-decided here, on the
// host, with glibc and the reference's expressions (planning_utils.cpp
// :562-635, :645-881; fast_terrain_map.cpp:94-157), compiled by g++ without
// FMA contraction exactly like the reference.  Only flagged attempts ever run
// here: this is the tie-breaker of record, not a CPU path for the batch.
#pragma once

#include <cstdint>
#include <vector>

namespace gbp_host {

struct Terrain {
  int nx = 0, ny = 0;
  std::vector<double> x, y;  // ascending coordinates (FastTerrainMap x_data_, y_data_)
  std::vector<double> z;     // x-major z[ix * ny + iy] (z_data_[ix][iy])
};

struct Acc {
  uint32_t G = 0, V = 0, flags = 0;
};

// planning_utils.cpp:562-635 under the engine's conventions (gbp.h flags:
// OOD for an undefined lookup, NAN, LIMIT); never sets GBP_F_FRAGILE
bool is_valid_state(const Terrain &T, const double s[8], int phase, Acc &acc);

// isValidStateActionPair[Reverse][AdaptiveStepSize] (planning_utils.cpp
// :645-881): writes s_new / t_new only where the reference assigns them and
// reports that in flags (GBP_F_SNEW_SET / GBP_F_TNEW_SET), like the kernels
bool pair_check(const Terrain &T, const double s[8], const double a[10], int direction,
                int adaptive, double s_new[8], double *t_new, uint32_t *flags, uint32_t *counts);

// rrt.cpp:24 / :55-68 stateDistance (planning_utils.cpp:116-127)
double state_distance(const double *q1, const double *q2);
// planning_utils.cpp:106-115
double pose_distance(const double *q1, const double *q2);
// planning_utils.cpp:519-556
bool is_valid_action(const double a[10]);
// rrt_connect.cpp:53-66: the cubic-Hermite stance action from s_start to s_goal
void connect_action(const double *s_start, const double *s_goal, double t_s, double a[10]);
// RRTConnectClass::attemptConnect (rrt_connect.cpp:20-84), its recursion as a
// loop, with the engine's conventions (gbp.h): a failed check that left t_new
// / s_new unassigned is TRAPPED, a connection still open after level max_depth
// is TRAPPED (flags |= GBP_F_DEPTH_CAPPED).  s_new / a_new are written where the
// reference writes them; flags collects the levels' OOD / NAN / LIMIT bits.
int attempt_connect(const Terrain &T, const double *s_existing, const double *s, double t_s,
                    double s_new[8], double a_new[10], int direction, int adaptive, int max_depth,
                    uint32_t *flags);

}  // namespace gbp_host
