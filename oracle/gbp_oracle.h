/*
 * gbp_oracle.h — CPU restatement of the global_body_planner hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the HIP engine is compared
 * against; nothing in the product (global_body_planner_amd/, include/gbp.h's
 * implementation) may link, import or call it.  Only tests/, the smoke() of
 * __graft_entry__.py and bench.py's cpu_baseline leg use it.
 *
 * It restates, in plain C99 (FP64, no FMA contraction, glibc libm for
 * atan2/sin/cos/sqrt exactly like the reference's host build), the reference
 * functions cited on each declaration.  The bracket search is the reference's
 * O(N) linear scan (fast_terrain_map.cpp:101-117) so the CPU baseline timed
 * from it has the reference's cost model; orc_set_scan_mode(1) switches to a
 * bisection that returns the identical bracket (used only to make big parity
 * runs finish quickly).
 *
 * Parity status: the reference's own tests pin nothing (test/
 * test_global_body_planner.cpp asserts 1+1==2) and the reference cannot be
 * compiled here (its headers need ROS / grid_map / Eigen, absent from the
 * image), so bit-level parity against reference *outputs* is UNPINNED; the
 * restatement is pinned against the survey-recorded outputs of the compiled
 * reference in tests/test_oracle_pins.py.  See DESIGN.md.
 */
#ifndef GBP_ORACLE_H
#define GBP_ORACLE_H

#include <stdint.h>
#include "../include/gbp.h" /* flag / enum values only (the ABI contract) */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int nx, ny;
  const double *x, *y;          /* ascending coordinates               */
  const double *z;              /* x-major [nx][ny]: z[ix*ny+iy]       */
  const double *dx, *dy, *dz;   /* x-major, may be NULL => (0,0,1)     */
} orc_terrain;

/* per-check accumulator */
typedef struct {
  uint32_t G;      /* executed getGroundHeight calls  */
  uint32_t V;      /* executed isValidState calls     */
  uint32_t flags;  /* GBP_F_OOD / GBP_F_NAN / GBP_F_FRAGILE */
} orc_stats;

void orc_set_scan_mode(int mode); /* 0 = linear scan (reference), 1 = bisection */
int  orc_get_scan_mode(void);

/* fast_terrain_map.cpp:94-132.  *ood = 1 if no bracket exists (reference UB). */
double orc_ground_height(const orc_terrain *T, double x, double y, int *ood);
/* fast_terrain_map.cpp:135-157 */
int orc_height_is_nan(const orc_terrain *T, double x, double y, int *ood);
/* fast_terrain_map.cpp:160-213 */
void orc_surface_normal(const orc_terrain *T, double x, double y, double n[3], int *ood);

/* planning_utils.cpp:237-277 */
void orc_apply_stance(const double *s, const double *a, double t, double *out);
/* planning_utils.cpp:282-306 */
void orc_apply_flight(const double *s, double t_f, double *out);
/* planning_utils.cpp:324-370 */
void orc_apply_stance_reverse(const double *s, const double *a, double t, double *out);
/* planning_utils.cpp:519-556 */
int orc_is_valid_action(const double *a);
/* planning_utils.cpp:562-635 */
int orc_is_valid_state(const orc_terrain *T, const double *s, int phase, orc_stats *st);

/* planning_utils.cpp:645-881 (direction FORWARD -> isValidStateActionPair,
 * REVERSE -> isValidStateActionPairReverse; adaptive -> *AdaptiveStepSize).
 * s_new / t_new are only written where the reference writes them; the return
 * value is the reference's bool; *flags receives GBP_F_* bits. */
int orc_is_valid_pair(const orc_terrain *T, const double *s, const double *a, int direction,
                      int adaptive, double *s_new, double *t_new, uint32_t *flags,
                      uint32_t *counts);

/* planning_utils.cpp:106-132, planning_utils.h:133-145 */
double orc_pose_distance(const double *q1, const double *q2);
double orc_state_distance(const double *q1, const double *q2);
double orc_state_yaw_distance(const double *q1, const double *q2);

/* planner_class.cpp:185-200 (ties -> lowest index) */
int orc_nearest(const double *verts, int n_vert, const double *q, double *dist);

/* rrt.cpp:20-70 (newConfig) + rrt.cpp:84-101 (acceptance): candidate actions
 * are given explicitly (actions[6][10]).  Returns TRAPPED/ADVANCED/REACHED;
 * *chosen = index of the first valid candidate or -1. */
int orc_extend(const orc_terrain *T, const double *s_near, const double *target,
               const double *actions, int direction, int adaptive, double *s_new,
               double *a_new, int *chosen, uint32_t *counts);

/* rrt_connect.cpp:20-91 (attemptConnect, recursive).  Returns TRAPPED/ADVANCED/
 * REACHED; t_s <= 0 means "compute from poseDistance / V_NOM" (:85-91). */
int orc_attempt_connect(const orc_terrain *T, const double *s_existing, const double *s,
                        double t_s, double *s_new, double *a_new, int direction,
                        int adaptive);

/* ---- batch helpers (OpenMP over independent items, nthreads <= 0 => 1) --- */
void orc_validate_pairs(const orc_terrain *T, int64_t n, const double *s, const double *a,
                        const uint8_t *direction, int direction_all, int adaptive,
                        uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                        uint32_t *counts, int nthreads);
void orc_valid_states(const orc_terrain *T, int64_t n, const double *states,
                      const uint8_t *phase, int phase_all, uint8_t *valid, uint32_t *flags,
                      uint32_t *counts, int nthreads);
void orc_height_batch(const orc_terrain *T, int64_t n, const double *xy, double *h,
                      uint8_t *is_nan, uint8_t *ood, int nthreads);
void orc_normal_batch(const orc_terrain *T, int64_t n, const double *xy, double *nrm,
                      uint8_t *ood, int nthreads);
void orc_extend_batch(const orc_terrain *T, int64_t n, const double *s_near,
                      const double *target, const double *actions /* n*6*10 */,
                      const uint8_t *direction, int direction_all, int adaptive,
                      int32_t *result, int32_t *chosen, double *s_new, double *a_new,
                      uint32_t *counts, int nthreads);
void orc_nearest_batch(int64_t n_q, const double *q, int n_vert, const double *verts,
                       int32_t *idx, double *dist, int nthreads);
/* planner_class.cpp:173-182 in the vertex map's iteration order (see
 * orc_um_order); the _ordered form takes order 1 = ascending index */
void orc_neighbors_batch(int64_t n_q, const double *q, int n_vert, const double *verts,
                         double radius, int max_out, int32_t *out, int32_t *count, int nthreads);
void orc_neighbors_batch_ordered(int64_t n_q, const double *q, int n_vert, const double *verts,
                                 double radius, int max_out, int32_t *out, int32_t *count,
                                 int order, int nthreads);
/* libstdc++ std::unordered_map<int, State> filled with keys 0..n-1
 * (graph_class.cpp:28-31): key k's position when iterated, and all n keys in
 * iteration order */
int64_t orc_um_rank(int64_t k, int64_t n);
void orc_um_order(int64_t n, int32_t *out);

/* planner_class.cpp:151-171 (neighborhoodN): ascending (distance, index) */
/* planning_utils.h:146-155 and neighborhoodN with cost_add_yaw (glibc atan2) */
double orc_state_distance_yaw(const double *q1, const double *q2, int flag, double lw, double yw);
void orc_knn_yaw_batch(int64_t n_q, const double *q, int n_vert, const double *verts, int n_nearest,
                       int flag, double lw, double yw, int32_t *out, double *dist, int nthreads);
void orc_knn_batch(int64_t n_q, const double *q, int n_vert, const double *verts, int n_nearest,
                   int32_t *out, double *dist, int nthreads);

/* ---- counter-based samplers (Philox4x32-10), same keys as the engine ---- */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* uniform in [0,1): (hi:lo >> 11) * 2^-53 for each of the two 64-bit halves */
void orc_uniform2(uint64_t seed, uint64_t stream_id, uint32_t purpose, int64_t index,
                  uint32_t draw, double u[2]);
/* planner_class.cpp:38-76; returns number of tries (k+1) or -1 */
int orc_sample_state(const orc_terrain *T, uint64_t seed, uint64_t stream_id, int64_t index,
                     int require_phase, int max_tries, double *state);
/* planning_utils.cpp:392-442 */
void orc_sample_action(const double *normal, uint64_t seed, uint64_t stream_id, int64_t index,
                       double *action);
/* planning_utils.cpp:198-231 */
void orc_rotate_grf(const double *n, const double *f, double *out);
void orc_sample_states(const orc_terrain *T, int64_t n, uint64_t seed, uint64_t stream_id,
                       int64_t index_base, int require_phase, int max_tries, double *states,
                       int32_t *tries, int nthreads);
void orc_sample_actions(int64_t n, const double *normals, uint64_t seed, uint64_t stream_id,
                        int64_t index_base, double *actions, int nthreads);
/* direction-biased sampling (the engine's gbp_sampling; coin = uniform of purpose 3).
 * planner_class.cpp:22-35 + :82-148, one try of each index (s_from / s_to shared) */
void orc_sample_states_dir(const orc_terrain *T, int64_t n, uint64_t seed, uint64_t stream_id,
                           int64_t index_base, int state_flag, double state_p, int speed_direction,
                           const double *s_from, const double *s_to, double *states, int nthreads);
/* planning_utils.cpp:379-391 + :443-515: s[n][8] the state extended toward, s_near[n][8] */
void orc_sample_actions_dir(int64_t n, const double *normals, const double *s,
                            const double *s_near, const uint8_t *direction, int direction_all,
                            int action_flag, double action_p, uint64_t seed, uint64_t stream_id,
                            int64_t index_base, double *actions, int nthreads);

/* ---- the planner loop (batch-synchronous RRT-Connect / RRT*-Connect) ---- */
typedef struct {
  int cap;          /* rows of every array below                          */
  int n;            /* vertices (set by orc_plan)                         */
  double *v;        /* [cap][8] states                                    */
  double *a;        /* [cap][10] the action reaching each vertex (root 0) */
  int32_t *parent;  /* [cap] (root -1)                                    */
  double *g, *y;    /* [cap] cost / yaw to come (graph_class.cpp:36-42)   */
  int32_t *child, *sibling; /* [cap] successor lists (RRT* rewiring), may be NULL for RRT-Connect */
} orc_tree;

typedef struct {
  int batch;                 /* targets per half-iteration (1 = runRRTConnect)        */
  uint64_t seed, stream_a, stream_b; /* the trees' target streams                     */
  int adaptive;              /* adaptive-step pair checks (params.yaml:16)             */
  int state_flag, state_speed_direction, action_flag; /* gbp_sampling                 */
  double state_p, action_p;
  int64_t extend_base;       /* the first extend's index on the candidate stream       */
  int64_t max_halves;        /* stop after this many half-iterations (<= 0: at a solution) */
  int star;                  /* RRT*-Connect: choose-parent + rewire, runs max_halves  */
  double star_delta;         /* rrt_star_connect.h:59 (3.0)                            */
  int nthreads;              /* OpenMP threads for the per-item passes (<= 1: serial;   */
                             /* results identical: insertion stays in order)           */
  int64_t first_half;        /* warm start: the first half-iteration (draw indices)    */
  int warm;                  /* warm start: tr[k].n vertices given (v, a, parent; root  */
                             /* first, parents before children — RRT*: any tree rooted */
                             /* at 0), g / y derived                                   */
  int star_order;            /* RRT* neighbourhoods: 0 the vertex map's iteration order */
                             /* (the reference), 1 ascending index (tests only)        */
} orc_plan_cfg;

typedef struct {
  int found;
  int meet_a, meet_b;        /* RRT-Connect: the vertices the first REACHED connect joined */
  int64_t meet_half, halves;
  int64_t targets, extends, attempts, connects, depth_capped, rewires, solutions;
  int64_t ext_counter, draws_a, draws_b;
  double path_length, path_yaw;  /* g / y of the meeting vertices (rrt_connect.cpp:304-313) */
  int best_a, best_b;        /* RRT*: the cheapest connection ranked after each iteration */
  double best_cost;
} orc_plan_out;

/* one RRT* insertion (rrt_star_connect.cpp:18-66): t holds vertices 0..idx
 * (v), the parents of 0..idx-1 (a tree rooted at 0; g / y and the successor
 * lists are derived), vertex idx newly added with nearest vertex nn and
 * newConfig's action a_new; choose-parent and rewire update t's parent / a /
 * g / y in place.  order: 0 the vertex map's iteration order, 1 ascending
 * index.  Returns 0 or -1 (bad arguments). */
int orc_star_insert_one(const orc_terrain *T, orc_tree *t, int idx, int nn, const double *a_new,
                        double delta, int direction, int adaptive, int order, int64_t *rewires);

/* diagnostics of the RRT* insertions run so far (process-wide, serial):
 * [insertions, neighbours, max neighbours, rewires, subtree vertices updated,
 * largest subtree, summed subtree depths, deepest subtree]; reset clears */
void orc_star_stats(int64_t out[8], int reset);

/* tr[0] = Ta (start, FORWARD), tr[1] = Tb (goal, REVERSE); returns 0, -1 (bad
 * arguments) or -2 (a tree's capacity is exhausted) */
int orc_plan(const orc_terrain *T, const double *start, const double *goal,
             const orc_plan_cfg *cfg, orc_tree *tr, orc_plan_out *out);
/* rrt_connect.cpp:139-227 (FORWARD attemptConnect, cost without yaw terms);
 * out_states[n][8], out_actions[n-1][10]; returns the new state count */
int orc_post_process_path(const orc_terrain *T, int n, const double *states,
                          const double *actions, int adaptive, double *out_states,
                          double *out_actions, double *path_length, double *path_yaw,
                          double *path_cost);

/* the samplers' reproducible transcendentals (restating gbp_device.h rm_*):
 * fn 0 log(x), 1 sincos(x) -> out[2n] (sin, cos), 2 atan2(y, x), 3 acos(x) */
void orc_rmath(int fn, int64_t n, const double *x, const double *y, double *out);

#ifdef __cplusplus
}
#endif
#endif
