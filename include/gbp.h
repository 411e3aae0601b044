/*
 * gbp.h — C ABI of the MI355X batched RRT-Connect extend/validity engine.
 *
 * This is the drop-in boundary for the hot path of LiuShenLan/global_body_planner
 * (reference snapshot 2025-02-04).  Every entry point below replaces one reference
 * C++ interface; the reference file:line it stands in for is cited on each.
 *
 *   - plain C: opaque handles, int status codes (GBP_OK = 0, < 0 = error), no
 *     exceptions cross this boundary, no torch / HIP types in the signatures
 *     (a stream is passed as an opaque `void*` = hipStream_t, NULL = default).
 *   - State  = double[8]  {x, y, z, dx, dy, dz, p, dp}   (planning_utils.h:57-61)
 *   - Action = double[10] {a_x_td, a_y_td, a_z_td, a_x_to, a_y_to, a_z_to,
 *                          t_s, t_f, a_p_td, a_p_to}     (planning_utils.h:58-62)
 *     Batches are AoS `double[n][8]` / `double[n][10]`, i.e. exactly the
 *     std::array layout, so a std::vector<State> can be passed as-is.
 *   - All arithmetic is IEEE FP64 in the reference operation order, compiled
 *     without FMA contraction, so decisions are bit-exact with the reference
 *     algorithm (see DESIGN.md "Parity").
 *   - `_dev` entry points take DEVICE pointers and enqueue on `stream`
 *     (asynchronous); `_host` entry points take host pointers and block.
 *   - A handle is used by one host thread at a time; there is no global mutable
 *     state, so distinct handles (e.g. one per GPU) are fully reentrant.
 */
#ifndef GBP_H
#define GBP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define GBP_OK              0
#define GBP_E_INVALID_ARG  (-1)
#define GBP_E_BAD_HANDLE   (-2)
#define GBP_E_ALLOC        (-3)
#define GBP_E_HIP          (-4)
#define GBP_E_SHAPE        (-5)
#define GBP_E_NO_DEVICE    (-6)
#define GBP_E_UNSUPPORTED  (-7)

/* ---- reference enums (planning_utils.h:50-54, rrt.h:7-9) ---------------- */
#define GBP_FLIGHT          0
#define GBP_STANCE          1
#define GBP_CONNECT_STANCE  2
#define GBP_FORWARD         0
#define GBP_REVERSE         1
#define GBP_TRAPPED         0
#define GBP_ADVANCED        1
#define GBP_REACHED         2

#define GBP_STATE_DIM       8
#define GBP_ACTION_DIM     10
#define GBP_NUM_GEN_STATES  6   /* planning_utils.h:45 */
/* attemptConnect (rrt_connect.cpp:20-84) recurses without a bound; the
 * engine stops a connection after this many levels and reports it TRAPPED
 * (counted as depth_capped).  Each level's stance time shrinks by >= one
 * KINEMATICS_RES step except in degenerate reverse cases, so a cap of 1024
 * covers t_s up to 51 s (a 38 m connect at V_NOM) without truncation.      */
#define GBP_CONNECT_MAX_DEPTH 1024

/* ---- per-attempt flag word (output of the validate/extend entry points) -- */
#define GBP_F_VALID      (1u << 0)  /* the pair check returned true                      */
#define GBP_F_OOD        (1u << 1)  /* a lookup whose reference result is UB (point outside
                                       [x_0,x_{N-1}) x [y_0,y_{N-1}), fast_terrain_map.cpp:96-117)
                                       was reached; by this engine's convention the state is
                                       invalid (DESIGN.md "Out-of-domain convention")       */
#define GBP_F_NAN        (1u << 2)  /* a state failed on a NaN terrain cell                 */
#define GBP_F_SNEW_SET   (1u << 3)  /* the reference assigned s_new (else buffer untouched) */
#define GBP_F_TNEW_SET   (1u << 4)  /* the reference assigned t_new (else buffer untouched) */
#define GBP_F_FRAGILE    (1u << 5)  /* a trig-dependent comparison was within 1e-12 of its
                                       threshold (decision could differ across libm builds) */
#define GBP_F_LIMIT      (1u << 6)  /* the pair needed more than GBP_MAX_SAMPLES state checks
                                       (t_s + t_f > ~350 s, e.g. a connect longer than ~262 m at
                                       V_NOM, or t_s = inf where the reference never
                                       terminates); the check is stopped and reported invalid.
                                       The cap keeps G = 9 V below the 16-bit counter field. */
#define GBP_F_RESOLVED   (1u << 7)  /* a FRAGILE attempt whose outputs were re-decided on the
                                       host with glibc trig (gbp_resolve_fragile_host)        */
#define GBP_MAX_SAMPLES  7000u
#define GBP_F_DEPTH_CAPPED (1u << 12) /* a connect stopped at GBP_CONNECT_MAX_DEPTH (TRAPPED) */
#define GBP_F_STAGE_SHIFT 8u        /* bits 8..11: stage in which the check ended          */
#define GBP_F_STAGE_MASK  (0xFu << GBP_F_STAGE_SHIFT)
#define GBP_STAGE_FWD_STANCE 1u     /* planning_utils.cpp:718-730 */
#define GBP_STAGE_FWD_FLIGHT 2u     /* :735-741 */
#define GBP_STAGE_FWD_LAND   3u     /* :743-749 */
#define GBP_STAGE_REV_FLIGHT 4u     /* :842-847 */
#define GBP_STAGE_REV_STANCE 5u     /* :852-863 */
#define GBP_STAGE_REV_START  6u     /* :866-872 */

/* lookup counters: counts[i] = G | (V << 16), G = executed getGroundHeight calls,
   V = executed isValidState calls (reference semantics).         */
#define GBP_COUNT_G(c) ((c) & 0xFFFFu)
#define GBP_COUNT_V(c) ((c) >> 16)

/* ---- opaque handles ------------------------------------------------------ */
typedef struct gbp_terrain gbp_terrain;
typedef void *gbp_stream; /* hipStream_t; NULL = the device's null stream */

/* ---- library / device ---------------------------------------------------- */
int         gbp_version(void);                 /* 10000*major + 100*minor + patch */
const char *gbp_status_string(int status);
int         gbp_device_count(int *count);
int         gbp_device_alloc(int device, size_t bytes, void **ptr);
int         gbp_device_free(void *ptr);
int         gbp_memcpy_h2d(void *dst, const void *src, size_t bytes, gbp_stream stream);
int         gbp_memcpy_d2h(void *dst, const void *src, size_t bytes, gbp_stream stream);
int         gbp_stream_synchronize(gbp_stream stream);

/* ---- terrain (replaces FastTerrainMap storage + loadData,
 *      fast_terrain_map.h:97-118, fast_terrain_map.cpp:10-28) -------------- */
#define GBP_STORAGE_AUTO 0  /* fp32 if every z value round-trips through float, else fp64 */
#define GBP_STORAGE_F32  1  /* lossless for grid_map-sourced maps (fast_terrain_map.cpp:60) */
#define GBP_STORAGE_F64  2

/* x[nx], y[ny] ascending coordinates; z, dx, dy, dz are x-major [nx][ny]
 * (z[ix*ny + iy] == z_data_[ix][iy]).  dx/dy/dz may be NULL => (0, 0, 1),
 * as loadDataFromGridMap does for maps without slope layers (:70-74). */
int gbp_terrain_create(int device, int nx, int ny, const double *x, const double *y,
                       const double *z, const double *dx, const double *dy,
                       const double *dz, int storage, gbp_terrain **out);
int gbp_terrain_destroy(gbp_terrain *t);
/* bounds = {x_0, x_{N-1}, y_0, y_{M-1}} (the getXData().front()/back() values) */
int gbp_terrain_info(const gbp_terrain *t, int *nx, int *ny, int *storage,
                     double bounds[4], int *device);

/* engine options (per handle) */
#define GBP_OPT_KERNEL        1  /* GBP_KERNEL_* for the validate/extend entry points */
#define GBP_OPT_BLOCK         2  /* threads per workgroup (multiple of 64, <= 512; the
                                    direct kernel uses min(block, 256))               */
/* keys 3, 6, 7, 11, 12 (grid size, dynamic work sources, chunking, prefix,
   oversubscription) were measured slower than static per-wave slices and removed */
#define GBP_OPT_WAVES         4  /* register budget: min waves per SIMD (2..4)        */
#define GBP_OPT_LDS_COORDS    5  /* 1: stage coordinate vectors in LDS when they fit  */
#define GBP_OPT_HELPERS       8  /* 1: a drained wave's idle lanes evaluate the remaining
                                    attempts' next samples ahead (default 1)          */
#define GBP_OPT_AFFINE_COORDS 9  /* 1 (default): compute grid coordinates when the host
                                    verified x[i] == a + h*(i - b) bit for bit         */
#define GBP_OPT_COORD_MODE   10  /* read-only: 2 computed, 1 LDS-staged, 0 global      */
#define GBP_OPT_XCD_MAP      13  /* 1 = each XCD takes one contiguous eighth of the batch
                                    (workgroup b runs on XCD b % 8): for batches the
                                    caller ordered by position                         */
#define GBP_OPT_FAST_RCP     14  /* 1 (default): the bilinear 1/((x2-x1)(y2-y1)) by two
                                    Newton steps when gbp_terrain_create verified them
                                    bit-exact for every spacing pair; get: 1 = in use   */
#define GBP_OPT_FRAGILE_EPS  15  /* the FRAGILE margin in units of 1e-15 (default 1000 =
                                    1e-12, the smallest accepted): a wider margin flags
                                    and re-decides more attempts on the host, with the
                                    same results (tests use it to force host resolutions) */
/* 16, 17, 19: retired (round 4) — a Morton-sorted nearest-neighbour index, the
   packed fp32 VALU filter and a two-stream draw overlap, each measured no
   faster than the default path; setting them is an error     */
#define GBP_OPT_NN_STATS     18  /* 1: the matrix-core search counts its fp64 re-checks
                                    in gbp_plan_status.stat_nn_* (diagnostics: costs
                                    same-address atomics; default 0)                  */
#define GBP_KERNEL_DIRECT     0  /* one lane per attempt                              */
#define GBP_KERNEL_PERSISTENT 1  /* persistent waves, lanes re-packed per sample      */
int gbp_terrain_set_option(gbp_terrain *t, int key, int64_t value);
int gbp_terrain_get_option(const gbp_terrain *t, int key, int64_t *value);

/* ---- batched terrain queries ---------------------------------------------
 * FastTerrainMap::getGroundHeight + heightIsNan (fast_terrain_map.cpp:94-157)
 * xy[n][2] in; height[n], is_nan[n], ood[n] out (any output may be NULL).
 * An ood point gets height NaN and is_nan 1 (reference: undefined). */
int gbp_height_batch_dev(gbp_terrain *t, int64_t n, const double *xy, double *height,
                         uint8_t *is_nan, uint8_t *ood, gbp_stream stream);
int gbp_height_batch_host(gbp_terrain *t, int64_t n, const double *xy, double *height,
                          uint8_t *is_nan, uint8_t *ood);
/* FastTerrainMap::getSurfaceNormal (fast_terrain_map.cpp:160-213): normal[n][3] */
int gbp_normal_batch_dev(gbp_terrain *t, int64_t n, const double *xy, double *normal,
                         uint8_t *ood, gbp_stream stream);
int gbp_normal_batch_host(gbp_terrain *t, int64_t n, const double *xy, double *normal,
                          uint8_t *ood);

/* ---- state validity (planning_utils::isValidState, planning_utils.cpp:562-635)
 * states[n][8], phase[n] (or NULL => phase_all) -> valid[n], flags[n], counts[n] */
int gbp_valid_states_dev(gbp_terrain *t, int64_t n, const double *states,
                         const uint8_t *phase, int phase_all, uint8_t *valid,
                         uint32_t *flags, uint32_t *counts, gbp_stream stream);
int gbp_valid_states_host(gbp_terrain *t, int64_t n, const double *states,
                          const uint8_t *phase, int phase_all, uint8_t *valid,
                          uint32_t *flags, uint32_t *counts);

/* ---- THE HOT PATH: batched state-action pair checks ----------------------
 * planning_utils::isValidStateActionPair / isValidStateActionPairReverse
 * (+ the AdaptiveStepSize variants when adaptive != 0),
 * planning_utils.cpp:645-881.
 *   s[n][8], a[n][10]; direction[n] (GBP_FORWARD / GBP_REVERSE) or NULL =>
 *   direction_all.  Outputs (any may be NULL except flags):
 *   valid[n]      the returned bool
 *   s_new[n][8]   written ONLY where the reference assigns s_new (GBP_F_SNEW_SET),
 *                 otherwise the caller's contents are left untouched, exactly
 *                 like the reference's in/out reference parameter
 *   t_new[n]      likewise (GBP_F_TNEW_SET)
 *   flags[n]      GBP_F_* word
 *   counts[n]     G | V << 16                                               */
int gbp_validate_pairs_dev(gbp_terrain *t, int64_t n, const double *s, const double *a,
                           const uint8_t *direction, int direction_all, int adaptive,
                           uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                           uint32_t *counts, gbp_stream stream);
int gbp_validate_pairs_host(gbp_terrain *t, int64_t n, const double *s, const double *a,
                            const uint8_t *direction, int direction_all, int adaptive,
                            uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                            uint32_t *counts);

/* ---- counter-based samplers (Philox4x32-10, keyed (seed, stream, index)) ---
 * Identical draws regardless of batching / device count.  The distributions
 * are the reference's; its unseeded rand() / clock-seeded engines
 * (planning_utils.cpp:435, planner_class.cpp:51) are not reproducible, so the
 * engine defines its own reproducible streams.
 *
 * PlannerClass::randomState (planner_class.cpp:38-76), index i of stream.
 * If require_phase >= 0 the draw is repeated (k = 0..max_tries-1) until
 * isValidState(state, require_phase) holds; tries[i] = k+1 (or -1 if none). */
int gbp_sample_states_dev(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                          int64_t index_base, int require_phase, int max_tries,
                          double *states, int32_t *tries, gbp_stream stream);
int gbp_sample_states_host(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                           int64_t index_base, int require_phase, int max_tries,
                           double *states, int32_t *tries);
/* getRandomAction(surf_norm) (planning_utils.cpp:392-442) with rotate_grf
 * (:198-231): actions[n][10] from normals[n][3]; draw (stream_id, index_base+i). */
int gbp_sample_actions_dev(int64_t n, const double *normals, uint64_t seed,
                           uint64_t stream_id, int64_t index_base, double *actions,
                           gbp_stream stream);
int gbp_sample_actions_host(gbp_terrain *t, int64_t n, const double *normals, uint64_t seed,
                            uint64_t stream_id, int64_t index_base, double *actions);

/* ---- direction-biased sampling (ROS params state_direction_sampling/... and
 *      action_direction_sampling/..., config/params.yaml:21-27, forwarded by
 *      global_body_planner.cpp:193-205 to RRTClass::set_state_direction_sampling /
 *      set_action_direction_sampling, rrt.cpp:268-278).  Off by default, as in
 *      the reference.  The reference's coin is `rand()/RAND_MAX <= p`; the engine's
 *      is a Philox uniform of its own purpose (index, try) so both branches keep
 *      their counter-addressed draws. */
typedef struct {
  int32_t state_flag;            /* randomState -> randomStateDirection with probability state_p */
  int32_t state_speed_direction; /* speed_direction_flag: velocity heading = atan2(to - from) */
  double state_p;                /* probability_threshold */
  int32_t action_flag;           /* getRandomAction -> getRandomActionDirection with prob. action_p */
  int32_t reserved;
  double action_p;
} gbp_sampling;
/* The handle's sampling configuration (NULL = off): applied by every entry
 * point that draws newConfig's candidate actions (gbp_extend_batch_*,
 * gbp_extend_resolve_host, gbp_extend_tree_*) and by the device planner loop's
 * targets (gbp_plan_half_dev: s_from / s_to as rrt_connect.cpp:248-252, :283-287,
 * the trees' last vertices and roots when the half starts). */
int gbp_terrain_set_sampling(gbp_terrain *t, const gbp_sampling *cfg);
int gbp_terrain_get_sampling(const gbp_terrain *t, gbp_sampling *cfg);
/* PlannerClass::randomState(terrain, flag, p, speed_direction_flag, s_from, s_to)
 * (planner_class.cpp:22-35): index i of stream draws the coin, then either
 * randomStateDirection (:82-148: x, y uniform over the s_from / s_to rectangle,
 * heading atan2(to - from) when speed_direction) or randomState (:38-76) from
 * the same draws as gbp_sample_states_dev.  s_from[8], s_to[8] are HOST arrays;
 * cfg NULL = the handle's configuration. */
int gbp_sample_states_dir_dev(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                              int64_t index_base, const gbp_sampling *cfg, const double *s_from,
                              const double *s_to, double *states, gbp_stream stream);
int gbp_sample_states_dir_host(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                               int64_t index_base, const gbp_sampling *cfg, const double *s_from,
                               const double *s_to, double *states);
/* getRandomAction(surf_norm, direction, flag, p, s, s_near) (planning_utils.cpp:379-391):
 * the coin, then getRandomActionDirection(surf_norm, s_from, s_to) (:443-515,
 * FORWARD: s_near -> s, REVERSE: s -> s_near) or getRandomAction(surf_norm).
 * normals[n][3], s[n][8] (the state extended toward), s_near[n][8], direction[n]
 * (or NULL => direction_all); cfg NULL = the handle's configuration. */
int gbp_sample_actions_dir_dev(gbp_terrain *t, int64_t n, const double *normals, const double *s,
                               const double *s_near, const uint8_t *direction, int direction_all,
                               const gbp_sampling *cfg, uint64_t seed, uint64_t stream_id,
                               int64_t index_base, double *actions, gbp_stream stream);
int gbp_sample_actions_dir_host(gbp_terrain *t, int64_t n, const double *normals, const double *s,
                                const double *s_near, const uint8_t *direction, int direction_all,
                                const gbp_sampling *cfg, uint64_t seed, uint64_t stream_id,
                                int64_t index_base, double *actions);

/* ---- batched extend (RRTClass::newConfig + the acceptance half of
 *      RRTClass::extend, rrt.cpp:20-102) --------------------------------------
 * For extend i: s_near[i] (the nearest vertex, found by gbp_nearest_batch),
 * target[i] (the state the tree is extended towards).  Candidate action j
 * (j = 0..5) is getRandomAction(getSurfaceNormal(target)) drawn from stream
 * (seed, extend_base + i, j) — with the handle's gbp_sampling, the reference's
 * getRandomAction(surf_norm, direction, flag, p, target, s_near) (rrt.cpp:34, :49)
 * as gbp_sample_actions_dir_dev; candidates are checked (forward or reverse by
 * direction) and the LOWEST valid j is taken — the sequential newConfig.
 * result[i] = TRAPPED / ADVANCED / REACHED (isWithinBounds(s_new, target));
 * chosen[i] = j or -1; s_new[i], a_new[i] written when result != TRAPPED.   */
int gbp_extend_batch_dev(gbp_terrain *t, int64_t n, const double *s_near,
                         const double *target, const uint8_t *direction,
                         int direction_all, int adaptive, uint64_t seed,
                         int64_t extend_base, int32_t *result, int32_t *chosen,
                         double *s_new, double *a_new, uint32_t *counts,
                         uint32_t *flags, gbp_stream stream);
/* (flags[i]: OR of the executed candidates' VALID / OOD / NAN / FRAGILE / LIMIT
 *  bits; a FRAGILE extend is re-decided by gbp_extend_resolve_host.  The _host
 *  variant does that itself: its outputs are final.) */
int gbp_extend_batch_host(gbp_terrain *t, int64_t n, const double *s_near,
                          const double *target, const uint8_t *direction,
                          int direction_all, int adaptive, uint64_t seed,
                          int64_t extend_base, int32_t *result, int32_t *chosen,
                          double *s_new, double *a_new, uint32_t *counts,
                          uint32_t *flags);

/* ---- FRAGILE attempts: the host re-decision ---------------------------------
 * The kernels form isValidState's rotation without libm; where a decision's
 * margin is below 1e-12 (a height within 1e-12 of H_MIN / H_MAX, a lookup
 * point within 1e-12 of a grid line) the attempt is flagged GBP_F_FRAGILE,
 * because glibc's atan2 / cos / sin (the reference's) could decide it the
 * other way.  These entry points re-run exactly the flagged entries on the
 * host with glibc and the reference's expressions (planning_utils.cpp
 * :562-881, compiled without FMA like the reference) and overwrite their
 * outputs; flags get GBP_F_RESOLVED (FRAGILE cleared).  Host pointers; the
 * _host entry points above call them already, the _dev entry points leave it
 * to the caller.  Entries the host check does not assign keep the buffer's
 * contents.  n_resolved (may be NULL) = how many were re-decided. */
int gbp_resolve_fragile_host(gbp_terrain *t, int64_t n, const double *s, const double *a,
                             const uint8_t *direction, int direction_all, int adaptive,
                             uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                             uint32_t *counts, int64_t *n_resolved);
int gbp_resolve_fragile_states_host(gbp_terrain *t, int64_t n, const double *states,
                                    const uint8_t *phase, int phase_all, uint8_t *valid,
                                    uint32_t *flags, uint32_t *counts, int64_t *n_resolved);
/* newConfig + acceptance (rrt.cpp:20-101) re-decided for every extend whose
 * flags carry GBP_F_FRAGILE (same arguments as gbp_extend_batch_dev, host
 * pointers): the six candidate actions are regenerated on the device from
 * the same stream, then checked in order with the glibc pair check. */
int gbp_extend_resolve_host(gbp_terrain *t, int64_t n, const double *s_near, const double *target,
                            const uint8_t *direction, int direction_all, int adaptive,
                            uint64_t seed, int64_t extend_base, int32_t *result, int32_t *chosen,
                            double *s_new, double *a_new, uint32_t *counts, uint32_t *flags,
                            int64_t *n_resolved);

/* ---- nearest neighbour (PlannerClass::getNearestNeighbor,
 *      planner_class.cpp:185-200) ----------------------------------------------
 * vertices[n_vert][8] (device-resident SoA-free flat tree), queries[n_q][8];
 * index[i] = argmin_v stateDistance(query_i, v) with ties to the LOWEST index
 * (the reference ties to unordered_map iteration order). */
int gbp_nearest_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                          const double *vertices, int32_t *index, double *dist,
                          gbp_stream stream);
int gbp_nearest_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                           const double *vertices, int32_t *index, double *dist);

/* ---- radius neighbourhood (PlannerClass::neighborhoodDist,
 *      planner_class.cpp:173-182; used by RRT*-Connect, rrt_star_connect.cpp:28)
 * out[i][0..max_out): the vertices with 0 < stateDistance(query_i, v) <= radius
 * in the order the reference's vertex map holding keys 0..n_vert-1 iterates
 * them (gbp_vertex_map_order); count[i] = how many there are (entries beyond
 * max_out are not written). */
int gbp_neighbors_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                            const double *vertices, double radius, int max_out, int32_t *out,
                            int32_t *count, gbp_stream stream);
int gbp_neighbors_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                             const double *vertices, double radius, int max_out, int32_t *out,
                             int32_t *count);

/* ---- the reference vertex map's iteration order ------------------------------
 * GraphClass stores a tree's vertices in std::unordered_map<int, State>
 * (graph_class.h:155) filled with keys 0, 1, ... (graph_class.cpp:28-31) and
 * neighborhoodDist / RRT*'s choose-parent and rewire loops follow its iteration
 * order (planner_class.cpp:176-179, rrt_star_connect.cpp:31-64).  The order is
 * libstdc++'s (GCC 11.4): out[n] = the keys 0..n-1 as iterated; *rank = the
 * position of `key` (0 <= key < n).  Host functions, no device needed. */
int gbp_vertex_map_order(int64_t n, int32_t *out);
int gbp_vertex_map_rank(int64_t key, int64_t n, int64_t *rank);

/* ---- k nearest (PlannerClass::neighborhoodN, planner_class.cpp:151-171) ----
 * out[i][0..k), k = min(n_nearest, n_vert): the vertices of smallest
 * stateDistance(query_i, v) in the order the reference pops its min-heap of
 * std::pair<double, int> — ascending distance, equal distances by ascending
 * index; a NaN distance orders after every number.  dist[i][...] (may be NULL)
 * their distances; entries k .. n_nearest-1 are -1 / NaN.  1 <= n_nearest <=
 * GBP_KNN_MAX.  The reference's cost_add_yaw variant: gbp_knn_yaw_batch_dev. */
#define GBP_KNN_MAX 64
int gbp_knn_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                      const double *vertices, int n_nearest, int32_t *out, double *dist,
                      gbp_stream stream);
int gbp_knn_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                       const double *vertices, int n_nearest, int32_t *out, double *dist);

/* neighborhoodN with cost_add_yaw set (planner_class.cpp:151-171 with
 * stateDistance(q, v, true, lw, yw), planning_utils.h:146-155): the order key
 * is poseDistance(q, v) * length_weight + stateYawDistance(q, v) * yaw_weight,
 * ordered as gbp_knn_batch_dev.  The yaws atan2(s[4], s[3]) are the caller's
 * (query_yaw[n_query], vertex_yaw[n_vert], glibc's bits: no device atan2
 * reproduces them); the _host entry forms them with glibc itself. */
int gbp_knn_yaw_batch_dev(int64_t n_query, const double *queries, const double *query_yaw,
                          int64_t n_vert, const double *vertices, const double *vertex_yaw,
                          double length_weight, double yaw_weight, int n_nearest, int32_t *out,
                          double *dist, gbp_stream stream);
int gbp_knn_yaw_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                           const double *vertices, double length_weight, double yaw_weight,
                           int n_nearest, int32_t *out, double *dist);
/* atan2(s[4], s[3]) with glibc (the reference's yaw of a state, planning_utils.h:135) */
double gbp_host_yaw(const double *state);

/* ---- streams ------------------------------------------------------------ */
int gbp_stream_create(int device, gbp_stream *out);  /* a non-blocking HIP stream */
int gbp_stream_destroy(gbp_stream stream);

/* ---- device-resident trees (GraphClass / PlannerClass storage,
 *      graph_class.cpp:28-77, planner_class.cpp) ------------------------------
 * A tree lives in HBM as SoA arrays: states [cap][8], the action that reached
 * each vertex [cap][10], parent [cap] (-1 at the root), g [cap] (cost to come,
 * g[parent] + poseDistance, graph_class.cpp:36-42), and its vertex count, kept
 * on the device so that kernels append to it without a host round trip.  The
 * yaw cost y (stateYawDistance, an atan2) is left to the host, which computes
 * it along the returned path with glibc, as the reference does. */
typedef struct gbp_tree gbp_tree;
typedef struct gbp_plan_ws gbp_plan_ws;
int gbp_tree_create(int device, int64_t capacity, gbp_tree **out);
int gbp_tree_destroy(gbp_tree *tree);
/* GraphClass::init (graph_class.cpp:141-152): count = 1, vertex 0 = root */
int gbp_tree_init(gbp_tree *tree, const double *root, gbp_stream stream);
/* grows the arrays (contents kept); synchronises the stream */
int gbp_tree_reserve(gbp_tree *tree, int64_t capacity, gbp_stream stream);
int gbp_tree_capacity(gbp_tree *tree, int64_t *capacity);
int gbp_tree_size(gbp_tree *tree, int64_t *count, gbp_stream stream);  /* synchronous */
/* host copies of vertices [first, first + n); any output may be NULL (synchronous) */
int gbp_tree_read(gbp_tree *tree, int64_t first, int64_t n, double *states, double *actions,
                  int32_t *parents, double *g, gbp_stream stream);
/* appends n vertices (addVertex + addEdge + addAction) in order; g computed on
 * the device; parents may name vertices appended earlier in the same call */
int gbp_tree_append_host(gbp_tree *tree, int64_t n, const double *states, const double *actions,
                         const int32_t *parents, gbp_stream stream);
/* replaces the tree with n >= 1 given vertices: an RRT*-Connect tree, whose
 * rewiring gives vertices parents added after them (rrt_star_connect.cpp:55-62).
 * parents[0] = -1, every other parent in [0, n) and the whole a tree rooted at
 * vertex 0 (else GBP_E_INVALID_ARG, nothing changed); g is derived on the
 * device from the root down (graph_class.cpp:131-138 keeps g[c] = g[parent] +
 * poseDistance).  Synchronises the stream. */
int gbp_tree_load_host(gbp_tree *tree, int64_t n, const double *states, const double *actions,
                       const int32_t *parents, gbp_stream stream);
/* PlannerClass::getNearestNeighbor (planner_class.cpp:185-200) for n device
 * queries[n][8] against the tree (count read on the device): index[n], ties to
 * the lowest index like gbp_nearest_batch_dev.  Uses ws's status and scratch
 * (n <= its max_batch). */
int gbp_tree_nearest_dev(gbp_plan_ws *ws, gbp_tree *tree, int64_t n, const double *queries,
                         int32_t *index, gbp_stream stream);
/* the tree's device arrays (for gbp_nearest_batch_dev and the like): READ ONLY —
 * vertices are written through init / append only, which also keep the fp16
 * rows and magnitude bounds the matrix-core search relies on */
int gbp_tree_device_ptrs(gbp_tree *tree, double **states, int32_t **count);

/* ---- the device planner loop (RRTConnectClass::runRRTConnect,
 *      rrt_connect.cpp:230-314, batch-synchronous) ---------------------------
 * One half-iteration, enqueued on `stream` without any host synchronisation:
 *   stage 0  `batch` draws of T's randomState stream (planner_class.cpp:38-76),
 *            index target_index_base + i, and isValidState(STANCE) (:254)
 *   stage 1  the valid draws, compacted in order (wave ballot + prefix, look-back)
 *   stage 2  nearest vertex of T per target, newConfig's 6 candidates per target
 *            from the extend stream (gbp_extend_batch_dev's), their pair checks,
 *            the first valid one and the acceptance test (rrt.cpp:20-101)
 *   stage 3  non-TRAPPED successors appended to T in target order
 *   stage 4  each new vertex connected to its nearest vertex of O
 *            (attemptConnect, rrt_connect.cpp:20-120), direction opposite
 *   stage 5  non-TRAPPED connections appended to O in order; the first REACHED
 *            one is recorded (meet) and every later enqueued stage is a no-op
 * A FRAGILE decision halts the sequence after its stage (status.halt, every
 * later kernel a no-op): gbp_plan_resolve_host re-decides the flagged items
 * with glibc and returns the stage to resume the halted half-iteration at
 * (first_stage).  The trees must have room for `batch` more vertices each (an
 * append past a tree's capacity is not written and sets status.error bit 1). */
#define GBP_PLAN_HALT_TARGETS 1u
#define GBP_PLAN_HALT_EXTEND  2u
#define GBP_PLAN_HALT_CONNECT 4u
#define GBP_PLAN_HALT_STAR    8u  /* RRT*: an insertion's connect check (resume stage 7) */
#define GBP_PLAN_HALT_STAR_PAIRS 16u /* RRT*: a half's neighbour pairs (status.star_pairs) exceed
                                        max_pairs: gbp_plan_star_config with at least that many,
                                        then gbp_plan_resolve_host (resume stage 6) */
typedef struct {
  uint32_t halt;          /* GBP_PLAN_HALT_* of the stage that stopped the sequence */
  uint32_t done;          /* a connection REACHED */
  uint32_t error;         /* must be 0: bit 0 a bounded device spin ran out,
                             bit 1 an append found its tree full, bit 2 (RRT*)
                             the insertion's neighbour pairs or the REACHED
                             connections exceeded the workspace, bit 3 (RRT*)
                             a successor list that is not a tree */
  int32_t halt_half;      /* the half-iteration that halted */
  int32_t n_targets;      /* valid targets of the last executed half */
  int32_t n_validate;     /* candidates launched (6 n_targets, 0 when gated) */
  int32_t n_added;        /* successors appended to T */
  int32_t added_base;     /* T's count before them */
  int32_t n_conn_added;   /* connections appended to O */
  int32_t meet_half;      /* the half-iteration whose connection REACHED */
  uint64_t meet;          /* (connection index << 32) | O vertex of the first REACHED */
  int64_t ext_base;       /* extend stream base of the last half */
  int64_t ext_counter;    /* RRTClass extend counter after it */
  int64_t stat_targets, stat_attempts, stat_added, stat_conn_added;
  int64_t stat_fragile_resolved, stat_depth_capped;
  /* the gate: sequence number of the first planner kernel launch that raised
   * halt or done (~0: none).  Every launch carries its own number and is a
   * no-op only if the gate was raised by an EARLIER launch, so all workgroups
   * of the launch that raised it still finish their items. */
  uint64_t gate_seq;
  /* the matrix-core nearest-neighbour search's fp64 re-checks (k_nn_hreduce):
   * half-chunks of 16 rows re-checked, and segments scanned in full */
  int64_t stat_nn_rechecks, stat_nn_scans;
  /* the half whose targets were compacted last, and the counters before it:
   * a compaction re-run for the same half (resumed at stage 1 after a FRAGILE
   * halt) starts from them again */
  int32_t ext_half;
  uint32_t commit_fin;    /* reserved (unused since the look-ahead search) */
  int64_t ext_prev, stat_targets_prev;
  /* reserved (unused): gbp_plan_halves_dev's drawn-ahead targets are
   * counted in the workspace's look-ahead state (gbp_plan.hip gbp_plan_la) */
  int32_t pre_targets, pre_fragile;
  /* RRT*-Connect (gbp_plan_star_config): the last half's neighbour pairs
   * (new vertex, vertex before it within delta) and their connect checks
   * launched; the REACHED connections so far (shared_a / shared_b of
   * rrt_star_connect.cpp:136-175) and the cheapest of them ranked after every
   * iteration (:181-193, ties to the earliest): best_a / best_b, best_cost
   * (INFINITY: none); the connect checks of the insertions (2 per pair) and
   * the rewires */
  int32_t star_pairs, star_rows, n_shared, best_a, best_b;
  int32_t star_vrows;     /* = star_rows (round 6: the rows are the connect checks
                             themselves, k_star_check; kept for the layout) */
  double best_cost;
  int64_t stat_star_connects, stat_rewires;
} gbp_plan_status;
int gbp_plan_ws_create(gbp_terrain *t, int64_t max_batch, gbp_plan_ws **out);
int gbp_plan_ws_destroy(gbp_plan_ws *ws);
/* zeroes the status (meet = ~0) and sets the extend counter */
int gbp_plan_reset(gbp_plan_ws *ws, int64_t extend_counter, gbp_stream stream);
int gbp_plan_half_dev(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *T, gbp_tree *O, int32_t half,
                      int direction, int64_t batch, uint64_t seed, uint64_t target_stream,
                      int64_t target_index_base, int adaptive, int first_stage,
                      gbp_stream stream);
int gbp_plan_status_read(gbp_plan_ws *ws, gbp_plan_status *out, gbp_stream stream);
/* half-iterations first_half .. first_half + n_halves - 1 (half h extends tree
 * h % 2: Ta FORWARD toward target stream stream_a, Tb REVERSE toward
 * stream_b, draws from index (h / 2) * batch), the first from first_stage:
 * gbp_plan_half_dev for each.  first_stage > 0 resumes a half that halted
 * (gbp_plan_resolve_host's *resume_stage); a fresh half starts at stage 0.
 * Half numbers identify a half's draws and must increase between
 * gbp_plan_reset calls. */
int gbp_plan_halves_dev(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *Ta, gbp_tree *Tb,
                        int32_t first_half, int32_t n_halves, int64_t batch, uint64_t seed,
                        uint64_t stream_a, uint64_t stream_b, int adaptive, int first_stage,
                        gbp_stream stream);
/* RRT*-Connect (rrt_star_connect.cpp:12-67, the batched form of
 * RRTStarConnectClass::buildRRTStarConnectBatched): with enable set, every
 * half-iteration of gbp_plan_half_dev / gbp_plan_halves_dev inserts its new
 * vertices as RRT*'s extend does, between stages 3 and 4:
 *   stage 6  the neighbourhood of each new vertex among the vertices before it
 *            (stateDistance <= delta, > 0: neighborhoodDist, planner_class.cpp:
 *            173-182, in the vertex map's iteration order), and the two depth-0 connect decisions
 *            per neighbour (choose-parent attemptConnect(s_near, s_new), rewire
 *            attemptConnect(s_new, s_near)), their pair checks batched
 *   stage 7  the insertions replayed in order: choose-parent, addEdge, rewire
 *            with the g of every rewired subtree updated (graph_class.cpp:131-138)
 * and stage 5 keeps every REACHED connection (no early stop) and, after tree
 * Tb's half, ranks the cheapest with the current g values (status best_*).
 * max_pairs sizes the neighbour pairs of one half: a half with more halts
 * with GBP_PLAN_HALT_STAR_PAIRS (status.star_pairs = the count; calling this
 * again with a larger max_pairs reallocates the sets and keeps the run's
 * list of kept connections, and gbp_plan_resolve_host resumes the half at
 * stage 6).  max_shared bounds the REACHED connections of a run (status.error
 * bit 2 when exceeded).  A FRAGILE insertion check halts with
 * GBP_PLAN_HALT_STAR (resume at stage 7).  enable = 0 returns the workspace
 * to RRT-Connect. */
int gbp_plan_star_config(gbp_plan_ws *ws, int enable, double delta, int64_t max_pairs,
                         int64_t max_shared);
/* diagnostics: per half-iteration timing events (hipEvents with timing, on
 * the streams the stages run on) while enabled; gbp_plan_stage_times adds up
 * every timed half completed so far, in microseconds:
 *   us[0] the whole half (its first launch's start to stage 5's end),
 *   us[1] stages 0-3 (targets, the extends' search, their pair checks, select,
 *         append), us[2] stage 6 (RRT*: neighbourhoods, connect checks and
 *         their pair checks), us[3] stage 7 on the replay's stream (RRT*:
 *         replay, plus the best connection's ranking after Tb's halves),
 *   us[4] stages 4-5 (the connects' search, attemptConnect, append),
 *   with n >= 7 also us[5] stage 6 up to its pair checks (neighbourhoods,
 *   connect actions) and us[6] those pair checks,
 * and *halves the number of halves summed (n >= 5; reset clears).  A half's
 * events are read once the caller has synchronised its stream (status read). */
int gbp_plan_stage_timing(gbp_plan_ws *ws, int enable);
int gbp_plan_stage_times(gbp_plan_ws *ws, double *us, int n, int64_t *halves, int reset);
/* re-decides the halted stage's FRAGILE items on the host (T, O, direction,
 * batch of the halted half) and clears the halt; *resume_stage = the stage to
 * resume that half at (-1: nothing was halted) */
int gbp_plan_resolve_host(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *T, gbp_tree *O,
                          int direction, int64_t batch, int adaptive, int *resume_stage,
                          int64_t *n_resolved, gbp_stream stream);
/* RRTClass::extend (rrt.cpp:77-102) for n targets against a device tree
 * (nearest neighbour inside): targets[n][8] on the device
 * (n_dev, if not NULL, holds the count on the device, n its maximum);
 * result[i] = TRAPPED / ADVANCED / REACHED, new_vertex[i] = the appended vertex
 * or -1; candidate j of extend i is drawn from the extend stream at index
 * (extend_base + i) * 8 + j, as gbp_extend_batch_dev.  Uses ws's scratch (n <=
 * its max_batch).  T must have room for n more vertices (gbp_tree_reserve;
 * gbp_extend_tree_host reserves itself): appends past the capacity are
 * dropped and set status.error bit 1.  If a decision is FRAGILE the append halts (status.halt =
 * GBP_PLAN_HALT_EXTEND): gbp_plan_resolve_host(.., O = NULL, ..) then
 * gbp_extend_tree_finish_dev complete it.  gbp_extend_tree_host does all of
 * that synchronously from host targets. */
int gbp_extend_tree_dev(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *T, int64_t n,
                        const double *targets, const int32_t *n_dev, int direction, int adaptive,
                        uint64_t seed, int64_t extend_base, int32_t *result, int32_t *new_vertex,
                        gbp_stream stream);
int gbp_extend_tree_finish_dev(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *T, int64_t n,
                               int direction, int32_t *result, int32_t *new_vertex,
                               gbp_stream stream);
int gbp_extend_tree_host(gbp_terrain *t, gbp_plan_ws *ws, gbp_tree *T, int64_t n,
                         const double *targets, int direction, int adaptive, uint64_t seed,
                         int64_t extend_base, int32_t *result, int32_t *new_vertex,
                         int64_t *n_resolved);

#ifdef __cplusplus
}
#endif
#endif /* GBP_H */
