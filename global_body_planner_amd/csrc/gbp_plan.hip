// gbp_plan.hip — device-resident trees and the batch-synchronous RRT-Connect
// half-iteration as one stream-ordered kernel sequence (SURVEY §8(f) row 1,
// §8(b) items 4-5).
//
// One half-iteration of RRTConnectClass::runRRTConnect at batch B
// (rrt_connect.cpp:246-312, the batched form of csrc/host/gbp_planner.cpp
// RRTConnectClass::extendBatch + connectBatch), tree T extended toward B
// random targets, every new vertex connected to the other tree O:
//
//   stage 0-1 k_targets         B draws of PlannerClass::randomState
//                               (planner_class.cpp:38-76) + isValidState(STANCE),
//                               the valid ones compacted in draw order (and their
//                               fp16 rows) in the same launch; a FRAGILE draw
//                               halts the sequence here (resumed at stage 1:
//                               k_compact_targets alone)
//   stage 2  k_nn_mfma/k_nn_hreduce    getNearestNeighbor in T on the matrix cores
//                               (planner_class.cpp:185-200); extra workgroups of the
//                               same launch draw newConfig's 6 candidate actions
//                               (rrt.cpp:25-50; k_extend_prep when they are
//                               direction-biased), the reduce copies s_near
//            k_validate_persistent (gbp_engine.hip)  the candidates' pair checks
//            k_select           newConfig's first valid candidate + acceptance (rrt.cpp:52-68)
//   stage 3  k_append          non-TRAPPED successors appended to T in target order
//                               (rrt.cpp:86-92; graph_class.cpp:28-42)
//   stage 4  k_nn_mfma/k_nn_hreduce    the new vertices' nearest vertex in O
//            k_connect          RRTConnectClass::attemptConnect (rrt_connect.cpp:20-91),
//                               one wave per connection, the wave's 64 lanes
//                               evaluating the pair check's samples together
//   stage 5  k_append          non-TRAPPED connections appended to O in order;
//                               the first REACHED one ends the search
//
// RRT*-Connect (gbp_plan_star_config) inserts T's new vertices between
// stages 3 and 4 (rrt_star_connect.cpp:18-66):
//   stage 6  k_star_count       neighbourhoods in the vertex map's order, chunked
//                               (its last workgroup scans the items' offsets)
//            k_star_fill        the neighbour lists
//            k_star_check       one wave per connect check: its action and pair check
//   stage 7  k_star_replay      (own stream) the ordered choose-parent / rewire replay
// and stage 5's append also lists every REACHED connection (the ranking,
// k_star_rank, follows Tb's halves on the replay's stream).
//
// Every count (targets, candidates, appended vertices) stays on the device:
// the host enqueues many half-iterations and reads one small status record
// per group.  The appends are ordered compactions: a wave ballot + popcount
// ranks a workgroup's kept items, the workgroups chain their counts with a
// decoupled look-back (Merrill & Garland, "Single-pass parallel prefix scan
// with decoupled look-back", 2016), so vertices land in exactly the order of
// the host planner's insertion loop.
//
// FRAGILE decisions (gbp.h) stop the sequence at the next gate: the kernel
// that meets one sets status.halt; every later kernel of the group returns at
// once; the host re-decides the flagged items with glibc
// (gbp_plan_resolve_host), patches the stage's outputs, and resumes.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <type_traits>
#include <vector>

#include "gbp.h"
#include "gbp_device.h"
#include "gbp_internal.h"
#include "gbp_lane.h"
#include "gbp_um_order.h"

using namespace gbp;
static_assert(sizeof(gbp_plan_status) == 216, "engine.PlanStatus mirrors this layout");

// ============================================================================
// handles
// ============================================================================
struct gbp_tree {
  int device = 0;
  int64_t cap = 0;
  double *v = nullptr;        // [cap][8] vertex states (GraphClass vertices)
  _Float16 *vh = nullptr;     // [cap][NH_ROW] fp16 split rows (matrix-core search, nn_put_hrow)
  float *hm = nullptr;        // [16]: [0, 8) max |64 v[j][k]|, [8] (bits) 1 = a row outside fp16
  double *a = nullptr;        // [cap][10] the action that reached each vertex
  double *g = nullptr;        // [cap] cost to come: g[parent] + poseDistance
  int32_t *parent = nullptr;  // [cap], -1 at the root
  // successor lists (graph_class.cpp:28-58 successors_), first child / next
  // sibling: the RRT*-Connect rewiring updates g over a rewired vertex's
  // subtree (graph_class.cpp:131-138); kept by every append (child order is
  // immaterial: a child's g depends on its parent's alone)
  int32_t *child = nullptr, *sibling = nullptr;  // [cap], -1 = none
  int32_t *prev = nullptr;    // [cap] previous sibling (-1: first child): O(1) removeEdge
  int32_t *bfs = nullptr;     // [2 cap] scratch: the subtree update's two level queues
  int32_t *count = nullptr;   // [1] number of vertices (device resident)
};

// the segment scans k_nn_hreduce lists (a fourth unit of a segment within
// the threshold: the segment's rows in fp64) and their merge; one set for the
// caller's stream, one for the look-ahead stream
constexpr int NSC_CAP = 16384;  // listed scans per search (more: scanned in the reduce)
constexpr int NSC_UNITS = NSC_CAP * 8;  // (scan, part) results: NSC_CAP x NSC_P
struct NsBuf {
  uint32_t cap;             // list capacity (NSC_CAP; GBP_NSC_CAP lowers it: tests)
  int2 *list;               // (query, segment)
  uint32_t *cnt;            // listed
  double *ed;               // [NSC_UNITS] a scan part's minimum
  int32_t *ei;              // ... its index (lowest at that minimum)
  double *hd;               // [bmax] the reduce's own answer
  int32_t *hi;
  int2 *qh;                 // [bmax] a query's first entry and its entries
};

// the look-ahead search's device state (gbp_plan_ws::la), by half % 3 (the
// drawn-ahead target sets) and by parity (the searched trees' snapshots)
struct gbp_plan_la {
  int32_t nt[3];     // valid targets drawn for the half (ordered_rank's total)
  uint32_t frag[3];  // half + 1 when one of its draws was FRAGILE
  int32_t nv[2];     // the searched tree's vertex count when its search was launched
  uint32_t go[2];    // 0: the sequence had stopped when the search was launched (it idles)
};

struct gbp_plan_ws {
  int device = 0;
  int num_cus = 256;
  int64_t bmax = 0;            // largest batch of draws per half-iteration
  gbp_plan_status *st = nullptr;
  unsigned long long *tiles = nullptr;  // look-back tile states
  uint32_t epoch = 0;          // per-compaction tag of the tile states
  uint64_t seq = 0;            // launch sequence number of the planner kernels (gated())
  int nn_stats = 0;            // GBP_OPT_NN_STATS: k_nn_hreduce counts its re-checks in the status
  int nn_items = 4096;         // matrix-core search: work items (= waves) per launch
  int64_t ntiles = 0;
  // stage 0-1: three sets, by half % 3 (with the look-ahead search, half
  // h + 2's targets are drawn while half h + 1's are searched and half h
  // still reads its own); cand..tqh point at the set of the half being
  // enqueued or resolved (select_targets)
  struct TargetSet {
    double *cand, *targets;
    uint32_t *cflag;
    _Float16 *tqh;
  } tset[3] = {};
  double *cand = nullptr;      // [bmax][8] drawn states
  uint32_t *cflag = nullptr;   // [bmax] their isValidState flags
  double *targets = nullptr;   // [bmax][8] the valid ones, in draw order
  _Float16 *tqh = nullptr;     // [bmax][NH_ROW] their fp16 rows (k_nn_mfma's queries)
  // stage 2-3; nn, cs and ca in two sets by the half's parity (the
  // look-ahead search of half h + 1 writes its own while half h reads)
  int32_t *nn = nullptr;       // [bmax] nearest vertex of T per target
  double *cs = nullptr;        // [6 bmax][8] candidate s_near
  double *ca = nullptr;        // [6 bmax][10] candidate actions
  int32_t *nnp[2] = {};
  double *csp[2] = {}, *cap[2] = {};
  double *csn = nullptr;       // [6 bmax][8] candidate s_new
  uint32_t *cf = nullptr;      // [6 bmax] candidate flags
  uint32_t *cc = nullptr;      // [6 bmax] candidate counts
  int32_t *eres = nullptr;     // [bmax] extend result
  int32_t *echo = nullptr;     // [bmax] chosen candidate
  double *esn = nullptr;       // [bmax][8]
  double *ean = nullptr;       // [bmax][10]
  uint32_t *ef = nullptr;      // [bmax] extend flags
  int32_t *evtx = nullptr;     // [bmax] new vertex index (or -1)
  // stage 4-5
  int32_t *nno = nullptr;      // [bmax] nearest vertex of O per new vertex
  int32_t *kres = nullptr;     // [bmax] connect result
  double *ksn = nullptr;       // [bmax][8]
  double *kan = nullptr;       // [bmax][10]
  uint32_t *kf = nullptr;      // [bmax] connect flags
  // nearest-neighbour partials: NN_MAX_CHUNKS * bmax slots, pd[c * nq + qi]
  // (nn_d2 / nn_i2: the look-ahead search's, on its own stream)
  double *nn_d = nullptr, *nn_d2 = nullptr;
  int32_t *nn_i = nullptr, *nn_i2 = nullptr;
  // the direct search for a few queries (k_nn_small): per-workgroup partials
  // and the completion count of its last-workgroup reduce
  double *ns_d = nullptr;
  int32_t *ns_i = nullptr;
  uint32_t *ns_fin = nullptr;
  int ns_grid = 1;             // its workgroups (one per CU of an XCD)
  int64_t ns_capq = 0;         // queries its partials hold (ns_grid x ns_capq slots)
  NsBuf nsb[2] = {};           // k_nn_scan's lists: the caller's stream, the look-ahead's
  // the look-ahead search (gbp_plan_halves_dev): half h + 1's targets drawn
  // and searched on la_stream while half h's extends, connects and appends
  // run on the caller's stream (la_go: main -> side, la_done: side -> main)
  gbp_plan_la *la = nullptr;   // device: counts, snapshots, flags
  unsigned long long *la_tiles = nullptr;  // look-back tiles of the drawn-ahead targets
  hipStream_t la_stream = nullptr;
  hipEvent_t la_go = nullptr, la_done = nullptr;
  void *block = nullptr;       // the one allocation all of the above live in
  // RRT*-Connect (gbp_plan_star_config; star = 0: RRT-Connect): stages 6-7
  int star = 0;
  double star_delta = 3.0;     // rrt_star_connect.h:59
  int64_t star_max_pairs = 0, star_max_shared = 0;
  int64_t star_items = 0;      // scan items per half (new vertex x position chunk)
  int star_grid = 0;           // count / fill / check workgroups cap (GBP_STAR_GRID, tests; 0: none)
  int64_t star_ch = 1024;      // map positions per scan item before growth (STAR_CH)
  int32_t star_lds[3] = {-1, -1, -1};  // the replay's LDS limits (GBP_STAR_LDS, tests; -1: RP, RK, RQ)
  // a half's insertion buffers, one set per tree (half & 1): half h's replay
  // runs on star_stream beside half h's connects and half h + 1, which fills
  // the other set; half h + 2 refills this one only after the replay (its
  // stage 5 waits for it first)
  struct StarSet {
    unsigned long long *scnt = nullptr;  // [star_items] neighbours per scan item (k_star_count: tile_word)
    int32_t *sioff = nullptr;    // [star_items] the items' offsets
    int32_t *soff = nullptr;     // [bmax + 1] each new vertex's first pair
    int32_t *snb = nullptr;      // [max_pairs] the neighbour of each pair
    int32_t *sown = nullptr;     // [max_pairs] its new vertex (k)
    int32_t *srowof = nullptr;   // [2 max_pairs] connect check -> pair-check row (-1: none)
    double *srs = nullptr;       // [2 max_pairs][8] rows: the pair checks' states
    double *sra = nullptr;       // [2 max_pairs][10] and actions
    uint32_t *srf = nullptr;     // [2 max_pairs] their flags
    int64_t *meta = nullptr;     // [4] n_added, added_base, pairs (k_star_count's scan); shared count (stage-5 append)
    uint32_t *sfin = nullptr;    // [64] k_star_count's finished-workgroup count (zeroed, self-resetting)
  } ss[2];
  int32_t *kvtx = nullptr;     // [bmax] O's vertex of each connection (-1: none)
  // the replay (and the best connection's ranking) off the caller's stream:
  // e6 (stage 6 done) and e5 (stage 5 done) main -> star, rdone[k] star -> main
  // (tree k's last replay / ranking), sdone the call's join
  hipStream_t star_stream = nullptr;
  hipEvent_t star_e6 = nullptr, star_e5 = nullptr, star_rdone[2] = {nullptr, nullptr},
             star_sdone = nullptr;
  // gbp_plan_stage_timing: a ring of per-half timing events (start, after
  // stage 3, after stage 6, replay start / end, end), read back once complete
  bool timing = false;
  struct TimedHalf {
    hipEvent_t ev[8] = {};  // + [6] after stage 6's connect actions, [7] after their pair checks
    bool pending = false, star = false;
    int32_t half = 0;
  };
  TimedHalf *tring = nullptr;  // [ntring] (a plain array: no template of a gbp type exported)
  size_t ntring = 0, tnext = 0;
  double tsum[7] = {0, 0, 0, 0, 0, 0, 0};
  int64_t tcount = 0;
  int32_t *sshared = nullptr;  // [max_shared][2] the REACHED connections (a, b)
  void *star_block = nullptr;
};

namespace {

constexpr int WAVE = 64;
constexpr int TB = 256;            // threads of the grid-stride kernels
constexpr int CB = 1024;           // threads (items) per look-back tile
constexpr int NN_MAX_CHUNKS = 32;  // partial slots per query at the largest batch
constexpr uint32_t LOOKBACK_SPIN_LIMIT = 1u << 24;

// the gate every planner kernel checks first: a FRAGILE halt or a found
// connection raised by an EARLIER launch makes the rest of the enqueued
// sequence a no-op.  Each launch carries its sequence number `seq`
// (gbp_plan_ws::seq); the launch that raises the gate records its own
// (gate_seq, atomicMin), so a workgroup dispatched after another workgroup of
// the same launch raised it still computes its items — the host's
// resolution and resume rely on every item of the halted stage being final.
__device__ __forceinline__ bool gated(const gbp_plan_status *st, uint64_t seq) {
  return __hip_atomic_load(&st->gate_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < seq;
}
__device__ __forceinline__ void raise_gate(gbp_plan_status *st, uint64_t seq) {
  atomicMin((unsigned long long *)&st->gate_seq, (unsigned long long)seq);
}

__device__ __forceinline__ void copy8(double *d, const double *s) {
#pragma unroll
  for (int k = 0; k < 8; k++) d[k] = s[k];
}
__device__ __forceinline__ void copy10(double *d, const double *s) {
#pragma unroll
  for (int k = 0; k < 10; k++) d[k] = s[k];
}

// ---- ordered compaction across the grid ---------------------------------------
// Block b of a CB-thread grid keeps the items whose `keep` is set; returns the
// item's rank among all kept items of the grid (blocks in order, threads in
// order within a block).  Tile states are 64-bit words (epoch | flag | count),
// published and polled with agent-scope atomic RMW operations (executed at
// memory, coherent across the XCDs' L2s).  Every block of the grid must call
// this exactly once.  The grid must be resident at once (callers launch at
// most a few hundred 1024-thread blocks).  *total gets the grid's total
// (written by the last block).
__device__ __forceinline__ unsigned long long tile_word(uint32_t epoch, uint32_t flag, uint32_t v) {
  return ((unsigned long long)epoch << 32) | ((unsigned long long)flag << 30) | (v & 0x3FFFFFFFu);
}

__device__ uint32_t ordered_rank(bool keep, unsigned long long *tiles, uint32_t epoch,
                                 int32_t *total, gbp_plan_status *st, uint32_t tile, uint32_t ntile) {
  __shared__ uint32_t wsum[CB / WAVE];
  __shared__ uint32_t s_excl;
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const unsigned long long m = __ballot(keep);
  const uint32_t wr = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
  if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
  __syncthreads();
  uint32_t woff = 0, bsum = 0;
  for (int i = 0; i < (int)(blockDim.x / WAVE); i++) {
    if (i < w) woff += wsum[i];
    bsum += wsum[i];
  }
  if (threadIdx.x == 0) {
    const uint32_t b = tile;
    uint32_t excl = 0;
    if (b > 0) {
      __hip_atomic_exchange(&tiles[b], tile_word(epoch, 1, bsum), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
      int j = (int)b - 1;
      uint32_t spins = 0;
      for (;;) {
        const unsigned long long x =
            __hip_atomic_fetch_add(&tiles[j], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t flag = (uint32_t)(x >> 30) & 3u;
        if ((uint32_t)(x >> 32) != epoch || flag == 0) {
          if (++spins > LOOKBACK_SPIN_LIMIT) {  // bounded: report, never hang
            atomicOr(&st->error, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        excl += (uint32_t)(x & 0x3FFFFFFFu);
        if (flag == 2 || j == 0) break;
        --j;
      }
    }
    __hip_atomic_exchange(&tiles[b], tile_word(epoch, 2, excl + bsum), __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
    s_excl = excl;
    if (b == ntile - 1) *total = (int32_t)(excl + bsum);
  }
  __syncthreads();
  return s_excl + woff + wr;
}
__device__ __forceinline__ uint32_t ordered_rank(bool keep, unsigned long long *tiles, uint32_t epoch,
                                                 int32_t *total, gbp_plan_status *st) {
  return ordered_rank(keep, tiles, epoch, total, st, blockIdx.x, gridDim.x);
}

// stateDistance(q, vertex j) exactly as the reference evaluates it
// (planning_utils.cpp:116-127): the exact stage of every search below
__device__ __forceinline__ double nn_dist64(const double qq[8], const double *vj) {
  double sum = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double d = vj[k] - qq[k];
    sum = sum + 1.0 * d * d;
  }
  return sqrt(sum);
}

// lexicographic (distance, index) minimum: the lowest index among equal
// distances; a NaN distance never wins
__device__ __forceinline__ void ns_min(double &d, int &i, double od, int oi) {
  if (od < d || (od == d && oi < i)) {
    d = od;
    i = oi;
  }
}

// ============================================================================
// nearest neighbour in a device tree on the matrix cores (planner_class.cpp:185-200)
// ============================================================================
// The filter's scores S_j = |F_j|^2 - 2 G.F_j (F_j = 64 v_j, G = 64 q: scaled
// by a power of two, so exactly; |G - F_j|^2 = |G|^2 + S_j) for a tile of 32
// vertex rows x 32 queries are two v_mfma_f32_32x32x16_f16 with fp32
// accumulation, from each coordinate split into two fp16 parts (hi + lo):
//   MFMA 1  K = [F_hi(8) | F_lo(8)] . [-2 G_hi | -2 G_hi]
//   MFMA 2  K = [F_hi(8) | N_1 N_2 N_3 0..] . [-2 G_lo | 2^14 2^14 2^14 0..]
// with N_1 + N_2 + N_3 the row's fp64 squared norm times 2^-14 in three fp16
// parts (nn_put_hrow).  The dropped G_lo.F_lo term and the parts' rounding are
// ~2^-20 of the products, so the matrix cores score 1024 (query, vertex) pairs
// per 64 MFMA cycles (the packed fp32 VALU filter of round 2 spent ~4.5
// instructions per pair and pass).  The VALU only reduces: per lane (its
// query and its 32 rows of two consecutive chunks: a "lane-unit") the minimum
// by v_min3, then the three smallest unit minima with their units and a bound
// m4 on every other unit (NhTop: v_med3 / v_cndmask, branch-free).  Work item
// = (4 query tiles = 128 queries, a segment of whole units), one wave each;
// the two lanes of a query merge their lists and the (m1..m4, units) entry goes
// to the partial slots; k_nn_hreduce then takes B = min m1 over the segments
// and re-checks in fp64 every listed unit whose minimum is <= T(B), and every
// row of a segment whose m4 is <= T(B) (a fourth unit within the threshold:
// ~4 per planner half-iteration).
// Why no minimiser is lost (everything in the scaled units; M_k = the tree's
// hmax[k] >= max_j |F_jk|; S~_j the computed score):
//   * each fp16 split has |x - hi - lo| <= 2^-20 |x| + 2^-14 (lo may be
//     subnormal or flushed), the dropped G_lo F_lo term is <= 2^-20 |G_k||F_k|,
//     the norm's three parts are within 2^-29 |F|^2 + 1, and 32 fp32
//     accumulations (rounding or truncating) add at most
//     gamma (sum |terms|), gamma = 33 * 2^-23; so |S~_j - S_j| <= eps(G)
//     (nh_eps: gamma (1.01 MM + 2.02 GM) + 2^-29 MM + 1 + 2 sum_k
//     [(4 * 2^-20 |G_k| + 1.01 * 2^-14) M_k + 1.01 * 2^-14 |G_k| + 2^-27], MM = sum M_k^2,
//     GM = sum |G_k| M_k);
//   * the fp64 minimiser j* (the reference's sqrt of an fp64 sum) has
//     |G - F_j*|^2 <= |G - F_i|^2 (1 + 5e-15) for every row i, so with i the
//     row scoring B: S~_j* <= B + 2 eps + 5e-15 (B + eps + |G|^2) <= T(B)
//     (nh_threshold: fp64, 1e-14, rounded up to fp32) — and so does every row
//     tying with j*.  Its unit has minimum <= T: it is listed (checked), or
//     three other units of that segment are listed and then m4 <= T (the
//     segment is scanned).
// Rows with |F_k| >= 2^13 (|v_k| >= 128) or NaN mark the tree (hbad): its
// searches scan in fp64.  So do queries with |G_k| >= 2^13 or NaN.
constexpr int NH_ROW = 32;             // fp16 per row: F_hi[8] F_lo[8] F_hi[8] N_1 N_2 N_3 0[5]
constexpr double NH_SCALE = 64.0;      // F = 64 v (exact)
constexpr double NH_LIM = 8192.0;      // |F_k| < 2^13: |F|^2 * 2^-14 < 2^15 fits fp16
constexpr double NH_NSCALE = 0x1p-14;  // the norm parts are |F|^2 * 2^-14 ...
constexpr float NH_NCONST = 16384.0f;  // ... times 2^14 on the query side
constexpr int NS_MAXQ = 32;            // k_nn_small: queries it takes (the connects')
constexpr int NS_GQ = 4;               // ... scored together per pass
constexpr int NS_TB = 256;
constexpr int NS_BLOCKS = 1024;        // its largest grid
constexpr int NH_NT = 4;               // query tiles (32 queries) per wave
constexpr int NH_ITEMS = 4096;         // waves a search aims for
constexpr int NH_MAX_SEG = 64;         // segments per query (the reduce reads them all)
constexpr int NH_TB = 256;             // 4 independent waves per workgroup
constexpr int NH_RTB = 256;            // reduce: workgroup size
constexpr int NH_G = 16;               // reduce: lanes per query

typedef _Float16 nh8 __attribute__((ext_vector_type(8)));
typedef float nhacc __attribute__((ext_vector_type(16)));

// fp16 hi + lo of a scaled coordinate (|x| < 2^13)
__device__ __forceinline__ void nh_split(double x, _Float16 &hi, _Float16 &lo) {
  hi = (_Float16)(float)x;
  lo = (_Float16)(float)(x - (double)hi);
}

// row j of the fp16 rows; hm = {hmax[8], hbad}
__device__ __forceinline__ void nn_put_hrow(_Float16 *__restrict__ vh, float *__restrict__ hm,
                                            int64_t j, const double *s, bool init) {
  nh8 fh, fl, nr;
  double n = 0.0;
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double x = s[k] * NH_SCALE;
    const bool ok = fabs(x) < NH_LIM;
    bad = bad || !ok;
    _Float16 hi, lo;
    nh_split(ok ? x : 0.0, hi, lo);
    fh[k] = hi;
    fl[k] = lo;
    n = n + x * x;
    const float ax = ok ? (float)fabs(x) : 0.f;
    if (!hm) continue;  // a query row
    if (init)
      hm[k] = ax;
    else
      atomicMax((unsigned int *)(hm + k), __float_as_uint(ax));
  }
  const double ns = bad ? 0.0 : n * NH_NSCALE;
  const _Float16 n1 = (_Float16)(float)ns;
  const double r1 = ns - (double)n1;
  const _Float16 n2 = (_Float16)(float)r1;
  const _Float16 n3 = (_Float16)(float)(r1 - (double)n2);
  nr = nh8{n1, n2, n3, 0, 0, 0, 0, 0};
  nh8 *r = (nh8 *)(vh + (int64_t)NH_ROW * j);
  r[0] = fh;
  r[1] = fl;
  r[2] = fh;
  r[3] = nr;
  if (!hm) return;
  if (init)
    ((uint32_t *)hm)[8] = bad ? 1u : 0u;
  else if (bad)
    atomicOr((uint32_t *)hm + 8, 1u);
}

// items: query groups (NH_NT tiles) x segments of cps chunks (32 rows); at
// most NN_MAX_CHUNKS * bmax partial slots (pm[seg * nq + qi])
__device__ __forceinline__ void nh_geometry(int64_t nq, int64_t nv, int64_t bmax, int items,
                                            int64_t &nqg, int64_t &nseg, int64_t &cps, int64_t &nch) {
  nch = nv > 0 ? (nv + 31) / 32 : 1;
  nqg = nq > 0 ? (nq + 32 * NH_NT - 1) / (32 * NH_NT) : 1;
  int64_t want = (items + nqg - 1) / nqg;
  const int64_t slots = (NN_MAX_CHUNKS * bmax) / (nq > 0 ? nq : 1);
  if (want > slots) want = slots;
  if (want > NH_MAX_SEG) want = NH_MAX_SEG;
  if (want > nch) want = nch;
  if (want < 1) want = 1;
  cps = (nch + want - 1) / want;
  cps += cps & 1;  // whole units (pairs of chunks)
  nseg = (nch + cps - 1) / cps;
}

// eps(G) above; q: the query (G = 64 q), hm: the tree's hmax
__device__ __forceinline__ double nh_eps(const double (&q)[8], const float *__restrict__ hm) {
  double mm = 0.0, gm = 0.0, lin = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double m = (double)hm[k] * (1.0 + 0x1p-22), ag = fabs(q[k] * NH_SCALE);
    mm += m * m;
    gm += ag * m;
    lin += (4.0 * 0x1p-20 * ag + 1.01 * 0x1p-14) * m + 1.01 * 0x1p-14 * ag + 0x1p-27;
  }
  const double gamma = 33.0 * 0x1p-23;
  return gamma * (1.01 * mm + 2.02 * gm) + 0x1p-29 * mm + 1.0 + 2.0 * lin;
}

__device__ __forceinline__ float nh_threshold(float B, double eps, double g2) {
  const double t = (double)B + 2.0 * eps + 1e-14 * (fabs((double)B) + eps + g2);
  return isnan(t) ? INFINITY : nextafterf((float)t, INFINITY);
}

// min of two (v_med3 against -inf: no canonicalising v_max as fminf brings)
__device__ __forceinline__ float nh_min2(float a, float b) {
  return __builtin_amdgcn_fmed3f(a, b, -INFINITY);
}
// min over the 16 scores of a lane: 7 v_min3 + 1 v_med3
__device__ __forceinline__ float nh_min16(const nhacc &a) {
  const float x0 = fminf(fminf(a[0], a[1]), a[2]), x1 = fminf(fminf(a[3], a[4]), a[5]);
  const float x2 = fminf(fminf(a[6], a[7]), a[8]), x3 = fminf(fminf(a[9], a[10]), a[11]);
  const float x4 = fminf(fminf(a[12], a[13]), a[14]);
  return nh_min2(fminf(fminf(x0, x1), x2), fminf(fminf(x3, x4), a[15]));
}

// a lane's three smallest unit minima (m1 <= m2 <= m3, units i1, i2, i3) and
// a lower bound m4 on every other unit's minimum; branch-free (3 v_cmp,
// 3 v_med3, 6 v_cndmask).  Planner trees are clustered: with two units a
// third within the threshold (a segment scan) came ~25 times per half-iteration.
struct NhTop {
  float m1 = INFINITY, m2 = INFINITY, m3 = INFINITY, m4 = INFINITY;
  int i1 = -1, i2 = -1, i3 = -1;
  __device__ __forceinline__ void insert(float cm, int c) {
    const bool lt1 = cm < m1, lt2 = cm < m2, lt3 = cm < m3;
    const float n4 = __builtin_amdgcn_fmed3f(m3, cm, m4), n3 = __builtin_amdgcn_fmed3f(m2, cm, m3);
    const float n2 = __builtin_amdgcn_fmed3f(m1, cm, m2), n1 = lt1 ? cm : m1;
    const int j1 = lt1 ? c : i1, j2a = lt1 ? i1 : c, j2 = lt2 ? j2a : i2;
    const int j3a = lt2 ? i2 : c, j3 = lt3 ? j3a : i3;
    m1 = n1;
    m2 = n2;
    m3 = n3;
    m4 = n4;
    i1 = j1;
    i2 = j2;
    i3 = j3;
  }
};

// pass of one wave over chunks [c0, c1) (c0 even; wave-uniform, as is nv):
// NT query tiles (B operands b1, b2).  Lane (r, h) reads row c*32 + r: part
// h (F_hi / F_lo) for MFMA 1 and part 2 + h (F_hi / norm) for MFMA 2, two
// 16-B loads with one address; the row arrays hold whole units (tree_alloc),
// rows past nv are masked.  A lane's unit u is its 32 rows of chunks 2u and
// 2u + 1 (rows 64u + 32b + 4h + (i & 3) + 8 (i >> 2), b < 2, i < 16): the
// top-2 bookkeeping runs once per unit
template <int NT>
__device__ __forceinline__ void nh_sweep(const _Float16 *__restrict__ vh, int c0, int c1, int nv,
                                         const nh8 (&b1)[NT], const nh8 (&b2)[NT], NhTop (&t)[NT]) {
  const int lane = threadIdx.x & (WAVE - 1), r = lane & 31, h = lane >> 5;
  const nh8 *base = (const nh8 *)vh + (NH_ROW / 8) * r + h;
  constexpr int64_t CS = NH_ROW * 4;  // nh8 per chunk
  // tile u's minimum over its lane-unit: the scores of chunks c and c + 1
  // (TAIL: rows past nv masked, chunk c + 1 absent when c + 1 >= c1)
  auto unit_min = [&](int u, int c, const nh8 (&a)[4], auto tail_tag) {
    constexpr bool TAIL = decltype(tail_tag)::value;
    float m = INFINITY;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      if (TAIL && c + k >= c1) break;
      nhacc acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * k], b1[u], nhacc{}, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * k + 1], b2[u], acc, 0, 0, 0);
      if (TAIL) {
        const int rem = nv - 32 * (c + k);
#pragma unroll
        for (int i = 0; i < 16; i++)
          if ((i & 3) + 8 * (i >> 2) + 4 * h >= rem) acc[i] = INFINITY;
      }
      m = k ? nh_min2(m, nh_min16(acc)) : nh_min16(acc);
    }
    return m;
  };
  auto load = [&](int c, nh8 (&d)[4]) {
    d[0] = base[CS * c];
    d[1] = base[CS * c + 2];
    d[2] = base[CS * (c + 1)];
    d[3] = base[CS * (c + 1) + 2];
  };
  // full units, the next unit's rows in flight while one is scored; a
  // scheduling barrier per tile keeps one tile's accumulators live at a time
  const int uf = min(c1, nv >> 5) & ~1;  // chunks [c0, uf) form full units
#ifndef GBP_NN_SERIAL
  // Full units, software-pipelined over two accumulators: a chunk's scores
  // (two MFMAs) are reduced while the next chunk's MFMAs run, so the wave's
  // VALU minimum and top-3 insert overlap its own matrix work instead of
  // waiting for it (the serial form, -DGBP_NN_SERIAL, scores a tile's two
  // chunks and then reduces them).  Job order: (tile 0, chunk c), (tile 0,
  // c + 1), (tile 1, c), ... then the next unit's (tile 0, c + 2) from the
  // rows loaded a unit ahead.
  if (c0 < uf) {
    auto score = [&](const nh8 (&a)[4], int k, int u) {
      nhacc acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * k], b1[u], nhacc{}, 0, 0, 0);
      return __builtin_amdgcn_mfma_f32_32x32x16_f16(a[2 * k + 1], b2[u], acc, 0, 0, 0);
    };
    // one unit's tiles; NEXT: the last tile's slots score the next unit's
    // first jobs (a branch-free body, so that the scheduling barriers hold
    // the order)
    auto unit = [&](const nh8 (&a)[4], const nh8 (&p)[4], int c, nhacc &X, nhacc &Y, auto next_tag) {
      constexpr bool NEXT = decltype(next_tag)::value;
#pragma unroll
      for (int u = 0; u < NT; u++) {
        float m = nh_min16(X);
        __builtin_amdgcn_sched_barrier(0);
        if (u + 1 < NT)
          X = score(a, 0, u + 1);
        else if (NEXT)
          X = score(p, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        m = nh_min2(m, nh_min16(Y));
        t[u].insert(m, c >> 1);
        __builtin_amdgcn_sched_barrier(0);
        if (u + 1 < NT)
          Y = score(a, 1, u + 1);
        else if (NEXT)
          Y = score(p, 1, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    nh8 a[4], p[4];
    load(c0, a);
    nhacc X = score(a, 0, 0), Y = score(a, 1, 0);
    int c = c0;
    for (; c + 2 < uf; c += 2) {
      load(c + 2, p);
      unit(a, p, c, X, Y, std::true_type{});
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = p[k];
    }
    unit(a, a, c, X, Y, std::false_type{});
  }
#else
  if (c0 < uf) {
    nh8 a[4], p[4];
    load(c0, a);
    for (int c = c0; c < uf; c += 2) {
      if (c + 2 < uf) load(c + 2, p);
#pragma unroll
      for (int u = 0; u < NT; u++) {
        t[u].insert(unit_min(u, c, a, std::false_type{}), c >> 1);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = p[k];
    }
  }
#endif
  if (uf < c1) {  // the last unit: a lone chunk and/or rows past the tree's end
    nh8 a[4];
    load(uf, a);  // the row arrays hold whole units
#pragma unroll
    for (int u = 0; u < NT; u++) t[u].insert(unit_min(u, uf, a, std::true_type{}), uf >> 1);
  }
}

// newConfig's candidate actions for the extends (rrt.cpp:25 surface normal,
// :34 the six draws of the extend stream) do not depend on the nearest vertex
// unless the draws are direction-biased, so stage 2 computes them in extra
// workgroups of the search's launch (PREP): they run beside the MFMA waves
// (VALU and transcendental work next to matrix-core work) instead of as a
// launch of their own after the search (k_extend_prep); the reduce then
// copies s_near into the candidates (k_nn_hreduce cs).
// The next half's targets, drawn ahead in the same launch (draw_blocks > 0;
// gbp_plan_halves_dev, sampling not direction-biased: an inline search draws
// the next half's, the look-ahead search of half h + 1 those of half h + 2):
// blocks [0, draw_blocks) draw them into that half's target set and rank them
// (ordered_rank over those blocks on the look-ahead tiles: their count in
// gbp_plan_la::nt; a FRAGILE draw sets gbp_plan_la::frag = half + 1, and the
// half halts at its start in k_la_commit).  They come first in the grid so
// that their latency-bound work overlaps the matrix-core waves.
struct NhDraw {
  int draw_blocks;
  int32_t half;  // the half the draws are for
  int64_t n, base;
  uint64_t stream;
  double *cand, *targets;
  uint32_t *cflag;
  _Float16 *tqh;
  unsigned long long *tiles;
  uint32_t epoch;
  int32_t *count;   // the valid draws' total (gbp_plan_la::nt of the half)
  uint32_t *frag;   // set to half + 1 on a FRAGILE draw (gbp_plan_la::frag)
  // an inline search launching the look-ahead one: the next search's tree
  // snapshot and whether the sequence still runs (gbp_plan_la::nv / go)
  const int32_t *snap_src;
  int32_t *snap_dst;
  uint32_t *go_dst;
};
template <class ZT>
struct NhPrep {
  TerrainView<ZT> T;
  uint64_t seed;
  double *ca;
  gbp_sampling cfg;
  int direction;
  int first_block;  // blocks [first_block, gridDim.x) draw the actions
  NhDraw dr;        // blocks [0, dr.draw_blocks): the next half's targets
  // the look-ahead search (nt set): the half's count is *nt (its drawn-ahead
  // total), its extend base the counter after the current half's commit
  // (commit_targets), and n_validate is left to k_la_commit
  const int32_t *nt;
};

// three waves per SIMD (168 VGPRs): the pipelined sweep's two live
// accumulators would otherwise take it to 189 and two waves; the few values
// it spills around the sweep cost less (planner 5-s runs 181.4 vs 177.8 M
// extends/s, the serial sweep 179.5; profiles/r06i_nn_pipe_ab.txt)
#ifndef GBP_NN_WPE
#define GBP_NN_WPE __attribute__((amdgpu_waves_per_eu(3)))
#endif
template <int NT, class ZT, bool PREP>
__global__ __launch_bounds__(NH_TB) GBP_NN_WPE void k_nn_mfma(gbp_plan_status *__restrict__ st,
                                                   const int32_t *__restrict__ nq_dev,
                                                   const double *__restrict__ q,
                                                   const int32_t *__restrict__ q_off_dev,
                                                   const _Float16 *__restrict__ qh,
                                                   const _Float16 *__restrict__ vh,
                                                   const float *__restrict__ hm,
                                                   const int32_t *__restrict__ nv_dev, int64_t bmax,
                                                   float4 *__restrict__ pm, int4 *__restrict__ pid,
                                                   uint64_t seq, int n_items, NhPrep<ZT> pp,
                                                   const uint32_t *__restrict__ go, int small_max,
                                                   uint32_t *scan_cnt) {
  // the reduce's scan list starts empty (whatever this launch then does:
  // k_nn_scan / k_nn_scan_merge run after every search)
  if (blockIdx.x == 0 && threadIdx.x == 0) *scan_cnt = 0;
  if (PREP && pp.dr.snap_dst && blockIdx.x == 0 && threadIdx.x == 0) {
    *pp.dr.snap_dst = *pp.dr.snap_src;
    *pp.dr.go_dst = gated(st, seq) ? 0u : 1u;
  }
  if (gated(st, seq)) {
    if (PREP && !pp.nt && blockIdx.x == pp.first_block && threadIdx.x == 0) st->n_validate = 0;
    return;
  }
  if (go && *go == 0u) return;  // a look-ahead search launched after the sequence stopped
  if (!PREP && *nq_dev <= small_max) return;  // k_nn_small has them
  // the next half's targets (k_targets' work); float heights only: with fp64
  // heights the state check's registers would cost the search an occupancy step
  if constexpr (PREP && std::is_same_v<ZT, float>) if ((int)blockIdx.x < pp.dr.draw_blocks) {
    const NhDraw &d = pp.dr;
    const int64_t i = blockIdx.x * (int64_t)NH_TB + threadIdx.x;
    // s_from / s_to are unused: draws ahead are never direction-biased (the
    // host refuses draw_blocks > 0 with state_flag set); zeroed all the same
    double q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t f = 0;
    if (i < d.n) {
      sample_state_cfg_try(pp.T, pp.cfg, q, q, pp.seed, d.stream, d.base + i, 0, q);  // not biased
      Acc acc{0, 0, 0};
      const bool v = is_valid_state(pp.T, q, GBP_STANCE, acc);  // rrt_connect.cpp:254
      f = acc.flags | (v ? GBP_F_VALID : 0u);
      copy8(d.cand + 8 * i, q);
      d.cflag[i] = f;
    }
    const bool keep = f & GBP_F_VALID;
    if (__ballot(f & GBP_F_FRAGILE) && (threadIdx.x & (WAVE - 1)) == 0) *d.frag = (uint32_t)d.half + 1;
    const uint32_t r = ordered_rank(keep, d.tiles, d.epoch, d.count, st, blockIdx.x,
                                    (uint32_t)d.draw_blocks);
    if (keep) {
      copy8(d.targets + 8 * (size_t)r, q);
      nn_put_hrow(d.tqh, nullptr, r, q, false);
    }
    return;
  }
  if (PREP && (int)blockIdx.x >= pp.first_block) {  // the extends' candidate actions
    const int64_t n = pp.nt ? *pp.nt : st->n_targets, m = n * GBP_NUM_GEN_STATES;
    const int64_t base = pp.nt ? st->ext_counter : st->ext_base;
    if (!pp.nt && blockIdx.x == pp.first_block && threadIdx.x == 0) st->n_validate = (int32_t)m;
    for (int64_t c = (blockIdx.x - pp.first_block) * (int64_t)NH_TB + threadIdx.x; c < m;
         c += (int64_t)(gridDim.x - pp.first_block) * NH_TB) {
      const int64_t i = c / GBP_NUM_GEN_STATES;
      const int j = (int)(c - i * GBP_NUM_GEN_STATES);
      double nrm[3], a[10];
      surface_normal(pp.T, q[8 * i], q[8 * i + 1], nrm);  // rrt.cpp:25
      sample_action_cfg(nrm, pp.cfg, pp.direction, q + 8 * i, q + 8 * i /* unused: not biased */,
                        pp.seed, GBP_EXTEND_STREAM, (base + i) * 8 + j, a);  // rrt.cpp:34, :49
      copy10(pp.ca + 10 * c, a);
    }
    return;
  }
  const int64_t nq = *nq_dev, nv = *nv_dev, q_off = q_off_dev ? *q_off_dev : 0;
  int64_t nqg, nseg, cps, nch;
  nh_geometry(nq, nv, bmax, n_items, nqg, nseg, cps, nch);
  const bool tree_bad = ((const uint32_t *)hm)[8] != 0u || nv <= 0;
  const int lane = threadIdx.x & (WAVE - 1), r = lane & 31, h = lane >> 5;
  const int mb = PREP ? pp.dr.draw_blocks : 0;  // the search's first workgroup
  const int waves = ((PREP ? pp.first_block : (int)gridDim.x) - mb) * (NH_TB / WAVE);
  const int items = (int)(nqg * nseg);
  for (int item = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - mb) * (NH_TB / WAVE) + threadIdx.x / WAVE);
       item < items; item += waves) {
    // segment-major: a workgroup's waves score the same vertex rows against
    // consecutive query groups (their loads meet in the CU's L1): 215 vs 223 us
    // at 40k vertices, 43,690 queries (profiles/r05j_nn_ab*.txt)
    const int sg = item / (int)nqg, qg = item - sg * (int)nqg;
    const int c0 = sg * (int)cps, c1 = min((int)nch, c0 + (int)cps);
    nh8 b1[NT], b2[NT];
    NhTop t[NT];
    const nh8 ncst = {(_Float16)NH_NCONST, (_Float16)NH_NCONST, (_Float16)NH_NCONST, 0, 0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < NT; u++) {
      const int64_t qi = qg * (32 * NT) + 32 * u + r;
      const bool live = qi < nq;
      if (qh) {  // the queries' fp16 rows (nn_put_hrow layout: F_hi, F_lo)
        const nh8 *qr = (const nh8 *)(qh + (int64_t)NH_ROW * (q_off + (live ? qi : 0)));
        const nh8 zh = {}, hi = live ? qr[0] : zh, lo = live ? qr[1] : zh;
        b1[u] = hi * (_Float16)(-2.0f);
        b2[u] = h ? ncst : lo * (_Float16)(-2.0f);
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) {
          const double x = live ? q[8 * (q_off + qi) + k] * NH_SCALE : 0.0;
          _Float16 hi, lo;
          nh_split(fabs(x) < NH_LIM ? x : 0.0, hi, lo);  // a bad query is scanned in fp64
          b1[u][k] = (_Float16)(-2.0f) * hi;
          b2[u][k] = h ? ncst[k] : (_Float16)(-2.0f) * lo;
        }
      }
    }
    if (!tree_bad) nh_sweep<NT>(vh, c0, c1, (int)nv, b1, b2, t);
    // the two lanes of a query (rows 4h + ...): merge to one entry, the three
    // smallest lane-units (id = 2 unit + h) and a lower bound on the rest:
    // the other lane's three inserted into this lane's list
    if (tree_bad) {
#pragma unroll
      for (int u = 0; u < NT; u++) {
        const int64_t qi = (int64_t)qg * (32 * NT) + 32 * u + r;
        if (h == 0 && qi < nq) {
          pm[(int64_t)sg * nq + qi] = float4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
          pid[(int64_t)sg * nq + qi] = int4{-1, -1, -1, -1};
        }
      }
      continue;
    }
#pragma unroll
    for (int u = 0; u < NT; u++) {
      NhTop e = t[u];
      e.i1 = e.i1 >= 0 ? 2 * e.i1 + h : -1;
      e.i2 = e.i2 >= 0 ? 2 * e.i2 + h : -1;
      e.i3 = e.i3 >= 0 ? 2 * e.i3 + h : -1;
      const float o1 = __shfl_xor(e.m1, 32), o2 = __shfl_xor(e.m2, 32), o3 = __shfl_xor(e.m3, 32);
      const float o4 = __shfl_xor(e.m4, 32);
      const int p1 = __shfl_xor(e.i1, 32), p2 = __shfl_xor(e.i2, 32), p3 = __shfl_xor(e.i3, 32);
      e.insert(o1, p1);
      e.insert(o2, p2);
      e.insert(o3, p3);
      e.m4 = fminf(e.m4, o4);
      const int64_t qi = (int64_t)qg * (32 * NT) + 32 * u + r;
      if (h == 0 && qi < nq) {
        pm[(int64_t)sg * nq + qi] = float4{e.m1, e.m2, e.m3, e.m4};
        pid[(int64_t)sg * nq + qi] = int4{e.i1, e.i2, e.i3, 0};
      }
    }
  }
}

constexpr int NSC_TB = 256;  // k_nn_scan's workgroup
constexpr int NSC_P = 8;     // ... workgroups per listed scan
constexpr int NSM_TB = 256;   // k_nn_scan_merge

// 16 lanes per query: B, T(B), the fp64 re-checks, lexicographic (distance,
// index) minimum; nothing < inf (a NaN query): index 0.  (Writing the six
// extend candidates from here instead of k_extend_prep was measured slower:
// the sampler's registers halved the reduce's occupancy, 16 + 15.9 -> 63 us.)
__global__ __launch_bounds__(NH_RTB) void k_nn_hreduce(gbp_plan_status *st,
                                                       const int32_t *__restrict__ nq_dev,
                                                       const double *__restrict__ q,
                                                       const int32_t *__restrict__ q_off_dev,
                                                       const double *__restrict__ v,
                                                       const float *__restrict__ hm,
                                                       const int32_t *__restrict__ nv_dev,
                                                       int64_t bmax, const float4 *__restrict__ pm,
                                                       const int4 *__restrict__ pid,
                                                       int32_t *__restrict__ out, uint64_t seq,
                                                       int stats, double *__restrict__ cs, int n_items,
                                                       const uint32_t *__restrict__ go, int small_max,
                                                       NsBuf sb) {
  if (gated(st, seq)) return;
  if (go && *go == 0u) return;  // (k_nn_mfma)
  if (*nq_dev <= small_max) return;  // (k_nn_mfma)
  const int64_t nq = *nq_dev, nv = *nv_dev, q_off = q_off_dev ? *q_off_dev : 0;
  int64_t nqg, nseg, cps, nch;
  nh_geometry(nq, nv, bmax, n_items, nqg, nseg, cps, nch);
  const bool tree_bad = ((const uint32_t *)hm)[8] != 0u || nv <= 0;
  const int sl = threadIdx.x & (NH_G - 1);
  const int64_t groups = (int64_t)gridDim.x * (NH_RTB / NH_G);
  const int64_t iters = (nq + groups - 1) / groups;  // whole groups iterate together
  for (int64_t it = 0; it < iters; it++) {
    const int64_t qi = it * groups + blockIdx.x * (int64_t)(NH_RTB / NH_G) + threadIdx.x / NH_G;
    const bool live = qi < nq;
    double qq[8], g2 = 0.0;
    bool qbad = false;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      qq[k] = live ? q[8 * (q_off + qi) + k] : 0.0;
      const double gk = qq[k] * NH_SCALE;
      qbad = qbad || !(fabs(gk) < NH_LIM);
      g2 += gk * gk;
    }
    // the group's entries, lane sl reading segments sl, sl + NH_G, ...
    constexpr int NK = NH_MAX_SEG / NH_G;
    float B = INFINITY, w4[NK];
#pragma unroll
    for (int k = 0; k < NK; k++) {
      const int64_t s = sl + NH_G * k;
      const float4 e = live && s < nseg ? pm[s * nq + qi] : float4{INFINITY, INFINITY, INFINITY, INFINITY};
      B = fminf(B, e.x);
      w4[k] = e.w;
    }
#pragma unroll
    for (int off = NH_G / 2; off > 0; off >>= 1) B = fminf(B, __shfl_xor(B, off, NH_G));
    const float T = nh_threshold(B, nh_eps(qq, hm), g2);
    double best = INFINITY;
    int bi = 0x7FFFFFFF, nrc = 0, nsc = 0;
    bool full = live && (qbad || tree_bad || !(B < INFINITY));
    const int gbit = (threadIdx.x & (WAVE - 1)) & ~(NH_G - 1);
    constexpr uint32_t GM = NH_G == 32 ? 0xFFFFFFFFu : (1u << NH_G) - 1u;
    // segments with a fourth unit within T are scanned in full by k_nn_scan:
    // the query's entries listed contiguously (its group's leader reserves
    // them); a full list turns the query into a whole-tree fp64 scan here
    int qn = 0, qbase = 0;  // (group-uniform)
    {
      uint32_t bal[NK], tot = 0;
#pragma unroll
      for (int k = 0; k < NK; k++) {
        bal[k] = (uint32_t)(__ballot(live && !full && sl + NH_G * k < nseg && w4[k] <= T) >> gbit) & GM;
        tot += __popc(bal[k]);
      }
      nsc += sl == 0 ? (int)tot : 0;
      if (tot) {
        uint32_t base = 0;
        if (sl == 0) base = atomicAdd(sb.cnt, tot);
        base = (uint32_t)__shfl((int)base, gbit);
        const bool fits = base + tot <= sb.cap;
        uint32_t off = base;
#pragma unroll
        for (int k = 0; k < NK; k++) {
          if ((bal[k] >> sl) & 1u) {
            const uint32_t slot = off + __popc(bal[k] & ((1u << sl) - 1u));
            if (slot < sb.cap)  // (past a full list: reserved, unused)
              sb.list[slot] = fits ? int2{(int)qi, (int)(sl + NH_G * k)} : int2{-1, 0};
          }
          off += __popc(bal[k]);
        }
        if (fits) {
          qn = (int)tot;
          qbase = (int)base;
        } else {
          full = live;
        }
      }
    }
    if (full) {  // the whole tree in fp64
      for (int64_t j = sl; j < nv; j += NH_G) {
        const double d = nn_dist64(qq, v + 8 * j);
        if (d < best) {  // ascending per lane: the first index at its minimum
          best = d;
          bi = (int)j;
        }
      }
    }
    // the half-chunks to re-check go round the group: a half-chunk's 16 rows
    // one per lane
    const bool part = live && !full;
    for (int64_t s0 = 0; s0 < nseg; s0 += NH_G) {
      const int64_t s = s0 + sl;
      bool chk1 = false, chk2 = false, chk3 = false;
      int4 hid = {-1, -1, -1, 0};
      if (part && s < nseg) {
        const float4 e = pm[s * nq + qi];  // L2-warm since the first pass
        if (!(e.w <= T) && e.x <= T) {  // (a segment in full: listed above)
          hid = pid[s * nq + qi];
          chk1 = hid.x >= 0;
          chk2 = e.y <= T && hid.y >= 0;
          chk3 = e.z <= T && hid.z >= 0;
        }
      }
      uint32_t cmask = (uint32_t)(__ballot(chk1) >> gbit) & GM;
      uint32_t cmask2 = (uint32_t)(__ballot(chk2) >> gbit) & GM;
      uint32_t cmask3 = (uint32_t)(__ballot(chk3) >> gbit) & GM;
      nrc += sl == 0 ? __popc(cmask) + __popc(cmask2) + __popc(cmask3) : 0;
      while (__ballot((cmask | cmask2 | cmask3) != 0u)) {
        if (cmask | cmask2 | cmask3) {
          int h;
          if (cmask) {
            const int src = __ffs(cmask) - 1;
            cmask &= cmask - 1u;
            h = __shfl(hid.x, src, NH_G);
          } else if (cmask2) {
            const int src = __ffs(cmask2) - 1;
            cmask2 &= cmask2 - 1u;
            h = __shfl(hid.y, src, NH_G);
          } else {
            const int src = __ffs(cmask3) - 1;
            cmask3 &= cmask3 - 1u;
            h = __shfl(hid.z, src, NH_G);
          }
          // the lane-unit's 32 rows, 32 / NH_G per lane
#pragma unroll
          for (int r = 0; r < 32 / NH_G; r++) {
            const int x = sl + NH_G * r, b = x >> 4, i = x & 15;
            const int64_t j =
                (int64_t)(h >> 1) * 64 + 32 * b + 4 * (h & 1) + (i & 3) + 8 * (i >> 2);
            if (j < nv) {
              const double d = nn_dist64(qq, v + 8 * j);
              if (d < best || (d == best && j < bi)) {
                best = d;
                bi = (int)j;
              }
            }
          }
        }
      }
    }
#pragma unroll
    for (int off = NH_G / 2; off > 0; off >>= 1) {
      const double od = __shfl_xor(best, off, NH_G);
      const int oi = __shfl_xor(bi, off, NH_G);
      if (od < best || (od == best && oi < bi)) {
        best = od;
        bi = oi;
      }
    }
    if (live && sl == 0) out[qi] = bi == 0x7FFFFFFF ? 0 : bi;
    if (cs && live && sl < GBP_NUM_GEN_STATES)  // s_near of the six candidates (k_extend_prep)
      copy8(cs + 8 * (qi * GBP_NUM_GEN_STATES + sl), v + 8 * (int64_t)(bi == 0x7FFFFFFF ? 0 : bi));
    // a query with listed scans: its answer so far, for k_nn_scan_merge
    if (qn && sl == 0) {
      sb.hd[qi] = best;
      sb.hi[qi] = bi;
      sb.qh[qi] = int2{qbase, qn};
    }
    if (!stats) continue;  // diagnostics (GBP_OPT_NN_STATS): same-address atomics serialise
    for (int off = 32; off > 0; off >>= 1) {
      nrc += __shfl_xor(nrc, off);
      nsc += __shfl_xor(nsc, off);
    }
    if ((threadIdx.x & (WAVE - 1)) == 0 && (nrc | nsc)) {
      atomicAdd((unsigned long long *)&st->stat_nn_rechecks, (unsigned long long)nrc);
      atomicAdd((unsigned long long *)&st->stat_nn_scans, (unsigned long long)nsc);
    }
  }
}

// the listed segment scans (a ~3k-row segment walked by one wave was the
// reduce's tail: 80 -> 31 us at 40k vertices without it), each over NSC_P
// workgroups: unit u = (scan u / NSC_P, part u % NSC_P) writes its rows'
// lexicographic (distance, index) minimum.  k_nn_scan_merge then folds, per
// query, its scans' units into the reduce's answer and rewrites out / the
// candidates' s_near where it changed.  Never gated: k_nn_mfma empties the
// list first thing, whatever the sequence does.
__global__ __launch_bounds__(NSC_TB) void k_nn_scan(const int32_t *__restrict__ nq_dev,
                                                    const double *__restrict__ q,
                                                    const int32_t *__restrict__ q_off_dev,
                                                    const double *__restrict__ v,
                                                    const int32_t *__restrict__ nv_dev, int64_t bmax,
                                                    int n_items, NsBuf sb) {
  const uint32_t n = min(*sb.cnt, sb.cap);
  if (n == 0) return;
  const int64_t nq = *nq_dev, nv = *nv_dev, q_off = q_off_dev ? *q_off_dev : 0;
  int64_t nqg, nseg, cps, nch;
  nh_geometry(nq, nv, bmax, n_items, nqg, nseg, cps, nch);
  __shared__ double sd[NSC_TB / WAVE];
  __shared__ int si[NSC_TB / WAVE];
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const uint32_t units = n * NSC_P;
  for (uint32_t e = blockIdx.x; e < units; e += gridDim.x) {
    const int2 L = sb.list[e / NSC_P];
    if (L.x < 0) continue;  // (workgroup-uniform)
    double qq[8];
#pragma unroll
    for (int k = 0; k < 8; k++) qq[k] = q[8 * (q_off + L.x) + k];
    const int64_t j0 = L.y * cps * 32, j1 = min(nv, min(nch, (L.y + 1) * cps) * 32);
    const int64_t len = (j1 - j0 + NSC_P - 1) / NSC_P, p0 = j0 + (e % NSC_P) * len;
    const int64_t p1 = min(j1, p0 + len);
    double d = INFINITY;
    int i = 0x7FFFFFFF;
    for (int64_t j = p0 + threadIdx.x; j < p1; j += NSC_TB) ns_min(d, i, nn_dist64(qq, v + 8 * j), (int)j);
    for (int off = WAVE / 2; off > 0; off >>= 1) ns_min(d, i, __shfl_xor(d, off), __shfl_xor(i, off));
    if (lane == 0) {
      sd[w] = d;
      si[w] = i;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 1; k < NSC_TB / WAVE; k++) ns_min(d, i, sd[k], si[k]);
      sb.ed[e] = d;
      sb.ei[e] = i;
    }
    __syncthreads();
  }
}

// per listed query (its first entry): its units folded into the reduce's
// answer (hd / hi); out and the candidates' s_near rewritten where it changed
// (the list is emptied by the next search's k_nn_mfma)
__global__ __launch_bounds__(NSM_TB) void k_nn_scan_merge(NsBuf sb, const double *__restrict__ v,
                                                          int32_t *__restrict__ out,
                                                          double *__restrict__ cs) {
  const uint32_t n = min(*sb.cnt, sb.cap);
  for (uint32_t e = blockIdx.x * NSM_TB + threadIdx.x; e < n; e += gridDim.x * NSM_TB) {
    const int qx = sb.list[e].x;
    if (qx < 0) continue;
    const int2 h = sb.qh[qx];
    if (h.x != (int)e) continue;  // not the query's first entry
    double d = sb.hd[qx];
    int i = sb.hi[qx];
    const int i0 = i;
    for (int f = h.x; f < h.x + h.y; f++)
#pragma unroll
      for (int k = 0; k < NSC_P; k++) ns_min(d, i, sb.ed[f * NSC_P + k], sb.ei[f * NSC_P + k]);
    if (i == i0) continue;
    const int o = i == 0x7FFFFFFF ? 0 : i;
    out[qx] = o;
    if (cs)
      for (int k = 0; k < GBP_NUM_GEN_STATES; k++)
        copy8(cs + 8 * ((int64_t)qx * GBP_NUM_GEN_STATES + k), v + 8 * (int64_t)o);
  }
}

// A few queries (the connect stage's: the vertices one half added, ~1-10 at
// the planner's batch) against a tree of tens of thousands of vertices: the
// matrix-core search would give each query a few long-running waves and its
// reduce a latency chain (~25 + 18 us per half at 40k vertices); here every
// thread scores its vertices in fp64 for up to NS_GQ queries at a time
// (nn_dist64: the exact stage itself, nothing to re-check), workgroups reduce
// (distance, index) lexicographically (the lowest index among ties,
// planner_class.cpp:185-200; NaN never wins, so a NaN query gets index 0 as
// in k_nn_hreduce) and the last workgroup to finish reduces the partials.
// k_nn_mfma / k_nn_hreduce return at once when nq <= NS_MAXQ (small_max).
__global__ __launch_bounds__(NS_TB) void k_nn_small(gbp_plan_status *st, const int32_t *__restrict__ nq_dev,
                                                     const double *__restrict__ q,
                                                     const int32_t *__restrict__ q_off_dev,
                                                     const double *__restrict__ v,
                                                     const int32_t *__restrict__ nv_dev,
                                                     int32_t *__restrict__ out, double *__restrict__ pd,
                                                     int32_t *__restrict__ pi, uint32_t *fin, int64_t capq,
                                                     uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t nq = *nq_dev, nv = *nv_dev, q_off = q_off_dev ? *q_off_dev : 0;
  if (nq <= 0 || nq > capq) return;
  __shared__ double sd[NS_TB / WAVE][NS_GQ];
  __shared__ int si[NS_TB / WAVE][NS_GQ];
  __shared__ bool last;
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  for (int64_t k0 = 0; k0 < nq; k0 += NS_GQ) {
    double qq[NS_GQ][8], bd[NS_GQ];
    int bi[NS_GQ];
#pragma unroll
    for (int g = 0; g < NS_GQ; g++) {
      const int64_t k = min(k0 + g, nq - 1);
#pragma unroll
      for (int c = 0; c < 8; c++) qq[g][c] = q[8 * (q_off + k) + c];
      bd[g] = INFINITY;
      bi[g] = 0x7FFFFFFF;
    }
    for (int64_t j = blockIdx.x * (int64_t)NS_TB + threadIdx.x; j < nv; j += (int64_t)gridDim.x * NS_TB) {
#pragma unroll
      for (int g = 0; g < NS_GQ; g++) ns_min(bd[g], bi[g], nn_dist64(qq[g], v + 8 * j), (int)j);
    }
#pragma unroll
    for (int g = 0; g < NS_GQ; g++) {
      for (int off = WAVE / 2; off > 0; off >>= 1)
        ns_min(bd[g], bi[g], __shfl_xor(bd[g], off), __shfl_xor(bi[g], off));
      if (lane == 0) {
        sd[w][g] = bd[g];
        si[w][g] = bi[g];
      }
    }
    __syncthreads();
    if (threadIdx.x < NS_GQ && k0 + threadIdx.x < nq) {
      double d = sd[0][threadIdx.x];
      int i = si[0][threadIdx.x];
      for (int ww = 1; ww < NS_TB / WAVE; ww++) ns_min(d, i, sd[ww][threadIdx.x], si[ww][threadIdx.x]);
      pd[(k0 + threadIdx.x) * gridDim.x + blockIdx.x] = d;
      pi[(k0 + threadIdx.x) * gridDim.x + blockIdx.x] = i;
      __threadfence();  // (before this workgroup counts itself finished)
    }
    __syncthreads();
  }
  // the last workgroup to finish reduces every query's partials
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(fin, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  for (int64_t k = w; k < nq; k += NS_TB / WAVE) {
    double d = INFINITY;
    int i = 0x7FFFFFFF;
    for (int b = lane; b < (int)gridDim.x; b += WAVE)
      ns_min(d, i, __hip_atomic_load(&pd[k * gridDim.x + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_load(&pi[k * gridDim.x + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    for (int off = WAVE / 2; off > 0; off >>= 1) ns_min(d, i, __shfl_xor(d, off), __shfl_xor(i, off));
    if (lane == 0) out[k] = i == 0x7FFFFFFF ? 0 : i;
  }
  if (threadIdx.x == 0) *fin = 0;  // reset for the next launch (stream-ordered)
}

// ============================================================================
// stages 0-1: targets and their ordered compaction
// ============================================================================
// the extend stream of a half: RRTClass::extend_counter_ advances by the
// number of extends (csrc/host/gbp_planner.cpp extendBatch); the re-run of a
// compaction that halted on a FRAGILE draw (the host resumes the half at
// stage 1, gbp_plan_resolve_host) starts from the same counters.  Called by
// the compaction's last workgroup once the grid's total is known.
__device__ __forceinline__ void commit_targets(gbp_plan_status *st, int32_t half, bool resumed) {
  const int64_t base = resumed ? st->ext_prev : st->ext_counter;
  const int64_t tg = resumed ? st->stat_targets_prev : st->stat_targets;
  st->ext_half = half;
  st->ext_prev = base;
  st->stat_targets_prev = tg;
  st->ext_base = base;
  st->ext_counter = base + st->n_targets;
  st->stat_targets = tg + st->n_targets;
}

// stages 0-1 of a fresh half in one launch: thread i draws target i of T's
// randomState stream (planner_class.cpp:38-76) and checks isValidState(STANCE)
// (rrt_connect.cpp:254), then the workgroups rank the valid draws in draw order
// (ordered_rank: ballot + popcount, decoupled look-back) and write them with
// their fp16 query rows.  A FRAGILE draw halts the sequence here; the host
// re-decides it with glibc and resumes the half at stage 1, the compaction
// alone (k_compact_targets on the patched flags).
template <class ZT>
__global__ __launch_bounds__(TB) void k_targets(TerrainView<ZT> T, gbp_plan_status *st, int64_t n,
                                                uint64_t seed, uint64_t stream_id, int64_t base,
                                                double *__restrict__ cand,
                                                uint32_t *__restrict__ cflag,
                                                double *__restrict__ targets,
                                                _Float16 *__restrict__ tqh,
                                                unsigned long long *tiles, uint32_t epoch,
                                                int32_t half, uint64_t seq, gbp_sampling cfg,
                                                const double *__restrict__ tv,
                                                const int32_t *__restrict__ tcount,
                                                const double *__restrict__ ov, int direction) {
  if (gated(st, seq)) return;
  // direction-biased draws (rrt_connect.cpp:248-252, :283-287): s_from / s_to
  // are T's last vertex and O's root (FORWARD half, T = Ta), or O's root and
  // T's last vertex (REVERSE half, T = Tb), as the trees stand when the half
  // starts (the batch-synchronous snapshot; batch 1 is the reference's loop)
  const double *t_last = tv + 8 * (int64_t)(*tcount - 1);
  const double *s_from = direction == GBP_FORWARD ? t_last : ov;
  const double *s_to = direction == GBP_FORWARD ? ov : t_last;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  double q[8];
  uint32_t f = 0;
  if (i < n) {
    sample_state_cfg_try(T, cfg, s_from, s_to, seed, stream_id, base + i, 0, q);  // randomState
    Acc acc{0, 0, 0};
    const bool v = is_valid_state(T, q, GBP_STANCE, acc);   // rrt_connect.cpp:254
    f = acc.flags | (v ? GBP_F_VALID : 0u);
    copy8(cand + 8 * i, q);
    cflag[i] = f;
  }
  const bool keep = f & GBP_F_VALID;
  if (__ballot(f & GBP_F_FRAGILE) && (threadIdx.x & (WAVE - 1)) == 0) {  // the targets stage halts
    atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_TARGETS);
    st->halt_half = half;
    raise_gate(st, seq);
  }
  const uint32_t r = ordered_rank(keep, tiles, epoch, &st->n_targets, st);
  if (keep) {
    copy8(targets + 8 * (size_t)r, q);
    nn_put_hrow(tqh, nullptr, r, q, false);  // the search's query rows
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) commit_targets(st, half, false);
}

// stage 1 alone (a half resumed after a FRAGILE draw, on the host-patched
// flags): the compacted targets in draw order and their fp16 query rows
__global__ __launch_bounds__(CB) void k_compact_targets(gbp_plan_status *st, int64_t n,
                                                        const double *__restrict__ cand,
                                                        const uint32_t *__restrict__ cflag,
                                                        double *__restrict__ targets,
                                                        _Float16 *__restrict__ tqh,
                                                        unsigned long long *tiles, uint32_t epoch,
                                                        int32_t half, int resumed, uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t i = blockIdx.x * (int64_t)CB + threadIdx.x;
  const uint32_t f = i < n ? cflag[i] : 0u;
  const bool keep = f & GBP_F_VALID;
  if (__ballot(f & GBP_F_FRAGILE) && (threadIdx.x & (WAVE - 1)) == 0) {  // the targets stage halts
    atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_TARGETS);
    st->halt_half = half;
    raise_gate(st, seq);
  }
  const uint32_t r = ordered_rank(keep, tiles, epoch, &st->n_targets, st);
  if (keep) {
    copy8(targets + 8 * (size_t)r, cand + 8 * i);
    nn_put_hrow(tqh, nullptr, r, cand + 8 * i, false);  // the search's query rows
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) commit_targets(st, half, resumed != 0);
}

// stages 0-1 of a half whose targets were drawn ahead and searched by the
// look-ahead search (gbp_plan_halves_dev), the half's first launch on the
// caller's stream: the count and the counters, the FRAGILE halt at the half's
// start (what k_targets' last workgroup and its FRAGILE wave would have done),
// n_validate; then the search's answer completed: it saw T's first
// la->nv[half & 1] vertices (the count when it was launched), so every
// target compares its nearest with the vertices appended since (the previous
// half's connections) in fp64 — a later vertex wins only when strictly closer,
// as its index is higher (planner_class.cpp:185-200) — and rewrites its
// candidates' s_near.  Block 0 also records the next look-ahead search's
// snapshot of O (the tree the next half extends: unchanged until this half's
// connects) and whether it should run.
__global__ __launch_bounds__(TB) void k_la_commit(gbp_plan_status *st, gbp_plan_la *la, int32_t half,
                                                  const double *__restrict__ targets,
                                                  const double *__restrict__ tv,
                                                  const int32_t *__restrict__ tcount,
                                                  int32_t *__restrict__ nn, double *__restrict__ cs,
                                                  const int32_t *__restrict__ ocount, uint64_t seq) {
  const int slot = half % 3, p = half & 1;
  const bool g = gated(st, seq);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    la->nv[p ^ 1] = *ocount;
    bool go = !g;
    if (g) {
      st->n_validate = 0;  // the validate launch idles
    } else {
      const int32_t n = la->nt[slot];
      st->n_targets = n;
      commit_targets(st, half, false);
      const bool frag = la->frag[slot] == (uint32_t)half + 1;
      la->frag[slot] = 0;
      if (frag) {  // the targets stage halts
        atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_TARGETS);
        st->halt_half = half;
        raise_gate(st, seq);
        go = false;
      }
      st->n_validate = frag ? 0 : n * GBP_NUM_GEN_STATES;
    }
    la->go[p ^ 1] = go ? 1u : 0u;
  }
  if (g) return;
  const int64_t n = la->nt[slot], v0 = la->nv[p], v1 = *tcount;
  if (v1 <= v0) return;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double q[8];
    copy8(q, targets + 8 * i);
    const int32_t j0 = nn[i];
    int32_t bi = j0;
    double best = nn_dist64(q, tv + 8 * (int64_t)j0);
    for (int64_t j = v0; j < v1; j++) {
      const double d = nn_dist64(q, tv + 8 * j);
      if (d < best) {
        best = d;
        bi = (int32_t)j;
      }
    }
    if (bi != j0) {
      nn[i] = bi;
      for (int k = 0; k < GBP_NUM_GEN_STATES; k++)
        copy8(cs + 8 * (i * GBP_NUM_GEN_STATES + k), tv + 8 * (int64_t)bi);
    }
  }
}

// ============================================================================
// stage 2: newConfig (rrt.cpp:20-70)
// ============================================================================
template <class ZT>
__global__ __launch_bounds__(TB) void k_extend_prep(TerrainView<ZT> T, gbp_plan_status *st,
                                                    const double *__restrict__ targets,
                                                    const int32_t *__restrict__ nn,
                                                    const double *__restrict__ tv, uint64_t seed,
                                                    double *__restrict__ cs,
                                                    double *__restrict__ ca, uint64_t seq,
                                                    gbp_sampling cfg, int direction) {
  if (gated(st, seq)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) st->n_validate = 0;  // the validate launch idles
    return;
  }
  const int64_t n = st->n_targets, m = n * GBP_NUM_GEN_STATES, base = st->ext_base;
  if (blockIdx.x == 0 && threadIdx.x == 0) st->n_validate = (int32_t)m;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < m;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / GBP_NUM_GEN_STATES;
    const int j = (int)(c - i * GBP_NUM_GEN_STATES);
    double nv[3];
    surface_normal(T, targets[8 * i], targets[8 * i + 1], nv);  // rrt.cpp:25
    double a[10];
    sample_action_cfg(nv, cfg, direction, targets + 8 * i, tv + 8 * (int64_t)nn[i], seed,
                      GBP_EXTEND_STREAM, (base + i) * 8 + j, a);  // rrt.cpp:34, :49
    copy10(ca + 10 * c, a);
    copy8(cs + 8 * c, tv + 8 * (int64_t)nn[i]);
  }
}

// the first valid candidate (rrt.cpp:36-50) and the closer-than-s_near
// acceptance (rrt.cpp:52-68, :84-101)
__global__ __launch_bounds__(TB) void k_select(gbp_plan_status *st, const double *__restrict__ targets,
                                               const int32_t *__restrict__ nn,
                                               const double *__restrict__ tv,
                                               const double *__restrict__ ca,
                                               const double *__restrict__ csn,
                                               const uint32_t *__restrict__ cf,
                                               int32_t *__restrict__ eres,
                                               int32_t *__restrict__ echo,
                                               double *__restrict__ esn, double *__restrict__ ean,
                                               uint32_t *__restrict__ ef, int32_t half,
                                               uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t n = st->n_targets;
  bool frag = false;
  unsigned long long executed = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double sn[8], tg[8], sv[8];
    copy8(sn, tv + 8 * (int64_t)nn[i]);
    copy8(tg, targets + 8 * i);
    int found = -1;
    uint32_t fl = 0;
    for (int j = 0; j < GBP_NUM_GEN_STATES; j++) {
      const uint32_t f = cf[i * GBP_NUM_GEN_STATES + j];
      fl |= f & (GBP_F_VALID | GBP_F_OOD | GBP_F_NAN | GBP_F_FRAGILE | GBP_F_LIMIT);
      if (f & GBP_F_VALID) {
        found = j;
        break;
      }
    }
    executed += found >= 0 ? found + 1 : GBP_NUM_GEN_STATES;
    const double d0 = state_distance(sn, tg);
    double best = d0;
    int r = GBP_TRAPPED;
    if (found >= 0) {
      const int64_t c = i * GBP_NUM_GEN_STATES + found;
      copy8(sv, csn + 8 * c);
      const double cur = state_distance(sv, tg);
      if (cur < best) {
        best = cur;
        copy8(esn + 8 * i, sv);
        copy10(ean + 10 * i, ca + 10 * c);
        r = (cur <= GOAL_BOUNDS) ? GBP_REACHED : GBP_ADVANCED;  // isWithinBounds(s_new, s)
      }
    }
    eres[i] = r;
    echo[i] = found;
    ef[i] = fl;
    frag = frag || (fl & GBP_F_FRAGILE);
  }
  // one atomic per workgroup for the statistics (same-address atomics
  // serialise: one per wave cost ~2 us a launch), one per wave for the gate
  const int lane = threadIdx.x & (WAVE - 1);
  for (int off = WAVE / 2; off > 0; off >>= 1) executed += __shfl_down(executed, off);
  __shared__ unsigned long long s_exec[TB / WAVE];
  if (lane == 0) s_exec[threadIdx.x / WAVE] = executed;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long e = 0;
    for (int k = 0; k < TB / WAVE; k++) e += s_exec[k];
    if (e) atomicAdd((unsigned long long *)&st->stat_attempts, e);
  }
  if (__ballot(frag) && lane == 0) {
    atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_EXTEND);
    st->halt_half = half;
    raise_gate(st, seq);
  }
}

// ============================================================================
// stages 3 and 5: ordered appends (rrt.cpp:86-92, rrt_connect.cpp:107-116)
// ============================================================================
// RRT*'s list of the connections kept (rrt_star_connect.cpp:136-175:
// shared_a / shared_b), built by the stage-5 append itself when `list` is
// set (round 6; a one-workgroup launch after it before): the REACHED
// connections that were appended, in connection order, after the n_shared
// listed before — a second ordered look-back over tiles of their own
// (tiles2, epoch2; the grid's total in *tot2), the last tile publishing
// n_shared and meta[3] (the list's length for the ranking after Tb's half)
struct StarShared {
  int32_t *list = nullptr;
  int64_t max_shared = 0;
  int64_t *meta = nullptr;
  unsigned long long *tiles2 = nullptr;
  uint32_t epoch2 = 0;
  int32_t *tot2 = nullptr;
  int t_is_a = 0;
};

// mode 0: extend successors of the current targets into T (parent = nn[i]);
// mode 1: connections of the new vertices into O (parent = nno[k]), the first
// REACHED one in order recorded as the meeting point.
__global__ __launch_bounds__(CB) void k_append(gbp_plan_status *st, int mode,
                                               const int32_t *__restrict__ res,
                                               const int32_t *__restrict__ par,
                                               const double *__restrict__ sn,
                                               const double *__restrict__ an, double *__restrict__ tv,
                                               _Float16 *__restrict__ tvh, float *__restrict__ thm,
                                               double *__restrict__ ta, double *__restrict__ tg,
                                               int32_t *__restrict__ tp, int32_t *__restrict__ tcount,
                                               int32_t *__restrict__ vtx, unsigned long long *tiles,
                                               uint32_t epoch, int32_t half, int64_t cap,
                                               uint64_t seq, int32_t *tch,
                                               int32_t *tsib, int32_t *tprev, int star,
                                               StarShared sh = StarShared{}) {
  if (gated(st, seq)) return;
  __shared__ int32_t s_base;
  if (threadIdx.x == 0) s_base = *tcount;  // read before this block publishes its count
  __syncthreads();
  const int32_t base = s_base;
  const int64_t n = mode == 0 ? st->n_targets : st->n_added;
  const int64_t i = blockIdx.x * (int64_t)CB + threadIdx.x;
  const bool live = i < n;
  const int32_t r = live ? res[i] : GBP_TRAPPED;
  const bool keep = live && r != GBP_TRAPPED;
  int32_t *total = mode == 0 ? &st->n_added : &st->n_conn_added;
  const uint32_t rank = ordered_rank(keep, tiles, epoch, total, st);
  if (keep && (int64_t)base + rank >= cap) {
    // the caller reserved too little: drop, report, and gate every later
    // launch (a search over rows past cap would read out of bounds)
    atomicOr(&st->error, 2u);
    raise_gate(st, seq);
    if (vtx) vtx[i] = -1;
  } else if (keep) {
    const int32_t idx = base + (int32_t)rank, p = par[i];
    double s[8], pv[8];
    copy8(s, sn + 8 * i);
    copy8(pv, tv + 8 * (int64_t)p);
    copy8(tv + 8 * (int64_t)idx, s);
    nn_put_hrow(tvh, thm, idx, s, false);
    copy10(ta + 10 * (int64_t)idx, an + 10 * i);
    tp[idx] = p;
    tg[idx] = tg[p] + pose_distance(pv, s);  // graph_class.cpp:36-42 addEdge
    tch[idx] = -1;
    // the successor list: RRT*'s extends are joined by the insertion replay
    // (k_star_replay: choose-parent), everything else here.  A vertex is its
    // parent's first child once linked: its previous-sibling slot is cleared
    // before the exchange publishes it, and the next vertex linked to the same
    // parent (the only one the exchange returns it to) sets it afterwards.
    tprev[idx] = -1;
    if (mode == 0 && star) {
      tsib[idx] = -1;
    } else {
      __threadfence();
      const int32_t h = atomicExch(&tch[p], idx);
      tsib[idx] = h;
      if (h >= 0) tprev[h] = idx;
    }
    if (vtx) vtx[i] = idx;
    if (mode == 1 && r == GBP_REACHED && !star) {  // RRT*: every REACHED one is kept (StarShared)
      atomicMin((unsigned long long *)&st->meet,
                ((unsigned long long)i << 32) | (unsigned long long)(uint32_t)idx);
      st->meet_half = half;
      atomicOr(&st->done, 1u);
      raise_gate(st, seq);
    }
  } else if (live && vtx) {
    vtx[i] = -1;
  }
  if (sh.list) {  // (mode 1, RRT*: every block reaches here; ns read before any publishes)
    const int64_t ns = st->n_shared;
    const bool hit = keep && r == GBP_REACHED && (int64_t)base + rank < cap;
    const uint32_t r2 = ordered_rank(hit, sh.tiles2, sh.epoch2, sh.tot2, st);
    if (hit && ns + (int64_t)r2 < sh.max_shared) {
      // connection i joins T's new vertex added_base + i to O's appended row
      const int32_t tv_ = (int32_t)(st->added_base + i), ov = (int32_t)(base + rank);
      sh.list[2 * (ns + r2)] = sh.t_is_a ? tv_ : ov;
      sh.list[2 * (ns + r2) + 1] = sh.t_is_a ? ov : tv_;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
      const int64_t tot = ns + *sh.tot2;
      if (tot > sh.max_shared) {
        atomicOr(&st->error, 4u);
        raise_gate(st, seq);
      } else {
        st->n_shared = (int32_t)tot;
        sh.meta[3] = tot;
      }
    }
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    // the rows actually written (the appended count is clamped at cap)
    const int32_t added = (int32_t)min<int64_t>(*total, cap - (int64_t)base);
    *total = added;
    *tcount = base + added;
    if (mode == 0) {
      st->added_base = base;
      st->stat_added += added;
    } else {
      st->stat_conn_added += added;
    }
  }
}

// ============================================================================
// stage 4: RRTConnectClass::attemptConnect (rrt_connect.cpp:20-91)
// ============================================================================
// rrt_connect.cpp:53-63
__device__ __forceinline__ void connect_action(const double *s_start, const double *s_goal,
                                               double t_s, double *a) {
  const double x_td = s_start[0], y_td = s_start[1], z_td = s_start[2];
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

// One pair check (planning_utils.cpp:645-881) by a whole wave: every lane
// holds the same Lane state (wave-uniform); per step, lane j evaluates the
// sample j positions ahead on the all-pass path (advance_on_success), then
// every lane replays the reference's transitions on the ballot of results in
// order, stopping at the first failure or decision (the all-pass path crosses
// stage boundaries deterministically) — exactly the reference's samples are
// counted.  Connect actions run t_s / 0.05 + 1
// stance samples (dozens to hundreds): a wave covers 64 of them per step.
template <class ZT, bool ADAPTIVE, int CM>
__device__ bool wave_pair_check(const TerrainView<ZT> &T, const double *s_in, const double *a_in,
                                int dir, double *s_new, double &t_new, uint32_t &flags) {
  const int lane = threadIdx.x & (WAVE - 1);
  double sv[8], av[10];
  copy8(sv, s_in);
  copy10(av, a_in);
  Lane L;
  L.s = sv;
  L.a = av;
  L.f = 0;
  L.acc = Acc{0, 0, 0};
  L.snew_kind = SN_NONE;
  L.tnew_set = 0;
  enter_stage(L, dir == GBP_FORWARD ? ST_FWD_STANCE : ST_REV_FLIGHT);
  bool decided = false;
  while (!decided) {
    int stg = L.stage;
    double t = L.t, ts = L.ts;
    bool has = true;
    for (int k = 0; k < lane && has; k++) has = advance_on_success<ADAPTIVE>(stg, av, t, ts);
    const double t_eval = lane == 0 ? stage_time(L) : sample_time(stg, av, t);
    Acc acc{0, L.acc.V + (uint32_t)lane, 0};
    bool ok = false;
    if (has) {
      double sc[8];
      sample_state(sv, av, stg, t_eval, sc);
      ok = is_valid_state<ZT, CM>(T, sc, stage_phase(stg), acc);
    }
    const unsigned long long okm = __ballot(ok), hasm = __ballot(has);
#ifdef GBP_SEQ_REPLAY
    // A/B arm: the samples replayed one at a time
    for (int j = 0; j < WAVE; j++) {
      if (!((hasm >> j) & 1ull)) break;
      const uint32_t fj = __shfl(acc.flags, j), gj = __shfl(acc.G, j);
      const bool okj = (okm >> j) & 1ull;
      L.acc.G += gj;
      L.acc.flags |= fj;
      if (fj & GBP_F_LIMIT) {
        decided = true;
        break;
      }
      L.acc.V += 1;
      decided = transition<ADAPTIVE>(L, okj);
      if (decided || !okj) break;
    }
#else
    // The replay in parallel.  hasm is a prefix of the lanes (a lane past a
    // deciding sample has none); the run [0, j0) of passing samples ends at
    // the first failing or LIMIT one.  Each lane of the run applies its own
    // sample's success transition to its speculated pre-state (stg, t, ts:
    // the same arithmetic the in-order replay performs), so the attempt's
    // state after the run is the last run lane's; s_new / t_new are the last
    // ones a run lane set; G, flags and V add up over the run.  Then the
    // stop lane's sample, if any, goes through the in-order transition.
    const unsigned long long limm = __ballot(has && (acc.flags & GBP_F_LIMIT));
    const unsigned long long stopm = hasm & (~okm | limm);
    const int j0 = stopm ? __builtin_ctzll(stopm) : __popcll(hasm);
    const bool inrun = lane < j0;
    Lane P = L;
    P.stage = stg;
    P.t = t;
    P.ts = ts;
    P.f = stage_bits((uint32_t)stg);
    P.snew_kind = SN_NONE;
    P.tnew_set = 0;
    bool dec = false;
    if (inrun) dec = transition<ADAPTIVE>(P, true);
    uint32_t g = inrun ? acc.G : 0u, fl = inrun ? acc.flags : 0u;
#pragma unroll
    for (int o = WAVE / 2; o > 0; o >>= 1) {
      g += __shfl_xor(g, o);
      fl |= __shfl_xor(fl, o);
    }
    L.acc.G += g;
    L.acc.flags |= fl;
    L.acc.V += (uint32_t)j0;
    if (j0 > 0) {
      const int jl = j0 - 1;
      L.stage = __shfl(P.stage, jl);
      L.t = __shfl(P.t, jl);
      L.ts = __shfl(P.ts, jl);
      L.tpre = __shfl(P.tpre, jl);
      L.f = __shfl(P.f, jl);
      decided = __shfl((int)dec, jl) != 0;
      const unsigned long long sm = __ballot(inrun && P.snew_kind != SN_NONE);
      if (sm) {
        const int js = 63 - __builtin_clzll(sm);
        L.snew_kind = __shfl(P.snew_kind, js);
        L.snew_p = __shfl(P.snew_p, js);
      }
      const unsigned long long tm = __ballot(inrun && P.tnew_set);
      if (tm) {
        const int jt = 63 - __builtin_clzll(tm);
        L.tnew = __shfl(P.tnew, jt);
        L.tnew_set = 1;
      }
    }
    if (!decided && stopm) {
      const uint32_t fj = __shfl(acc.flags, j0), gj = __shfl(acc.G, j0);
      L.acc.G += gj;
      L.acc.flags |= fj;
      if (fj & GBP_F_LIMIT) {
        decided = true;
      } else {
        L.acc.V += 1;
        decided = transition<ADAPTIVE>(L, ((okm >> j0) & 1ull) != 0);
      }
    }
#endif
  }
  uint32_t f = L.f | L.acc.flags;
  if (L.snew_kind != SN_NONE) {
    f |= GBP_F_SNEW_SET;
    sample_state(sv, av,
                 L.snew_kind == SN_STANCE_S ? ST_FWD_STANCE
                                            : (L.snew_kind == SN_FLIGHT_B ? ST_FWD_LAND : ST_REV_STANCE),
                 L.snew_p, s_new);
  }
  if (L.tnew_set) {
    f |= GBP_F_TNEW_SET;
    t_new = L.tnew;
  }
  flags = f;
  return (f & GBP_F_VALID) != 0;
}

// one wave per new vertex k of T: connect it to its nearest vertex of O with
// the recursion as a loop over levels (engine conventions of gbp.h: an
// unassigned t_new / s_new is TRAPPED; GBP_CONNECT_MAX_DEPTH levels)
template <class ZT, bool ADAPTIVE, int CM>
__global__ __launch_bounds__(TB) void k_connect(TerrainView<ZT> T, gbp_plan_status *st, int cdir,
                                                const double *__restrict__ tv,
                                                const double *__restrict__ ov,
                                                const int32_t *__restrict__ nno,
                                                int32_t *__restrict__ kres,
                                                double *__restrict__ ksn,
                                                double *__restrict__ kan,
                                                uint32_t *__restrict__ kf, int32_t half,
                                                uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t n = st->n_added, base = st->added_base;
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
  bool frag = false;
  unsigned long long capped = 0, checks = 0;
  for (int64_t k = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; k < n;
       k += waves) {
    double se[8], s[8], sn[8], an[10];
    copy8(se, ov + 8 * (int64_t)nno[k]);  // s_near in O (rrt_connect.cpp:101-102)
    copy8(s, tv + 8 * (base + k));
    double t_s = pose_distance(s, se) / V_NOM;  // rrt_connect.cpp:89
    int res = GBP_TRAPPED;
    uint32_t cf = 0;
    for (int depth = 0;; depth++) {
      if (depth > GBP_CONNECT_MAX_DEPTH) {
        cf |= GBP_F_DEPTH_CAPPED;
        break;
      }
      if (t_s <= KINEMATICS_RES) break;  // :23-24
      const double *s_start = cdir == GBP_FORWARD ? se : s;
      const double *s_goal = cdir == GBP_FORWARD ? s : se;
      connect_action(s_start, s_goal, t_s, an);
      if (!is_valid_action(an)) break;  // :66
      double psn[8], ptn = 0;
      uint32_t pf = 0;
      checks++;  // one pair check per level (BatchStats::attempts_checked)
      const bool ok = wave_pair_check<ZT, ADAPTIVE, CM>(T, cdir == GBP_FORWARD ? s_start : s_goal,
                                                        an, cdir, psn, ptn, pf);
      cf |= pf & (GBP_F_OOD | GBP_F_NAN | GBP_F_FRAGILE | GBP_F_LIMIT);
      if (pf & GBP_F_SNEW_SET) copy8(sn, psn);
      if (ok) {
        res = depth == 0 ? GBP_REACHED : GBP_ADVANCED;  // :74-80
        break;
      }
      if (!(pf & GBP_F_TNEW_SET) || !(pf & GBP_F_SNEW_SET)) break;
      copy8(s, psn);  // :77 recurse toward the returned state with t_s = t_new
      t_s = ptn;
    }
    if (lane == 0) {
      kres[k] = res;
      if (res != GBP_TRAPPED) copy8(ksn + 8 * k, sn);
      copy10(kan + 10 * k, an);
      kf[k] = cf;
    }
    frag = frag || (cf & GBP_F_FRAGILE);
    capped += (cf & GBP_F_DEPTH_CAPPED) ? 1 : 0;
  }
  if (lane == 0) {
    if (checks) atomicAdd((unsigned long long *)&st->stat_attempts, checks);
    if (capped) atomicAdd((unsigned long long *)&st->stat_depth_capped, capped);
    if (frag) {
      atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_CONNECT);
      st->halt_half = half;
      raise_gate(st, seq);
    }
  }
}

// ============================================================================
// RRT*-Connect insertion (rrt_star_connect.cpp:12-67), stages 6 and 7
// ============================================================================
// After stage 3 has appended the half's new vertices base + k (parent = their
// nearest vertex, not yet joined), every one is inserted in order as the
// reference's extend does: its neighbourhood is the vertices before it within
// delta (neighborhoodDist, planner_class.cpp:173-182, ascending index); the
// parent is the neighbour that REACHES it cheapest (choose-parent, :31-49),
// then every neighbour it REACHES more cheaply is rewired under it with the g
// of its subtree updated (:51-66, graph_class.cpp:131-138).  The connect
// decisions depend on the states alone, so stage 6 runs all of them at once:
// two per neighbour pair (choose-parent attemptConnect(s_near, s_new) and
// rewire attemptConnect(s_new, s_near), the depth-0 REACHED decision), their
// pair checks on the persistent kernel.  Stage 7 replays the insertions in
// order (one workgroup: a vertex's choices read the g values its predecessors
// left), each choice a block-wide reduction.

constexpr int RB = 1024;  // threads of the single-workgroup star kernels

__device__ __forceinline__ int block_sum_tb(int v, int *sh) {
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  for (int o = WAVE / 2; o > 0; o >>= 1) v += __shfl_down(v, o);
  if (lane == 0) sh[w] = v;
  __syncthreads();
  int t = 0;
  for (int i = 0; i < (int)(blockDim.x / WAVE); i++) t += sh[i];
  __syncthreads();
  return t;
}

// The neighbourhoods are scanned in the vertex map's iteration order
// (gbp_um_order.h: new vertex k sees keys 0..base+k, position p holding key
// um_key_at(p, base+k+1)), split into chunks of `ch` positions: item
// (k, c) = positions [c·ch, (c+1)·ch) of vertex k, k-major, so concatenating the
// items' hits in item order lists each vertex's neighbours in the reference's
// order.  A half adds a few vertices to trees of tens of thousands: one
// workgroup per vertex (the round-5 form) left nearly every CU idle.
constexpr int64_t STAR_CH = 1024;  // positions per item (grown until the items fit)
#ifndef GBP_STAR_GK
#define GBP_STAR_GK 1  // k_star_count / k_star_fill workgroups per CU
#endif
#ifndef GBP_STAR_GC
#define GBP_STAR_GC 2  // k_star_check workgroups (4 waves) per CU
#endif
#ifndef GBP_CONNECT_GC
#define GBP_CONNECT_GC 4  // k_connect workgroups (4 waves, one connection each) per CU
#endif

__device__ __forceinline__ void star_chunking(int64_t n_added, int64_t base, int64_t cap_items,
                                              int64_t ch0, int64_t &ch, int64_t &nch) {
  const int64_t nv = base + n_added;
  ch = ch0;  // STAR_CH (GBP_STAR_CH in tests); cap_items >= the batch >= n_added: it ends
  nch = (nv + ch - 1) / ch;
  while (n_added * nch > cap_items) {
    ch *= 2;
    nch = (nv + ch - 1) / ch;
  }
}

// stage 6a: hits per item; the grid's last workgroup to finish then scans
// them (star_scan_items: the items' offsets, k-major, and each vertex's
// first pair) — one launch, not a count and a one-workgroup scan
// an item's count, published by its workgroup as tile_word(epoch, 1, hits)
// with one agent-scope exchange (no fence: the word carries its own epoch)
__device__ __forceinline__ int64_t star_item_count(gbp_plan_status *st, unsigned long long *cnt,
                                                   int64_t i, uint32_t ep) {
  uint32_t spins = 0;
  for (;;) {
    const unsigned long long x =
        __hip_atomic_fetch_add(&cnt[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)(x >> 32) == ep) return (int64_t)(x & 0x3FFFFFFFu);
    if (++spins > LOOKBACK_SPIN_LIMIT) {  // bounded: report, never hang
      atomicOr(&st->error, 1u);
      return 0;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

__device__ void star_scan_items(gbp_plan_status *st, unsigned long long *cnt, uint32_t ep, int64_t N,
                                int64_t nch, int64_t n, int64_t base, int32_t *__restrict__ ioff,
                                int32_t *__restrict__ off, int64_t *__restrict__ meta,
                                int64_t max_pairs, int32_t half, uint64_t seq) {
  const int nt = (int)blockDim.x;
  const int64_t per = (N + nt - 1) / nt;
  const int64_t lo = min<int64_t>(N, threadIdx.x * per), hi = min<int64_t>(N, lo + per);
  int64_t sum = 0;
  for (int64_t i = lo; i < hi; i++) sum += star_item_count(st, cnt, i, ep);
  // block-wide exclusive scan of the threads' sums: waves, then the wave totals
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  int64_t inc = sum;
  for (int o = 1; o < WAVE; o <<= 1) {
    const int64_t u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  __shared__ int64_t wt[RB / WAVE + 1];
  if (lane == WAVE - 1) wt[w] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int i = 0; i < nt / WAVE; i++) {
      const int64_t v = wt[i];
      wt[i] = run;
      run += v;
    }
    wt[RB / WAVE] = run;
  }
  __syncthreads();
  const int64_t total = wt[RB / WAVE];
  int64_t run = wt[w] + inc - sum;
  for (int64_t i = lo; i < hi; i++) {
    const int32_t o = (int32_t)min<int64_t>(run, 0x7FFFFFFF);
    ioff[i] = o;
    if (i % nch == 0) off[i / nch] = o;  // vertex i / nch starts here
    run += star_item_count(st, cnt, i, ep);
  }
  if (threadIdx.x == 0) {
    off[n] = (int32_t)min<int64_t>(total, 0x7FFFFFFF);
    st->star_pairs = (int32_t)min<int64_t>(total, 0x7FFFFFFF);
    // the replay's own copy: it runs beside the next half, which rewrites st's
    meta[0] = n;
    meta[1] = base;
    meta[2] = min<int64_t>(total, 0x7FFFFFFF);
    st->star_rows = (int32_t)min<int64_t>(2 * total, 0x7FFFFFFF);  // rows = checks (k_star_check)
    st->star_vrows = st->star_rows;
    if (total > max_pairs) {  // the host grows the sets and resumes this half at stage 6
      atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_STAR_PAIRS);
      st->halt_half = half;
      raise_gate(st, seq);
    } else {
      st->stat_star_connects += 2 * total;  // a choose-parent and a rewire connect per pair
    }
  }
}

__global__ __launch_bounds__(RB) void k_star_count(gbp_plan_status *st, const double *__restrict__ tv,
                                                   double delta, unsigned long long *cnt,
                                                   int32_t *__restrict__ ioff, int32_t *__restrict__ off,
                                                   int64_t *__restrict__ meta, int64_t max_pairs,
                                                   uint32_t *__restrict__ fin, int64_t cap_items,
                                                   int64_t ch0, int32_t half, uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t n = st->n_added, base = st->added_base;
  int64_t ch, nch;
  star_chunking(n, base, cap_items, ch0, ch, nch);
  // the workgroups with an item take part in the finish count (the grid is
  // sized for the largest half; most of it exits here); with no items
  // workgroup 0 alone scans (an empty list still resets the half's counts)
  const int64_t N = n * nch, parts = max<int64_t>(1, min<int64_t>(gridDim.x, N));
  const uint32_t ep = (uint32_t)seq;  // this launch's epoch (seq grows every launch)
  if ((int64_t)blockIdx.x >= parts) return;
  __shared__ int sh[RB / WAVE];
  __shared__ bool last;
  for (int64_t it = blockIdx.x; it < N; it += gridDim.x) {
    const int64_t k = it / nch, c = it - k * nch;
    const int64_t nk = base + k + 1;  // the map holds keys 0..base+k (rrt_star_connect.cpp:22)
    const int m = um_epoch(nk);
    double q[8];
    copy8(q, tv + 8 * (base + k));
    const int64_t p1 = min<int64_t>((c + 1) * ch, nk);
    int hits = 0;
    for (int64_t p = c * ch + threadIdx.x; p < p1; p += blockDim.x) {
      const int64_t j = um_key_at(p, nk, m);
      const double d = state_distance(q, tv + 8 * j);  // planner_class.cpp:178
      hits += (d <= delta && d > 0) ? 1 : 0;
    }
    hits = block_sum_tb(hits, sh);
    if (threadIdx.x == 0)
      __hip_atomic_exchange(&cnt[it], tile_word(ep, 1, (uint32_t)hits), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) last = atomicAdd(fin, 1u) == (uint32_t)(parts - 1);
  __syncthreads();
  if (!last) return;
  star_scan_items(st, cnt, ep, N, nch, n, base, ioff, off, meta, max_pairs, half, seq);
  if (threadIdx.x == 0) *fin = 0;  // reset for the next half (stream-ordered)
}

// stage 6c: the neighbour lists, each item's hits in position order at its offset
__global__ __launch_bounds__(RB) void k_star_fill(gbp_plan_status *st, const double *__restrict__ tv,
                                                  double delta, const int32_t *__restrict__ ioff,
                                                  int32_t *__restrict__ nb, int32_t *__restrict__ own,
                                                  int64_t cap_items, int64_t ch0, uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t n = st->n_added, base = st->added_base;
  int64_t ch, nch;
  star_chunking(n, base, cap_items, ch0, ch, nch);
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  __shared__ int wc[RB / WAVE];
  for (int64_t it = blockIdx.x; it < n * nch; it += gridDim.x) {
    const int64_t k = it / nch, c = it - k * nch;
    const int64_t nk = base + k + 1;
    const int m = um_epoch(nk);
    double q[8];
    copy8(q, tv + 8 * (base + k));
    const int64_t p1 = min<int64_t>((c + 1) * ch, nk);
    int64_t run = ioff[it];
    for (int64_t p0 = c * ch; p0 < p1; p0 += blockDim.x) {
      const int64_t p = p0 + threadIdx.x;
      bool hit = false;
      int64_t j = 0;
      if (p < p1) {
        j = um_key_at(p, nk, m);
        const double d = state_distance(q, tv + 8 * j);
        hit = d <= delta && d > 0;
      }
      const unsigned long long bm = __ballot(hit);
      if (lane == 0) wc[w] = __popcll(bm);
      __syncthreads();
      int before = 0, total = 0;
      for (int i = 0; i < (int)(blockDim.x / WAVE); i++) {
        if (i < w) before += wc[i];
        total += wc[i];
      }
      if (hit) {
        const int64_t at = run + before + __popcll(bm & ((1ull << lane) - 1ull));
        nb[at] = (int32_t)j;
        own[at] = (int32_t)k;
      }
      run += total;
      __syncthreads();
    }
  }
}

// stage 6d's connect check c of the half's pairs (rrt_connect.cpp:20-70 at
// depth 0; pair c >> 1 = (new vertex idx, neighbour j); c even: choose-parent
// attemptConnect(s_near, s_new, poseDistance(s_new, s_near) / V_NOM), odd:
// rewire attemptConnect(s_new, s_near, ...)): whether it needs a pair check
// (the rest are not REACHED: t_s <= KINEMATICS_RES or an invalid action,
// :23-24, :66), its action a and the state sp the check starts from
__device__ __forceinline__ bool star_row(const double *__restrict__ tv, int dir, int64_t idx,
                                         int64_t j, bool rewire, double (&a)[10], double (&sp)[8]) {
  double sn[8], sj[8];
  copy8(sn, tv + 8 * idx);
  copy8(sj, tv + 8 * j);
  const double *se = rewire ? sn : sj, *sq = rewire ? sj : sn;  // (s_existing, s)
  const double t_s = (rewire ? pose_distance(sj, sn) : pose_distance(sn, sj)) / V_NOM;
  if (!(t_s > KINEMATICS_RES)) return false;
  const double *s_start = dir == GBP_FORWARD ? se : sq, *s_goal = dir == GBP_FORWARD ? sq : se;
  connect_action(s_start, s_goal, t_s, a);
  copy8(sp, dir == GBP_FORWARD ? s_start : s_goal);
  return is_valid_action(a);
}

// stage 6e: the connect checks, one wave per check c: its action
// (star_row, every lane alike) and, when it has one, its pair check
// (wave_pair_check, as k_connect: the 64 lanes evaluate 64 successive
// samples of the action, then replay them in order).  The checks are few
// (hundreds per half) and their actions long (connect actions, tens of
// samples): the persistent validate kernel's fixed cost was ~90 us for them
// (63 us per half in the planner), this one's a few steps of one wave per
// check.  Rows are the checks themselves (row c: rs / ra / rf[c], rowof[c]
// = c or -1; rf[c] = 0 for a check with no pair check); flags as
// gbp_validate's (no s_new / t_new kept).  A FRAGILE decision halts the
// sequence (the host re-decides it with glibc and resumes at stage 7).
template <class ZT, bool ADAPTIVE, int CM>
__global__ __launch_bounds__(TB) void k_star_check(TerrainView<ZT> T, gbp_plan_status *st, int dir,
                                                   const double *__restrict__ tv,
                                                   const int32_t *__restrict__ nb,
                                                   const int32_t *__restrict__ own,
                                                   int32_t *__restrict__ rowof, double *__restrict__ rs,
                                                   double *__restrict__ ra, uint32_t *__restrict__ rf,
                                                   int32_t half, uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t m = 2 * (int64_t)st->star_pairs, base = st->added_base;
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t wv = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const int64_t nw = (int64_t)gridDim.x * blockDim.x / WAVE;
  uint32_t rows = 0;
  for (int64_t c = wv; c < m; c += nw) {
    double a[10], sp[8];
    const int64_t pr = c >> 1;
    const bool row = star_row(tv, dir, base + own[pr], nb[pr], (c & 1) != 0, a, sp);
    uint32_t f = 0;
    if (row) {
      double sn[8], tn = 0;
      wave_pair_check<ZT, ADAPTIVE, CM>(T, sp, a, dir, sn, tn, f);
      rows++;
    }
    if (lane == 0) {
      rowof[c] = row ? (int32_t)c : -1;
      rf[c] = f;
      if (row) {
        copy8(rs + 8 * c, sp);
        copy10(ra + 10 * c, a);
      }
      if (f & GBP_F_FRAGILE) {
        atomicOr(&st->halt, (uint32_t)GBP_PLAN_HALT_STAR);
        st->halt_half = half;
        raise_gate(st, seq);
      }
    }
  }
  if (lane == 0 && rows)  // the pair checks (engine attempts) made
    atomicAdd((unsigned long long *)&st->stat_attempts, (unsigned long long)rows);
}

// block-wide (min key, min index) over the RB threads; NaN keys never win
__device__ void block_argmin(double &key, int64_t &at, double *kd, int64_t *ki) {
  kd[threadIdx.x] = key;
  ki[threadIdx.x] = at;
  __syncthreads();
  for (int o = RB / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const double k2 = kd[threadIdx.x + o];
      const int64_t i2 = ki[threadIdx.x + o];
      const double k1 = kd[threadIdx.x];
      const int64_t i1 = ki[threadIdx.x];
      if (i2 >= 0 && (i1 < 0 || k2 < k1 || (k2 == k1 && i2 < i1))) {
        kd[threadIdx.x] = k2;
        ki[threadIdx.x] = i2;
      }
    }
    __syncthreads();
  }
  key = kd[0];
  at = ki[0];
  __syncthreads();
}

// Stage 7 runs on ONE wave: a half inserts a few vertices (~3 at config 5),
// each with ~100 neighbours, ~2 rewires and subtree updates of ~17 vertices
// over ~1-2 levels (oracle statistics of config 5's continuation), so its
// length is a chain of dependent steps — a 1024-thread workgroup paid a
// 10-barrier reduction ladder per choice and a 16-wave barrier per subtree
// level (61 us per half); one wave reduces by shuffles and its barriers
// cost nothing.
constexpr int RW = 64;

// wave-wide lexicographic (key, position) minimum; position < 0 never wins,
// NaN keys never win (the loops only keep comparable keys)
__device__ __forceinline__ void wave_argmin(double &key, int64_t &at) {
#pragma unroll
  for (int o = RW / 2; o > 0; o >>= 1) {
    const double k2 = __shfl_xor(key, o);
    const int64_t i2 = __shfl_xor(at, o);
    if (i2 >= 0 && (at < 0 || k2 < key || (k2 == key && i2 < at))) {
      key = k2;
      at = i2;
    }
  }
}

// wave-wide least non-negative position (-1 if none)
__device__ __forceinline__ int64_t wave_first(int64_t at) {
#pragma unroll
  for (int o = RW / 2; o > 0; o >>= 1) {
    const int64_t i2 = __shfl_xor(at, o);
    if (i2 >= 0 && (at < 0 || i2 < at)) at = i2;
  }
  return at;
}

// g over the subtree below vertex r (graph_class.cpp:131-138: every successor's
// g = its parent's + poseDistance), level by level, the wave's lanes taking a
// level's vertices; the queues hold (vertex, g) in LDS up to RQ entries per
// level, in the tree's scratch past that (bounded: a list that is not a tree —
// never built here — stops at nv vertices and returns false)
constexpr int RQ = 2048;
__device__ bool subtree_g(const double *__restrict__ tv, double *tg, const int32_t *tch,
                          const int32_t *tsib, int32_t r, double gr, int32_t *q0, int32_t *q1,
                          int32_t nv, int32_t rq) {
  __shared__ int32_t lq[2][RQ];
  __shared__ double lg[2][RQ];
  __shared__ int32_t s_next;
  int32_t nq = 1, total = 1, cur = 0;
  if (threadIdx.x == 0) {
    lq[0][0] = r;
    lg[0][0] = gr;
    s_next = 0;
  }
  __syncthreads();
  while (nq > 0) {
    for (int32_t i = threadIdx.x; i < nq; i += RW) {
      const int32_t p = i < rq ? lq[cur][i] : q0[i];
      const double gp = i < rq ? lg[cur][i] : tg[p];
      double vp[8];
      copy8(vp, tv + 8 * (int64_t)p);
      for (int32_t c = tch[p]; c >= 0; c = tsib[c]) {
        const double gc = gp + pose_distance(vp, tv + 8 * (int64_t)c);
        tg[c] = gc;
        const int32_t slot = atomicAdd(&s_next, 1);
        if (slot >= nv) break;
        if (slot < rq) {
          lq[cur ^ 1][slot] = c;
          lg[cur ^ 1][slot] = gc;
        } else {
          q1[slot] = c;
        }
      }
    }
    __syncthreads();
    const int32_t next = s_next;
    __syncthreads();
    if (threadIdx.x == 0) s_next = 0;
    total += min(next, nv);
    if (next > nv || total > nv) return false;
    nq = next;
    int32_t *t = q0;
    q0 = q1;
    q1 = t;
    cur ^= 1;
    __syncthreads();
  }
  return true;
}

// addEdge(p, c)'s successor entry: c becomes p's first child
__device__ __forceinline__ void link_child(int32_t *tch, int32_t *tsib, int32_t *tprev, int32_t p,
                                           int32_t c) {
  const int32_t h = tch[p];
  tsib[c] = h;
  tprev[c] = -1;
  if (h >= 0) tprev[h] = c;
  tch[p] = c;
}

// the half's pairs, what the replay needs of them that no insertion changes:
// the neighbour, poseDistance(neighbour, s_new) (:35 and :59 alike, argument
// order included) and whether its choose-parent (bit 0) / rewire (bit 1)
// connection REACHED; the first RP in LDS (the prologue fills them), the rest
// recomputed from global memory where read
constexpr int RP = 2048;  // pairs held in LDS (config 5: ~300 per half)
constexpr int RS = 4;     // a lane's neighbour slots per insertion in registers
constexpr int RK = 512;   // new vertices held in LDS (their nearest vertex and g0's distance)

// what the replay keeps in LDS (tests shrink it: GBP_STAR_LDS = "rp,rk,rq")
struct StarLds {
  int32_t rp = RP, rk = RK, rq = RQ;
};

struct PairInfo {
  int32_t j;
  uint32_t f;
  double d;
};

__device__ __forceinline__ PairInfo pair_info_global(int64_t i, const double *__restrict__ tv,
                                                     int64_t base, const int32_t *__restrict__ nb,
                                                     const int32_t *__restrict__ own,
                                                     const int32_t *__restrict__ rowof,
                                                     const uint32_t *__restrict__ rf) {
  PairInfo pi;
  pi.j = nb[i];
  const int32_t r0 = rowof[2 * i], r1 = rowof[2 * i + 1];
  pi.f = ((r0 >= 0 && (rf[r0] & GBP_F_VALID)) ? 1u : 0u) |
         ((r1 >= 0 && (rf[r1] & GBP_F_VALID)) ? 2u : 0u);
  pi.d = pose_distance(tv + 8 * (int64_t)pi.j, tv + 8 * (base + own[i]));
  return pi;
}

// stage 7: the ordered replay of rrt_star_connect.cpp:18-66, one wave
__global__ __launch_bounds__(RW) void k_star_replay(gbp_plan_status *st, const double *__restrict__ tv,
                                                    double *ta, double *tg, int32_t *tp, int32_t *tch,
                                                    int32_t *tsib, int32_t *tprev,
                                                    const int32_t *__restrict__ off,
                                                    const int32_t *__restrict__ nb,
                                                    const int32_t *__restrict__ own,
                                                    const int32_t *__restrict__ rowof,
                                                    const double *__restrict__ ra,
                                                    const uint32_t *__restrict__ rf,
                                                    const int64_t *__restrict__ meta, int32_t *q0,
                                                    int32_t *q1, const int32_t *tcount, StarLds lim,
                                                    uint64_t seq) {
  if (gated(st, seq)) return;
  const int32_t rp = lim.rp, rk = lim.rk;  // (RP, RK; smaller in tests: the global paths)
  const int64_t n = meta[0], base = meta[1], npairs = meta[2];
  const int32_t nv = *tcount;
  const int lane = threadIdx.x;
  __shared__ int32_t lj[RP];
  __shared__ uint32_t lf[RP];
  __shared__ double ld[RP];
  __shared__ int32_t lnn[RK], loff[RK + 1];
  __shared__ double ld0[RK];
  // prologue: every pair's static part and every new vertex's nearest vertex,
  // its offsets and poseDistance(s_new, s_nearest) (:28), all lanes at once
  for (int64_t i = lane; i < min<int64_t>(npairs, rp); i += RW) {
    const PairInfo pi = pair_info_global(i, tv, base, nb, own, rowof, rf);
    lj[i] = pi.j;
    lf[i] = pi.f;
    ld[i] = pi.d;
  }
  for (int64_t k = lane; k < min<int64_t>(n, rk); k += RW) {
    const int32_t nn = tp[base + k];  // stage 3 wrote the nearest vertex here
    lnn[k] = nn;
    ld0[k] = pose_distance(tv + 8 * (base + k), tv + 8 * (int64_t)nn);
    loff[k] = off[k];
  }
  const int64_t nk_l = n < rk ? n : rk;
  if (lane == 0) loff[nk_l] = off[nk_l];
  __syncthreads();
  auto pair = [&](int64_t i) -> PairInfo {
    if (i < rp) return PairInfo{lj[i], lf[i], ld[i]};
    return pair_info_global(i, tv, base, nb, own, rowof, rf);
  };
  int64_t rewires = 0;
  for (int64_t k = 0; k < n; k++) {
    const int32_t idx = (int32_t)(base + k);
    const int32_t nn = k < rk ? lnn[k] : tp[idx];
    const double d0 = k < rk ? ld0[k] : pose_distance(tv + 8 * (int64_t)idx, tv + 8 * (int64_t)nn);
    const int64_t i0 = k < rk ? loff[k] : off[k], i1 = k + 1 <= rk ? loff[k + 1] : off[k + 1];
    // this lane's first RS neighbours (positions i0 + lane + RW s)
    int32_t sj[RS];
    uint32_t sf[RS];
    double sd[RS];
#pragma unroll
    for (int q = 0; q < RS; q++) {
      const int64_t i = i0 + lane + RW * q;
      sf[q] = 0;
      sj[q] = 0;
      sd[q] = 0;
      if (i < i1) {
        const PairInfo pi = pair(i);
        sj[q] = pi.j;
        sf[q] = pi.f;
        sd[q] = pi.d;
      }
    }
    const int64_t ix = i0 + (int64_t)RW * RS;  // positions past the slots
    // choose-parent (:27-44): from the nearest vertex, the first neighbour whose
    // REACHED connection is strictly cheaper than the best so far — the first
    // in the map's order of the cheapest, when that beats the nearest vertex's
    double key = INFINITY;
    int64_t at = -1;
    double gq[RS];
#pragma unroll
    for (int q = 0; q < RS; q++) gq[q] = (sf[q] & 1u) ? tg[sj[q]] : 0.0;
    const double g0 = tg[nn] + d0;  // :28
#pragma unroll
    for (int q = 0; q < RS; q++) {
      if (!(sf[q] & 1u)) continue;
      const double gc = gq[q] + sd[q];  // :35
      if (gc == gc && (at < 0 || gc < key)) {  // the first of this lane's minimum
        key = gc;
        at = i0 + lane + RW * q;
      }
    }
    for (int64_t i = ix + lane; i < i1; i += RW) {
      const PairInfo pi = pair(i);
      if (!(pi.f & 1u)) continue;
      const double gc = tg[pi.j] + pi.d;
      if (gc == gc && (at < 0 || gc < key)) {
        key = gc;
        at = i;
      }
    }
    wave_argmin(key, at);
    int32_t pmin = nn;
    double gn = g0;
    int64_t row = -1;
    if (at >= 0 && key < g0) {
      pmin = pair(at).j;
      gn = key;
      row = rowof[2 * at];
    }
    // addEdge(s_min, s_new) + updateGYValue + addAction (:47-49)
    if (lane == 0) {
      tp[idx] = pmin;
      link_child(tch, tsib, tprev, pmin, idx);
      tg[idx] = gn;
    }
    if (row >= 0 && lane < 10) ta[10 * (int64_t)idx + lane] = ra[10 * row + lane];
    __syncthreads();
    // rewire (:51-66): in neighbour order; a rewire's subtree update can change
    // the g a later neighbour is tested with, so each round finds the first
    // neighbour (from the cursor on) that rewires now
    for (int64_t cur = i0; cur < i1;) {
      const double gi = tg[idx];
#pragma unroll
      for (int q = 0; q < RS; q++)
        gq[q] = ((sf[q] & 2u) && sj[q] != pmin && i0 + lane + RW * q >= cur) ? tg[sj[q]] : 0.0;
      at = -1;
#pragma unroll
      for (int q = 0; q < RS; q++) {
        const int64_t i = i0 + lane + RW * q;
        if (at < 0 && (sf[q] & 2u) && sj[q] != pmin && i >= cur && gq[q] > (gi + sd[q])) at = i;
      }
      if (at < 0) {
        for (int64_t i = max(ix, cur) + ((lane - (max(ix, cur) - i0)) % RW + RW) % RW; i < i1; i += RW) {
          const PairInfo pi = pair(i);
          if (!(pi.f & 2u) || pi.j == pmin) continue;
          if (tg[pi.j] > (gi + pi.d)) {
            at = i;
            break;  // a lane's candidates ascend: its first is its least
          }
        }
      }
      at = wave_first(at);
      if (at < 0) break;
      const PairInfo pj = pair(at);
      const int32_t j = pj.j;
      const int64_t rrow = rowof[2 * at + 1];
      const double gj = gi + pj.d;  // updateGYValue (:60)
      if (lane == 0) {
        // removeEdge(parent, j) (graph_class.cpp:44-58) + addEdge(s_new, j): j
        // leaves its parent's list (never s_new's: s_new's children are the
        // vertices rewired before it) for the head of s_new's; every load first
        const int32_t op = tp[j], pv = tprev[j], nx = tsib[j], h = tch[idx];
        const int32_t oh = op >= 0 ? tch[op] : -1;
        if (op >= 0) {
          if (pv >= 0)
            tsib[pv] = nx;
          else if (oh == j)
            tch[op] = nx;
          if (nx >= 0) tprev[nx] = pv;
        }
        tsib[j] = h;
        tprev[j] = -1;
        if (h >= 0) tprev[h] = j;
        tch[idx] = j;
        tp[j] = idx;
        tg[j] = gj;
      }
      if (lane < 10) ta[10 * (int64_t)j + lane] = ra[10 * rrow + lane];
      __syncthreads();
      rewires++;
      // the rewired vertex's successors (recursion of updateGYValue)
      if (tch[j] >= 0 && !subtree_g(tv, tg, tch, tsib, j, gj, q0, q1, nv, lim.rq)) {
        if (lane == 0) {
          atomicOr(&st->error, 8u);  // a successor list that is not a tree
          raise_gate(st, seq);
        }
        return;
      }
      __syncthreads();
      cur = at + 1;
    }
  }
  if (lane == 0 && rewires) st->stat_rewires += rewires;
}

// after Tb's half (star_stream, behind both trees' replays): the cheapest
// of the meta[3] connections listed so far ranked with the current g values
// (:181-193: strictly cheaper than the best so far; ties to the first)
__global__ __launch_bounds__(RB) void k_star_rank(gbp_plan_status *st, const int32_t *__restrict__ shared,
                                                  const int64_t *__restrict__ meta,
                                                  const double *__restrict__ ga,
                                                  const double *__restrict__ gb, uint64_t seq) {
  if (gated(st, seq)) return;
  const int64_t ns = meta[3];
  __shared__ double kd[RB];
  __shared__ int64_t ki[RB];
  double key = INFINITY;
  int64_t at = -1;
  for (int64_t p = threadIdx.x; p < ns; p += RB) {
    const double c = ga[shared[2 * p]] + gb[shared[2 * p + 1]];
    if (c == c && (at < 0 || c < key)) {
      key = c;
      at = p;
    }
  }
  block_argmin(key, at, kd, ki);
  if (threadIdx.x == 0 && at >= 0 && key < st->best_cost) {
    st->best_cost = key;
    st->best_a = shared[2 * at];
    st->best_b = shared[2 * at + 1];
  }
}

__global__ void k_tree_init(gbp_tree t, double r0, double r1, double r2, double r3, double r4,
                            double r5, double r6, double r7) {
  const double r[8] = {r0, r1, r2, r3, r4, r5, r6, r7};
  copy8(t.v, r);
  nn_put_hrow(t.vh, t.hm, 0, r, true);
  for (int k = 0; k < 10; k++) t.a[k] = 0.0;
  t.g[0] = 0.0;
  t.parent[0] = -1;
  t.child[0] = -1;
  t.sibling[0] = -1;
  t.prev[0] = -1;
  *t.count = 1;
}

__global__ void k_tree_append(gbp_tree t, int64_t n, const double *__restrict__ s,
                              const double *__restrict__ a, const int32_t *__restrict__ p) {
  // sequential in index order: a parent may be appended in the same call
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  int32_t c = *t.count;
  for (int64_t i = 0; i < n; i++, c++) {
    copy8(t.v + 8 * (int64_t)c, s + 8 * i);
    nn_put_hrow(t.vh, t.hm, c, s + 8 * i, false);
    copy10(t.a + 10 * (int64_t)c, a + 10 * i);
    t.parent[c] = p[i];
    t.g[c] = p[i] >= 0 ? t.g[p[i]] + pose_distance(t.v + 8 * (int64_t)p[i], s + 8 * i) : 0.0;
    t.child[c] = -1;
    t.sibling[c] = -1;
    t.prev[c] = -1;
    if (p[i] >= 0) {
      const int32_t h = t.child[p[i]];
      t.sibling[c] = h;
      if (h >= 0) t.prev[h] = c;
      t.child[p[i]] = c;
    }
  }
  *t.count = c;
}

// gbp_tree_load_host: the given vertices, successor lists, then g from the
// root down through the two level queues (one lane: a test's warm start)
__global__ void k_tree_load(gbp_tree t, int64_t n, const double *__restrict__ s,
                            const double *__restrict__ a, const int32_t *__restrict__ p) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (int64_t i = 0; i < n; i++) {
    copy8(t.v + 8 * i, s + 8 * i);
    nn_put_hrow(t.vh, t.hm, i, s + 8 * i, i == 0);
    copy10(t.a + 10 * i, a + 10 * i);
    t.parent[i] = p[i];
    t.child[i] = -1;
    t.sibling[i] = -1;
    t.prev[i] = -1;
  }
  for (int64_t i = 1; i < n; i++) {
    const int32_t h = t.child[p[i]];
    t.sibling[i] = h;
    if (h >= 0) t.prev[h] = (int32_t)i;
    t.child[p[i]] = (int32_t)i;
  }
  int32_t *q = t.bfs;
  int64_t qh = 0, qt = 0;
  t.g[0] = 0.0;
  q[qt++] = 0;
  while (qh < qt) {
    const int32_t u = q[qh++];
    for (int32_t c = t.child[u]; c >= 0 && qt < n; c = t.sibling[c]) {
      t.g[c] = t.g[u] + pose_distance(t.v + 8 * (int64_t)u, t.v + 8 * (int64_t)c);
      q[qt++] = c;
    }
  }
  *t.count = (int32_t)n;
}

__global__ void k_plan_reset(gbp_plan_status *st, int64_t ext_counter, gbp_plan_la *la) {
  *la = gbp_plan_la{};  // no drawn-ahead targets, empty snapshots
  gbp_plan_status z;
  memset(&z, 0, sizeof z);
  z.meet = ~0ull;
  z.gate_seq = ~0ull;
  z.halt_half = -1;
  z.ext_half = -1;
  z.meet_half = -1;
  z.ext_counter = ext_counter;
  z.best_a = z.best_b = -1;
  z.best_cost = INFINITY;
  *st = z;
}

// standalone gbp_extend_tree_dev: the batch becomes stage 2's targets
__global__ void k_extend_setup(gbp_plan_status *st, int64_t n, const int32_t *n_dev,
                               int64_t extend_base, const double *__restrict__ src,
                               double *__restrict__ targets, _Float16 *__restrict__ tqh) {
  const int64_t m = n_dev ? *n_dev : n;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    st->halt = 0;
    st->done = 0;
    st->gate_seq = ~0ull;
    st->n_targets = (int32_t)m;
    st->ext_base = extend_base;
  }
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < 8 * m;
       i += (int64_t)gridDim.x * blockDim.x)
    targets[i] = src[i];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x)
    nn_put_hrow(tqh, nullptr, i, src + 8 * i, false);  // the search's query rows
}

__global__ void k_set_queries(gbp_plan_status *st, int32_t n) {
  st->halt = 0;
  st->done = 0;
  st->gate_seq = ~0ull;
  st->n_targets = n;
}

__global__ void k_extend_out(const gbp_plan_status *st, int64_t n, const int32_t *__restrict__ eres,
                             const int32_t *__restrict__ evtx, int32_t *__restrict__ result,
                             int32_t *__restrict__ new_vertex) {
  if (st->halt) return;  // FRAGILE: gbp_extend_tree_finish_dev after the resolution
  const int64_t m = st->n_targets;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < m;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (result) result[i] = eres[i];
    if (new_vertex) new_vertex[i] = eres[i] != GBP_TRAPPED ? evtx[i] : -1;
  }
}

#define HIPCHK_P(expr)                        \
  do {                                        \
    hipError_t e_ = (expr);                   \
    if (e_ != hipSuccess) return GBP_E_HIP;   \
  } while (0)

bool tree_ok(const gbp_tree *t) { return t && t->v && t->count; }

// the target set of half `half` (its parity)
void select_targets(gbp_plan_ws *w, int32_t half) {
  const auto &ts = w->tset[half % 3];
  w->cand = ts.cand;
  w->cflag = ts.cflag;
  w->targets = ts.targets;
  w->tqh = ts.tqh;
  w->nn = w->nnp[half & 1];
  w->cs = w->csp[half & 1];
  w->ca = w->cap[half & 1];
}

uint32_t next_epoch(gbp_plan_ws *w) {
  if (++w->epoch == 0) w->epoch = 1;
  return w->epoch;
}

unsigned tiles_for(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + CB - 1) / CB); }

// qh: the queries' fp16 rows (nn_put_hrow layout, same offsets as q), or
// null (converted in the search); prep: the extends' candidates are drawn
// inside the search (returns *prepped); side: the look-ahead search's launch
// (its own partial slots, never gated, the tree's snapshot count)
struct NnSide {
  const int32_t *nv;   // the searched tree's vertex count at the snapshot
  const uint32_t *go;  // 0: idle
};
template <class ZT = float>
int nn_launch(gbp_plan_ws *w, const int32_t *nq_dev, const double *q, const int32_t *q_off_dev,
              const gbp_tree *tr, int32_t *out, int num_cus, hipStream_t s,
              const _Float16 *qh = nullptr, const NhPrep<ZT> *prep = nullptr,
              double *cs = nullptr, bool *prepped = nullptr, const NnSide *side = nullptr,
              bool small = false, bool small_any = false) {
  if (prepped) *prepped = false;
  // small: up to NS_MAXQ queries take the direct fp64 search (k_nn_small),
  // the matrix-core pair then returns at once (the count is on the device)
  const int small_max = small && !prep ? NS_MAXQ : 0;
  // ... and when k_nn_small's partials hold a whole batch of queries (the
  // workspace's max_batch, which bounds the count), it takes every count and
  // the other four launches are not made at all: in the steady state of the
  // planner and of config 5 they returned at once but cost ~21 us of the
  // caller's stream per half (the connects' queries are the half's new
  // vertices, a few; a large count is slower this way, never wrong)
  const bool direct_only = small_any && small_max && !side && w->ns_capq >= w->bmax;
  if (small_max)
    // one workgroup per CU of an XCD: in the planner the look-ahead search
    // holds the other seven (32 blocks 171.8 M extends/s, 64: 171.2, 128:
    // 169.3, 512: 160.8, the matrix-core pair alone 169.2; r05k_small_ab*.txt)
    hipLaunchKernelGGL(k_nn_small, dim3(w->ns_grid), dim3(NS_TB), 0, s, w->st, nq_dev, q, q_off_dev,
                       tr->v, side ? side->nv : tr->count, out, w->ns_d, w->ns_i, w->ns_fin,
                       direct_only ? w->ns_capq : (int64_t)NS_MAXQ, side ? 0 : ++w->seq);
  if (direct_only) return hipGetLastError() == hipSuccess ? GBP_OK : GBP_E_HIP;
  const int items = w->nn_items;
  const int gm = items / (NH_TB / WAVE);  // the search's workgroups: one wave per item
  float4 *pm = (float4 *)(side ? w->nn_d2 : w->nn_d);
  int4 *pid = (int4 *)(side ? w->nn_i2 : w->nn_i);
  const int32_t *nv = side ? side->nv : tr->count;
  const uint32_t *go = side ? side->go : nullptr;
  if (prep) {
    NhPrep<ZT> pp = *prep;
    const int gd = pp.dr.draw_blocks;
    pp.first_block = gd + gm;
    const int gp = (int)grid_for(GBP_NUM_GEN_STATES * w->bmax, NH_TB, num_cus * 4);
    hipLaunchKernelGGL((k_nn_mfma<NH_NT, ZT, true>), dim3(gd + gm + gp), dim3(NH_TB), 0, s, w->st,
                       nq_dev, q, q_off_dev, qh, tr->vh, tr->hm, nv, w->bmax, pm, pid,
                       side ? 0 : ++w->seq, items, pp, go, 0, w->nsb[side ? 1 : 0].cnt);
    if (prepped) *prepped = true;
  } else {
    hipLaunchKernelGGL((k_nn_mfma<NH_NT, float, false>), dim3(gm), dim3(NH_TB), 0, s, w->st,
                       nq_dev, q, q_off_dev, qh, tr->vh, tr->hm, nv, w->bmax, pm, pid,
                       side ? 0 : ++w->seq, items, NhPrep<float>{}, go, small_max, w->nsb[side ? 1 : 0].cnt);
  }
  hipLaunchKernelGGL(k_nn_hreduce, dim3(grid_for(NH_G * w->bmax, NH_RTB, num_cus * 8)),
                     dim3(NH_RTB), 0, s, w->st, nq_dev, q, q_off_dev, tr->v, tr->hm, nv, w->bmax,
                     (const float4 *)pm, (const int4 *)pid, out, side ? 0 : ++w->seq, w->nn_stats,
                     prep ? cs : nullptr, items, go, small_max, w->nsb[side ? 1 : 0]);
  hipLaunchKernelGGL(k_nn_scan, dim3(num_cus * 4), dim3(NSC_TB), 0, s, nq_dev, q, q_off_dev, tr->v, nv,
                     w->bmax, items, w->nsb[side ? 1 : 0]);
  hipLaunchKernelGGL(k_nn_scan_merge, dim3(16), dim3(NSM_TB), 0, s, w->nsb[side ? 1 : 0], tr->v, out,
                     prep ? cs : nullptr);
  return hipGetLastError() == hipSuccess ? GBP_OK : GBP_E_HIP;
}

// the look-ahead search of gbp_plan_halves_dev (targets not direction-biased,
// float heights, RRT-Connect): half h + 1's targets are drawn ahead (by half
// h's own search launch, or by half h's look-ahead search) and searched in
// O — the tree half h + 1 extends, unchanged until half h's connects — on
// la_stream while half h validates, selects, appends and connects on the
// caller's stream; half h + 1 then starts with k_la_commit (the commit and
// the vertices O gained since).  Same draws, ranks, nearest vertices and
// counters as the inline sequence.
struct LaHalf {
  bool searched = false;     // this half's targets and search came from the look-ahead
  bool launch_next = false;  // launch half + 1's look-ahead search
  bool draw_after = false;   // ... which draws half + 2's targets
  uint64_t stream_a = 0, stream_b = 0;  // the halves' target streams
};

// the targets of half h drawn ahead into their set (la->nt / frag count them)
NhDraw la_draw(gbp_plan_ws *w, int32_t h, int64_t batch, const LaHalf &L) {
  NhDraw d{};
  const auto &set = w->tset[h % 3];
  d.half = h;
  d.n = batch;
  d.base = (int64_t)(h >> 1) * batch;
  d.stream = (h & 1) ? L.stream_b : L.stream_a;
  d.cand = set.cand;
  d.targets = set.targets;
  d.cflag = set.cflag;
  d.tqh = set.tqh;
  d.draw_blocks = (int)((batch + NH_TB - 1) / NH_TB);
  d.tiles = w->la_tiles;
  d.epoch = next_epoch(w);
  d.count = &w->la->nt[h % 3];
  d.frag = &w->la->frag[h % 3];
  return d;
}

// enqueue half h1's look-ahead search on la_stream after everything the
// caller's stream holds so far; X: the tree h1 extends
int la_launch(gbp_terrain *t, gbp_plan_ws *w, const gbp_tree *X, int32_t h1, int64_t batch,
              uint64_t seed, const LaHalf &L, hipStream_t s) {
  HIPCHK_P(hipEventRecord(w->la_go, s));
  HIPCHK_P(hipStreamWaitEvent(w->la_stream, w->la_go, 0));
  const int slot = h1 % 3, p = h1 & 1;
  const auto &set = w->tset[slot];
  NhPrep<float> prep{view<float>(t), seed, w->cap[p], t->sampling,
                     (h1 & 1) ? GBP_REVERSE : GBP_FORWARD, 0, NhDraw{}, &w->la->nt[slot]};
  if (L.draw_after) prep.dr = la_draw(w, h1 + 1, batch, L);
  const NnSide side{&w->la->nv[p], &w->la->go[p]};
  int rc = nn_launch<float>(w, &w->la->nt[slot], set.targets, nullptr, X, w->nnp[p], t->num_cus,
                            w->la_stream, set.tqh, &prep, w->csp[p], nullptr, &side);
  if (rc) return rc;
  HIPCHK_P(hipEventRecord(w->la_done, w->la_stream));
  return GBP_OK;
}

// gbp_plan_stage_timing: fold every completed timed half into the sums
void timing_collect(gbp_plan_ws *w, bool wait) {
  for (size_t i = 0; i < w->ntring; i++) {
    auto &h = w->tring[i];
    if (!h.pending) continue;
    if (wait) (void)hipEventSynchronize(h.ev[5]);
    if (hipEventQuery(h.ev[5]) != hipSuccess) continue;
    float ms[7] = {0, 0, 0, 0, 0, 0, 0};
    (void)hipEventElapsedTime(&ms[0], h.ev[0], h.ev[5]);
    (void)hipEventElapsedTime(&ms[1], h.ev[0], h.ev[1]);
    if (h.star) {
      (void)hipEventElapsedTime(&ms[2], h.ev[1], h.ev[2]);
      (void)hipEventElapsedTime(&ms[3], h.ev[3], h.ev[4]);
      (void)hipEventElapsedTime(&ms[4], h.ev[2], h.ev[5]);
      (void)hipEventElapsedTime(&ms[5], h.ev[1], h.ev[6]);
      (void)hipEventElapsedTime(&ms[6], h.ev[6], h.ev[7]);
    } else {
      (void)hipEventElapsedTime(&ms[4], h.ev[1], h.ev[5]);
    }
    for (int k = 0; k < 7; k++) w->tsum[k] += 1e3 * (double)ms[k];
    w->tcount++;
    h.pending = false;
  }
}

// the next timing slot (its previous half folded in first), or nullptr
gbp_plan_ws::TimedHalf *timing_slot(gbp_plan_ws *w) {
  if (!w->timing || !w->ntring) return nullptr;
  gbp_plan_ws::TimedHalf *h = &w->tring[w->tnext];
  w->tnext = (w->tnext + 1) % w->ntring;
  if (h->pending) timing_collect(w, true);
  return h;
}

template <class ZT>
int enqueue_stages(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, gbp_tree *O, int32_t half,
                   int direction, int64_t batch, uint64_t seed, uint64_t target_stream,
                   int64_t target_base, int adaptive, int first_stage, int last_stage,
                   hipStream_t s, const LaHalf *la = nullptr) {
  const TerrainView<ZT> V = view<ZT>(t);
  const int cus = t->num_cus;
  gbp_plan_status *st = w->st;
  w->nn_stats = t->opt_nn_stats;
  select_targets(w, half);
  // stage order: 0 1 2 3 (RRT*: 6 7) 4 5 — the RRT* insertion runs between
  // the extends' append and the connects
  auto ord = [](int x) { return x == 6 ? 31 : x == 7 ? 32 : 10 * x; };
  auto run = [&](int x) { return ord(first_stage) <= ord(x) && ord(x) <= ord(last_stage); };
  const bool searched = la && la->searched;  // stages 0-2's draws and search done ahead
  if (searched && first_stage != 0) return GBP_E_INVALID_ARG;
  // whole halves only (a resumed one is not timed)
  gbp_plan_ws::TimedHalf *th = (O && first_stage == 0 && last_stage == 5) ? timing_slot(w) : nullptr;
  if (th) {
    th->star = w->star != 0;
    th->half = half;
    HIPCHK_P(hipEventRecord(th->ev[0], s));
  }
  if (searched && (!std::is_same_v<ZT, float> || t->sampling.state_flag || t->sampling.action_flag))
    return GBP_E_INVALID_ARG;
  if (searched) {
    HIPCHK_P(hipStreamWaitEvent(s, w->la_done, 0));
    hipLaunchKernelGGL(k_la_commit, dim3(grid_for(batch, TB, cus * 4)), dim3(TB), 0, s, st, w->la, half,
                       w->targets, T->v, T->count, w->nn, w->cs, O->count, ++w->seq);
    if (la->launch_next) {
      const int rc = la_launch(t, w, O, half + 1, batch, seed, *la, s);
      if (rc) return rc;
    }
  } else if (run(0) && run(1))  // a fresh half: draws + compaction, one launch
    hipLaunchKernelGGL(k_targets<ZT>, dim3((unsigned)((batch + TB - 1) / TB)), dim3(TB), 0, s, V,
                       st, batch, seed, target_stream, target_base, w->cand, w->cflag, w->targets,
                       w->tqh, w->tiles, next_epoch(w), half, ++w->seq, t->sampling, T->v, T->count,
                       O ? O->v : T->v, direction);
  else if (first_stage == 1 && run(1))  // resumed after a FRAGILE draw
    hipLaunchKernelGGL(k_compact_targets, dim3(tiles_for(batch)), dim3(CB), 0, s, st, batch,
                       w->cand, w->cflag, w->targets, w->tqh, w->tiles, next_epoch(w), half, 1,
                       ++w->seq);
  if (run(2)) {
    // the candidates' actions inside the search unless they are direction-biased
    // (then they depend on s_near: k_extend_prep after the search)
    NhPrep<ZT> prep{V, seed, w->ca, t->sampling, direction, 0, NhDraw{}, nullptr};
    const bool early = !t->sampling.action_flag;
    const bool launch = !searched && la && la->launch_next;
    if (launch) {
      // the next half's targets drawn beside this search (never direction-biased:
      // s_from / s_to unset) and O's snapshot for its look-ahead search
      if (!early || t->sampling.state_flag || !O || !std::is_same_v<ZT, float>)
        return GBP_E_INVALID_ARG;
      prep.dr = la_draw(w, half + 1, batch, *la);
      prep.dr.snap_src = O->count;
      prep.dr.snap_dst = &w->la->nv[(half + 1) & 1];
      prep.dr.go_dst = &w->la->go[(half + 1) & 1];
    }
    bool prepped = searched;
    int rc = GBP_OK;
    if (!searched)
      rc = nn_launch<ZT>(w, &st->n_targets, w->targets, nullptr, T, w->nn, cus, s, w->tqh,
                         early ? &prep : nullptr, w->cs, &prepped);
    if (!rc && launch) rc = la_launch(t, w, O, half + 1, batch, seed, *la, s);
    if (rc) return rc;
    const int64_t mmax = batch * GBP_NUM_GEN_STATES;
    if (!prepped)
      hipLaunchKernelGGL(k_extend_prep<ZT>, dim3(grid_for(mmax, TB, cus * 8)), dim3(TB), 0, s, V, st,
                         w->targets, w->nn, T->v, seed, w->cs, w->ca, ++w->seq, t->sampling,
                         direction);
    rc = gbp_internal_validate_dev_n(t, mmax, &st->n_validate, w->cs, w->ca, nullptr, direction,
                                     adaptive, nullptr, w->csn, nullptr, w->cf, w->cc, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_select, dim3(grid_for(batch, TB, cus * 4)), dim3(TB), 0, s, st, w->targets,
                       w->nn, T->v, w->ca, w->csn, w->cf, w->eres, w->echo, w->esn, w->ean, w->ef,
                       half, ++w->seq);
  }
  if (run(3))
    hipLaunchKernelGGL(k_append, dim3(tiles_for(batch)), dim3(CB), 0, s, st, 0, w->eres, w->nn,
                       w->esn, w->ean, T->v, T->vh, T->hm, T->a, T->g, T->parent, T->count, w->evtx,
                       w->tiles,
                       next_epoch(w), half, T->cap, ++w->seq, T->child, T->sibling, T->prev, w->star);
  if (th) HIPCHK_P(hipEventRecord(th->ev[1], s));
  const int kT = direction == GBP_FORWARD ? 0 : 1;  // T's tree index (Ta 0, Tb 1)
  gbp_plan_ws::StarSet &S = w->ss[half & 1];
  if (w->star && run(6)) {
    // RRT* insertion, stage 6: neighbourhoods, connect checks, their pair checks
    // one 1024-thread workgroup per CU at most (a half has ~100-200 items at
    // config 5; more are taken grid-stride): a grid of 8 per CU, nearly all
    // exiting at once, cost its dispatch
    unsigned gk = (unsigned)std::max<int64_t>(1, std::min<int64_t>(w->star_items, cus * GBP_STAR_GK));
    if (w->star_grid > 0) gk = std::min<unsigned>(gk, (unsigned)w->star_grid);
    hipLaunchKernelGGL(k_star_count, dim3(gk), dim3(RB), 0, s, st, T->v, w->star_delta, S.scnt,
                       S.sioff, S.soff, S.meta, w->star_max_pairs, S.sfin, w->star_items, w->star_ch,
                       half, ++w->seq);
    hipLaunchKernelGGL(k_star_fill, dim3(gk), dim3(RB), 0, s, st, T->v, w->star_delta, S.sioff,
                       S.snb, S.sown, w->star_items, w->star_ch, ++w->seq);
    if (th) HIPCHK_P(hipEventRecord(th->ev[6], s));
    const int64_t rmax = 2 * w->star_max_pairs;  // connect checks, one wave each
    const int cm = (t->opt_affine && t->affine) ? 2 : 0;
    unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cus * GBP_STAR_GC, (rmax + 3) / 4));
    if (w->star_grid > 0) g = std::min<unsigned>(g, (unsigned)w->star_grid);  // (tests: several checks a wave)
    const uint64_t cseq = ++w->seq;
#define GBP_SC(AD, CM)                                                                        \
  hipLaunchKernelGGL((k_star_check<ZT, AD, CM>), dim3(g), dim3(TB), 0, s, V, st, direction, T->v, \
                     S.snb, S.sown, S.srowof, S.srs, S.sra, S.srf, half, cseq)
    if (adaptive) {
      if (cm == 2) GBP_SC(true, 2); else GBP_SC(true, 0);
    } else {
      if (cm == 2) GBP_SC(false, 2); else GBP_SC(false, 0);
    }
#undef GBP_SC
    if (th) HIPCHK_P(hipEventRecord(th->ev[7], s));
    if (th) HIPCHK_P(hipEventRecord(th->ev[2], s));
  }
  if (w->star && run(7)) {
    // stage 7, the ordered replay, on star_stream: it changes T's parents, g
    // and successor lists only, which nothing reads before half h + 1's
    // stage 5 (its appends into T wait for it: rdone[kT]); the connects of
    // this half and the next half's extends of O run beside it
    HIPCHK_P(hipEventRecord(w->star_e6, s));
    HIPCHK_P(hipStreamWaitEvent(w->star_stream, w->star_e6, 0));
    if (th) HIPCHK_P(hipEventRecord(th->ev[3], w->star_stream));
    StarLds lds;
    if (w->star_lds[0] >= 0) {
      lds.rp = w->star_lds[0];
      lds.rk = w->star_lds[1];
      lds.rq = w->star_lds[2];
    }
    hipLaunchKernelGGL(k_star_replay, dim3(1), dim3(RW), 0, w->star_stream, st, T->v, T->a, T->g,
                       T->parent, T->child, T->sibling, T->prev, S.soff, S.snb, S.sown, S.srowof,
                       S.sra, S.srf, S.meta, T->bfs, T->bfs + T->cap, T->count, lds, ++w->seq);
    HIPCHK_P(hipEventRecord(w->star_rdone[kT], w->star_stream));
  }
  if (!O) return hipGetLastError() == hipSuccess ? GBP_OK : GBP_E_HIP;
  const int cdir = direction == GBP_FORWARD ? GBP_REVERSE : GBP_FORWARD;
  if (run(4)) {
    // queries: T's new vertices, rows [added_base, added_base + n_added)
    int rc = nn_launch<float>(w, &st->n_added, T->v, &st->added_base, O, w->nno, cus, s, T->vh, nullptr,
                       nullptr, nullptr, nullptr, true, true);
    if (rc) return rc;
    const int cm = (t->opt_affine && t->affine) ? 2 : 0;
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>(cus * GBP_CONNECT_GC, (batch + 3) / 4));
    const uint64_t kseq = ++w->seq;
#define GBP_KC(AD, CM)                                                                         \
  hipLaunchKernelGGL((k_connect<ZT, AD, CM>), dim3(g), dim3(TB), 0, s, V, st, cdir, T->v, O->v, \
                     w->nno, w->kres, w->ksn, w->kan, w->kf, half, kseq)
    if (adaptive) {
      if (cm == 2) GBP_KC(true, 2); else GBP_KC(true, 0);
    } else {
      if (cm == 2) GBP_KC(false, 2); else GBP_KC(false, 0);
    }
#undef GBP_KC
  }
  if (run(5)) {
    // O's last replay (half h - 1's, on star_stream) before appending into O
    if (w->star) HIPCHK_P(hipStreamWaitEvent(s, w->star_rdone[1 - kT], 0));
    const bool t_is_a = direction == GBP_FORWARD;
    StarShared ssh;
    if (w->star) {  // the REACHED connections kept, listed by the append itself
      ssh.list = w->sshared;
      ssh.max_shared = w->star_max_shared;
      ssh.meta = S.meta;
      ssh.tiles2 = w->tiles + tiles_for(batch);
      ssh.tot2 = (int32_t *)(S.sfin + 8);
      ssh.t_is_a = t_is_a ? 1 : 0;
    }
    const uint32_t ep1 = next_epoch(w);
    if (w->star) ssh.epoch2 = next_epoch(w);
    hipLaunchKernelGGL(k_append, dim3(tiles_for(batch)), dim3(CB), 0, s, st, 1, w->kres, w->nno,
                       w->ksn, w->kan, O->v, O->vh, O->hm, O->a, O->g, O->parent, O->count,
                       w->star ? w->kvtx : nullptr, w->tiles, ep1, half, O->cap, ++w->seq,
                       O->child, O->sibling, O->prev, w->star, ssh);
    if (w->star) {  // after Tb's half the best connection ranked
      if (half & 1) {
        // on star_stream behind this half's replay (Tb's g final) and half h - 1's
        // (Ta's); the next replay of Ta queues behind it, and half h + 1's
        // appends into Tb wait for it (rdone[kT] moves past it)
        HIPCHK_P(hipEventRecord(w->star_e5, s));
        HIPCHK_P(hipStreamWaitEvent(w->star_stream, w->star_e5, 0));
        hipLaunchKernelGGL(k_star_rank, dim3(1), dim3(RB), 0, w->star_stream, st, w->sshared, S.meta,
                           t_is_a ? T->g : O->g, t_is_a ? O->g : T->g, ++w->seq);
        HIPCHK_P(hipEventRecord(w->star_rdone[kT], w->star_stream));
      }
    }
  }
  if (th) {
    if (th->star) HIPCHK_P(hipEventRecord(th->ev[4], w->star_stream));
    HIPCHK_P(hipEventRecord(th->ev[5], s));
    th->pending = true;
  }
  return hipGetLastError() == hipSuccess ? GBP_OK : GBP_E_HIP;
}

}  // namespace

// ============================================================================
// C ABI (include/gbp.h "device trees and the device planner loop")
// ============================================================================
namespace {

struct Guard {
  int prev = -1;
  explicit Guard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~Guard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class T>
T *carve(char *&p, size_t count) {
  p = (char *)(((uintptr_t)p + 255) & ~(uintptr_t)255);
  T *r = (T *)p;
  p += count * sizeof(T);
  return r;
}

int tree_alloc(gbp_tree *t, int64_t cap) {
  double *v = nullptr, *a = nullptr, *g = nullptr;
  _Float16 *vh = nullptr;
  int32_t *p = nullptr, *ch = nullptr;
  if (hipMalloc(&v, 64 * cap) != hipSuccess) return GBP_E_ALLOC;
  if (hipMalloc(&a, 80 * cap) != hipSuccess || hipMalloc(&g, 8 * cap) != hipSuccess ||
      hipMalloc(&p, 4 * cap) != hipSuccess || hipMalloc(&ch, 20 * cap) != hipSuccess ||
      hipMalloc(&vh, 2 * NH_ROW * ((cap + 63) & ~(int64_t)63)) != hipSuccess) {
    (void)hipFree(v);
    if (a) (void)hipFree(a);
    if (g) (void)hipFree(g);
    if (p) (void)hipFree(p);
    if (ch) (void)hipFree(ch);
    return GBP_E_ALLOC;
  }
  t->v = v;
  t->vh = vh;
  t->a = a;
  t->g = g;
  t->parent = p;
  t->child = ch;  // [cap] first children, [cap] next / [cap] previous siblings, [2 cap] queues
  t->sibling = ch + cap;
  t->prev = ch + 2 * cap;
  t->bfs = ch + 3 * cap;
  t->cap = cap;
  return GBP_OK;
}

template <class T>
int d2h(T *dst, const T *src, size_t count, hipStream_t s) {
  HIPCHK_P(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyDeviceToHost, s));
  return GBP_OK;
}
template <class T>
int h2d(T *dst, const T *src, size_t count, hipStream_t s) {
  HIPCHK_P(hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, s));
  return GBP_OK;
}

}  // namespace

extern "C" {

int gbp_stream_create(int device, gbp_stream *out) {
  if (!out) return GBP_E_INVALID_ARG;
  Guard g(device);
  hipStream_t s = nullptr;
  HIPCHK_P(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *out = (gbp_stream)s;
  return GBP_OK;
}

int gbp_stream_destroy(gbp_stream stream) {
  if (stream) HIPCHK_P(hipStreamDestroy((hipStream_t)stream));
  return GBP_OK;
}

int gbp_tree_create(int device, int64_t capacity, gbp_tree **out) {
  if (!out || capacity < 1 || capacity > 0x7FFFFFFF) return GBP_E_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GBP_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return GBP_E_INVALID_ARG;
  Guard g(device);
  gbp_tree *t = new (std::nothrow) gbp_tree();
  if (!t) return GBP_E_ALLOC;
  t->device = device;
  if (hipMalloc(&t->count, 4) != hipSuccess || hipMalloc(&t->hm, 64) != hipSuccess ||
      tree_alloc(t, capacity) != GBP_OK) {
    gbp_tree_destroy(t);
    return GBP_E_ALLOC;
  }
  // the zeroing runs on the null stream, and the caller's planner streams are
  // non-blocking (gbp_stream_create): it must be complete before this returns,
  // or it can land after gbp_tree_init's count = 1 on another stream (seen as
  // a root overwritten by the first append under two processes per GPU)
  if (hipMemset(t->count, 0, 4) != hipSuccess || hipMemset(t->hm, 0, 64) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    gbp_tree_destroy(t);
    return GBP_E_HIP;
  }
  *out = t;
  return GBP_OK;
}

int gbp_tree_destroy(gbp_tree *t) {
  if (!t) return GBP_E_BAD_HANDLE;
  Guard g(t->device);
  (void)hipDeviceSynchronize();
  void *ptrs[] = {t->v, t->vh, t->hm, t->a, t->g, t->parent, t->child, t->count};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  delete t;
  return GBP_OK;
}

int gbp_tree_reserve(gbp_tree *t, int64_t capacity, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (capacity <= t->cap) return GBP_OK;
  if (capacity > 0x7FFFFFFF) return GBP_E_SHAPE;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  HIPCHK_P(hipStreamSynchronize(s));
  gbp_tree old = *t;
  int rc = tree_alloc(t, capacity);
  if (rc) {
    *t = old;
    return rc;
  }
  HIPCHK_P(hipMemcpyAsync(t->v, old.v, 64 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->vh, old.vh, 2 * NH_ROW * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->a, old.a, 80 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->g, old.g, 8 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->parent, old.parent, 4 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->child, old.child, 4 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->sibling, old.sibling, 4 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipMemcpyAsync(t->prev, old.prev, 4 * old.cap, hipMemcpyDeviceToDevice, s));
  HIPCHK_P(hipStreamSynchronize(s));
  (void)hipFree(old.v);
  (void)hipFree(old.vh);
  (void)hipFree(old.a);
  (void)hipFree(old.g);
  (void)hipFree(old.parent);
  (void)hipFree(old.child);
  return GBP_OK;
}

int gbp_tree_init(gbp_tree *t, const double *root, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (!root) return GBP_E_INVALID_ARG;
  Guard g(t->device);
  hipLaunchKernelGGL(k_tree_init, dim3(1), dim3(1), 0, (hipStream_t)stream, *t, root[0], root[1],
                     root[2], root[3], root[4], root[5], root[6], root[7]);
  HIPCHK_P(hipGetLastError());
  return GBP_OK;
}

int gbp_tree_size(gbp_tree *t, int64_t *count, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (!count) return GBP_E_INVALID_ARG;
  Guard g(t->device);
  int32_t c = 0;
  HIPCHK_P(hipMemcpyAsync(&c, t->count, 4, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK_P(hipStreamSynchronize((hipStream_t)stream));
  *count = c;
  return GBP_OK;
}

int gbp_tree_capacity(gbp_tree *t, int64_t *capacity) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (!capacity) return GBP_E_INVALID_ARG;
  *capacity = t->cap;
  return GBP_OK;
}

int gbp_tree_read(gbp_tree *t, int64_t first, int64_t n, double *states, double *actions,
                  int32_t *parents, double *g, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (first < 0 || n < 0 || first + n > t->cap) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  Guard gd(t->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = GBP_OK;
  if (!rc && states) rc = d2h(states, t->v + 8 * first, 8 * n, s);
  if (!rc && actions) rc = d2h(actions, t->a + 10 * first, 10 * n, s);
  if (!rc && parents) rc = d2h(parents, t->parent + first, n, s);
  if (!rc && g) rc = d2h(g, t->g + first, n, s);
  if (rc) return rc;
  HIPCHK_P(hipStreamSynchronize(s));
  return GBP_OK;
}

int gbp_tree_append_host(gbp_tree *t, int64_t n, const double *states, const double *actions,
                         const int32_t *parents, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!states || !actions || !parents))) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  int64_t c = 0;
  int rc = gbp_tree_size(t, &c, stream);
  if (rc) return rc;
  for (int64_t i = 0; i < n; i++)
    if (parents[i] < -1 || parents[i] >= c + i) return GBP_E_INVALID_ARG;
  if (c + n > t->cap) rc = gbp_tree_reserve(t, std::max<int64_t>(2 * t->cap, c + n), stream);
  if (rc) return rc;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  void *buf = nullptr;
  HIPCHK_P(hipMalloc(&buf, (size_t)n * (64 + 80 + 4) + 512));
  char *p = (char *)buf;
  double *ds = carve<double>(p, 8 * n), *da = carve<double>(p, 10 * n);
  int32_t *dp = carve<int32_t>(p, n);
  rc = h2d(ds, states, 8 * n, s);
  if (!rc) rc = h2d(da, actions, 10 * n, s);
  if (!rc) rc = h2d(dp, parents, n, s);
  if (!rc) {
    hipLaunchKernelGGL(k_tree_append, dim3(1), dim3(1), 0, s, *t, n, ds, da, dp);
    if (hipGetLastError() != hipSuccess) rc = GBP_E_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_tree_load_host(gbp_tree *t, int64_t n, const double *states, const double *actions,
                       const int32_t *parents, gbp_stream stream) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (n < 1 || n > 0x7FFFFFFE || !states || !actions || !parents || parents[0] != -1)
    return GBP_E_INVALID_ARG;
  // one tree rooted at 0: every parent in range, every vertex reached from the root
  {
    std::vector<int32_t> head(n, -1), next(n, -1), queue;
    for (int64_t i = 1; i < n; i++) {
      if (parents[i] < 0 || parents[i] >= n || parents[i] == i) return GBP_E_INVALID_ARG;
      next[i] = head[parents[i]];
      head[parents[i]] = (int32_t)i;
    }
    queue.reserve(n);
    queue.push_back(0);
    for (size_t h = 0; h < queue.size() && (int64_t)queue.size() <= n; h++)
      for (int32_t c = head[queue[h]]; c >= 0; c = next[c]) queue.push_back(c);
    if ((int64_t)queue.size() != n) return GBP_E_INVALID_ARG;
  }
  int rc = GBP_OK;
  if (n > t->cap) rc = gbp_tree_reserve(t, n, stream);
  if (rc) return rc;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  void *buf = nullptr;
  HIPCHK_P(hipMalloc(&buf, (size_t)n * (64 + 80 + 4) + 512));
  char *p = (char *)buf;
  double *ds = carve<double>(p, 8 * n), *da = carve<double>(p, 10 * n);
  int32_t *dp = carve<int32_t>(p, n);
  rc = h2d(ds, states, 8 * n, s);
  if (!rc) rc = h2d(da, actions, 10 * n, s);
  if (!rc) rc = h2d(dp, parents, n, s);
  if (!rc) {
    hipLaunchKernelGGL(k_tree_load, dim3(1), dim3(1), 0, s, *t, n, ds, da, dp);
    if (hipGetLastError() != hipSuccess) rc = GBP_E_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_tree_device_ptrs(gbp_tree *t, double **states, int32_t **count) {
  if (!tree_ok(t)) return GBP_E_BAD_HANDLE;
  if (states) *states = t->v;
  if (count) *count = t->count;
  return GBP_OK;
}

// the look-ahead stream: its search launches would otherwise hold every CU's
// registers for their whole duration (3 waves per SIMD at 162 VGPRs), and the
// caller's stream's short latency-bound launches (select, appends, the
// connects' search) would wait for them; the stream is masked to all XCDs
// but the last (CUs [0, 7/8 n)), which keeps one XCD for those.  Measured on
// the planner (config-3 pair, 4-s runs): 170 M extends/s unmasked, 180 M with
// 224 of 256 CUs, 176 M with 208 or 240; spreading the excluded CUs over the
// XCDs instead was slower (profiles/r05h_la_knobs*.txt).  GBP_LA_CUS
// overrides the count (0 or >= n: unmasked, lowest priority).  One stream per
// device for the process (creating a masked queue takes milliseconds: a
// planner's time to first solution must not pay it; gbp_terrain_create
// creates it ahead), shared by the device's workspaces.
extern "C++" __attribute__((visibility("hidden"))) hipStream_t gbp_internal_la_stream(int device,
                                                                             int num_cus) {
  static std::mutex mu;
  static std::map<int, hipStream_t> streams;
  std::lock_guard<std::mutex> lk(mu);
  auto it = streams.find(device);
  if (it != streams.end()) return it->second;
  int prev = -1;
  if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  if (prev != device && hipSetDevice(device) != hipSuccess) return nullptr;
  const char *env = getenv("GBP_LA_CUS");
  // the last XCD's CUs left out (from the device's XCC count, not
  // an assumed 8; one XCC or an unknown count: unmasked)
  int xcc = 0;
  if (hipDeviceGetAttribute(&xcc, hipDeviceAttributeNumberOfXccs, device) != hipSuccess) xcc = 0;
  const int n = num_cus, cus = env && *env ? atoi(env) : (xcc >= 2 ? n - n / xcc : n);
  hipStream_t st = nullptr;
  hipError_t e;
  if (cus > 0 && cus < n) {
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (int c = 0; c < cus; c++) mask[c / 32] |= 1u << (c % 32);
    e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
  } else {
    int lo = 0, hi = 0;
    e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&st, hipStreamNonBlocking, lo);
  }
  if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
  if (e != hipSuccess) return nullptr;
  if (streams.empty()) {
    // destroyed before the HIP runtime's own exit handlers run (registered
    // earlier, so they run later): a profiler's teardown walking the
    // process's queues at exit found this one still alive and faulted
    std::atexit([] {
      for (auto &kv : streams) (void)hipStreamDestroy(kv.second);
      streams.clear();
    });
  }
  streams[device] = st;
  return st;
}

static void ws_free(gbp_plan_ws *w) {
  if (w->ntring) {
    (void)hipDeviceSynchronize();
    for (size_t i = 0; i < w->ntring; i++)
      for (auto &e : w->tring[i].ev)
        if (e) (void)hipEventDestroy(e);
    delete[] w->tring;
  }
  if (w->la_go) (void)hipEventDestroy(w->la_go);
  if (w->la_done) (void)hipEventDestroy(w->la_done);
  if (w->star_stream) {
    (void)hipStreamSynchronize(w->star_stream);
    hipEvent_t ev[] = {w->star_e6, w->star_e5, w->star_rdone[0], w->star_rdone[1], w->star_sdone};
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(w->star_stream);
  }
  if (w->block) (void)hipFree(w->block);
  if (w->star_block) (void)hipFree(w->star_block);
  delete w;
}

int gbp_plan_ws_create(gbp_terrain *t, int64_t max_batch, gbp_plan_ws **out) {
  if (!t || !out) return GBP_E_INVALID_ARG;
  if (max_batch < 1 || max_batch > (1 << 24)) return GBP_E_INVALID_ARG;
  *out = nullptr;
  Guard g(t->device);
  gbp_plan_ws *w = new (std::nothrow) gbp_plan_ws();
  if (!w) return GBP_E_ALLOC;
  w->device = t->device;
  w->num_cus = t->num_cus;
  w->nn_stats = t->opt_nn_stats;
  w->bmax = max_batch;
  // 4096 items: 3072 (the waves resident at 162 VGPRs), 2048 and 6144 measured
  // slower in the planner (profiles/r04l_nn_items.txt)
  w->nn_items = NH_ITEMS;
  {
    const char *e = getenv("GBP_NN_ITEMS");  // (A/B sweeps; whole workgroups of NH_TB / WAVE waves)
    if (e && *e) w->nn_items = std::max(NH_TB / WAVE, std::min(1 << 16, atoi(e))) & ~(NH_TB / WAVE - 1);
  }
  w->ntiles = (max_batch + TB - 1) / TB + 1;  // k_targets' 256-draw tiles (k_compact_targets: 1024)
  const int64_t b = max_batch, m = GBP_NUM_GEN_STATES * max_batch;
  // k_nn_small's partials: NS_MAXQ queries per workgroup, or a whole batch
  // when that stays within 2^22 slots (~48 MB; bench's planner: 92,749 x 32)
  w->ns_grid = std::max(1, std::min(NS_BLOCKS, t->num_cus / 8));
  {
    const char *e = getenv("GBP_NS_GRID");  // (A/B sweeps)
    if (e && *e) w->ns_grid = std::max(1, std::min(1024, atoi(e)));
  }
  w->ns_capq = (int64_t)w->ns_grid * b <= ((int64_t)1 << 22) ? std::max<int64_t>(b, NS_MAXQ) : NS_MAXQ;
  const size_t nsbytes = (size_t)w->ns_grid * w->ns_capq * 12 + 512;
  const size_t bytes = nsbytes + sizeof(gbp_plan_status) + 16 * w->ntiles + 3 * (64 * b + 4 * b + 64 * b + 64 * b) +
                       1024 + m * (2 * 64 + 2 * 80 + 64 + 4 + 4) + b * (2 * 4 + 4 + 64 + 80 + 4 + 4) +
                       b * (4 + 4 + 64 + 80 + 4) + 2 * NN_MAX_CHUNKS * b * (16 + 16) + 64 * b + 512 +
                       64 * 256 + 0 /* ns partials: below */ + 1024 +
                       2 * ((size_t)NSC_CAP * 8 + (size_t)NSC_UNITS * 12 + 32 * b + 1024);
  if (hipMalloc(&w->block, bytes) != hipSuccess) {
    delete w;
    return GBP_E_ALLOC;
  }
  char *p = (char *)w->block;
  w->st = carve<gbp_plan_status>(p, 1);
  w->la = carve<gbp_plan_la>(p, 1);
  w->tiles = carve<unsigned long long>(p, w->ntiles);
  w->la_tiles = carve<unsigned long long>(p, w->ntiles);
  for (auto &ts : w->tset) {
    ts.cand = carve<double>(p, 8 * b);
    ts.cflag = carve<uint32_t>(p, b);
    ts.targets = carve<double>(p, 8 * b);
    ts.tqh = carve<_Float16>(p, 32 * b);
  }
  for (int k = 0; k < 2; k++) {
    w->nnp[k] = carve<int32_t>(p, b);
    w->csp[k] = carve<double>(p, 8 * m);
    w->cap[k] = carve<double>(p, 10 * m);
  }
  select_targets(w, 0);
  w->csn = carve<double>(p, 8 * m);
  w->cf = carve<uint32_t>(p, m);
  w->cc = carve<uint32_t>(p, m);
  w->eres = carve<int32_t>(p, b);
  w->echo = carve<int32_t>(p, b);
  w->esn = carve<double>(p, 8 * b);
  w->ean = carve<double>(p, 10 * b);
  w->ef = carve<uint32_t>(p, b);
  w->evtx = carve<int32_t>(p, b);
  w->nno = carve<int32_t>(p, b);
  w->kres = carve<int32_t>(p, b);
  w->ksn = carve<double>(p, 8 * b);
  w->kan = carve<double>(p, 10 * b);
  w->kf = carve<uint32_t>(p, b);
  w->nn_d = carve<double>(p, 2 * NN_MAX_CHUNKS * b);   // k_nn_mfma: float4 per slot
  w->nn_i = carve<int32_t>(p, 4 * NN_MAX_CHUNKS * b);  // k_nn_mfma: int4 per slot
  w->nn_d2 = carve<double>(p, 2 * NN_MAX_CHUNKS * b);
  w->nn_i2 = carve<int32_t>(p, 4 * NN_MAX_CHUNKS * b);
  w->ns_d = carve<double>(p, (int64_t)w->ns_grid * w->ns_capq);
  w->ns_i = carve<int32_t>(p, (int64_t)w->ns_grid * w->ns_capq);
  w->ns_fin = carve<uint32_t>(p, 64);
  for (auto &sb : w->nsb) {
    const char *cenv = getenv("GBP_NSC_CAP");  // (a small list: the fallback's test)
    sb.cap = (uint32_t)std::max(1, std::min(NSC_CAP, cenv && *cenv ? atoi(cenv) : NSC_CAP));
    sb.list = carve<int2>(p, NSC_CAP);
    sb.ed = carve<double>(p, NSC_UNITS);
    sb.ei = carve<int32_t>(p, NSC_UNITS);
    sb.cnt = carve<uint32_t>(p, 64);
    sb.hd = carve<double>(p, b);
    sb.hi = carve<int32_t>(p, b);
    sb.qh = carve<int2>(p, b);
  }
  bool ok = (size_t)(p - (char *)w->block) <= bytes &&
            hipMemset(w->ns_fin, 0, 4 * 64) == hipSuccess &&
            hipMemset(w->nsb[0].cnt, 0, 4 * 64) == hipSuccess &&
            hipMemset(w->nsb[1].cnt, 0, 4 * 64) == hipSuccess &&
            hipMemset(w->tiles, 0, 8 * w->ntiles) == hipSuccess &&
            hipMemset(w->la_tiles, 0, 8 * w->ntiles) == hipSuccess &&
            (w->la_stream = gbp_internal_la_stream(w->device, w->num_cus)) != nullptr &&
            hipEventCreateWithFlags(&w->la_go, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&w->la_done, hipEventDisableTiming) == hipSuccess;
  if (ok) {
    hipLaunchKernelGGL(k_plan_reset, dim3(1), dim3(1), 0, nullptr, w->st, (int64_t)0, w->la);
    ok = hipDeviceSynchronize() == hipSuccess;
  }
  if (!ok) {
    ws_free(w);
    return GBP_E_HIP;
  }
  *out = w;
  return GBP_OK;
}

int gbp_plan_ws_destroy(gbp_plan_ws *w) {
  if (!w) return GBP_E_BAD_HANDLE;
  Guard g(w->device);
  (void)hipDeviceSynchronize();
  ws_free(w);
  return GBP_OK;
}

int gbp_plan_star_config(gbp_plan_ws *w, int enable, double delta, int64_t max_pairs,
                         int64_t max_shared) {
  if (!w) return GBP_E_BAD_HANDLE;
  if (!enable) {
    w->star = 0;
    return GBP_OK;
  }
  if (!(delta >= 0) || max_pairs < 1 || max_pairs > (1 << 28) || max_shared < 1 ||
      max_shared > (1 << 28))
    return GBP_E_INVALID_ARG;
  Guard g(w->device);
  {
    const char *pe = getenv("GBP_STAR_PAIRS");  // (tests: a small first size, grown by the halts)
    if (pe && *pe && !w->star_block) max_pairs = std::max<int64_t>(1, std::min<int64_t>(max_pairs, atoll(pe)));
  }
  // a larger block keeps the run's list of kept connections (the ranking
  // after Tb's halves reads all of it); the per-half sets are rebuilt by the
  // half that resumes (GBP_PLAN_HALT_STAR_PAIRS)
  std::vector<int32_t> keep_shared;
  if (w->star_block && (max_pairs > w->star_max_pairs || max_shared > w->star_max_shared)) {
    (void)hipDeviceSynchronize();
    max_pairs = std::max(max_pairs, w->star_max_pairs);
    max_shared = std::max(max_shared, w->star_max_shared);
    keep_shared.resize(2 * (size_t)w->star_max_shared);
    if (hipMemcpy(keep_shared.data(), w->sshared, 8 * (size_t)w->star_max_shared,
                  hipMemcpyDeviceToHost) != hipSuccess)
      return GBP_E_HIP;
    (void)hipFree(w->star_block);
    w->star_block = nullptr;
  }
  if (!w->star_block) {
    const int64_t b = w->bmax, r = 2 * max_pairs;
    int64_t items = std::max<int64_t>(4 * b, 1 << 15);
    // (tests: GBP_STAR_ITEMS, at least the batch, and GBP_STAR_CH small grow
    // the chunks; GBP_STAR_GRID below makes every count / fill workgroup take
    // several items)
    const char *ie = getenv("GBP_STAR_ITEMS");
    if (ie && *ie) items = std::max<int64_t>(b, atoll(ie));
    const char *le = getenv("GBP_STAR_LDS");
    if (le && *le) {
      int a = RP, b2 = RK, c = RQ;
      if (sscanf(le, "%d,%d,%d", &a, &b2, &c) == 3) {
        w->star_lds[0] = std::max(0, std::min(a, RP));
        w->star_lds[1] = std::max(0, std::min(b2, RK));
        w->star_lds[2] = std::max(1, std::min(c, RQ));
      }
    }
    const char *ce = getenv("GBP_STAR_CH");
    w->star_ch = ce && *ce ? std::max<int64_t>(1, atoll(ce)) : STAR_CH;
    const size_t bytes = 2 * (12 * items + 4 * (b + 1) + 8 * max_pairs + r * (4 + 4 + 64 + 80 + 4) +
                              32 + 12 * 256) +
                         4 * b + 8 * max_shared + 4 * 256;
    if (hipMalloc(&w->star_block, bytes) != hipSuccess) {
      w->star_block = nullptr;
      w->star = 0;
      return GBP_E_ALLOC;
    }
    char *p = (char *)w->star_block;
    for (auto &S : w->ss) {
      S.scnt = carve<unsigned long long>(p, items);
      S.sioff = carve<int32_t>(p, items);
      S.soff = carve<int32_t>(p, b + 1);
      S.snb = carve<int32_t>(p, max_pairs);
      S.sown = carve<int32_t>(p, max_pairs);
      S.srowof = carve<int32_t>(p, r);
      S.srs = carve<double>(p, 8 * r);
      S.sra = carve<double>(p, 10 * r);
      S.srf = carve<uint32_t>(p, r);
      S.meta = carve<int64_t>(p, 4);
      S.sfin = carve<uint32_t>(p, 64);
    }
    w->star_items = items;
    const char *ge = getenv("GBP_STAR_GRID");
    w->star_grid = ge && *ge ? std::max(1, atoi(ge)) : 0;
    w->kvtx = carve<int32_t>(p, b);
    w->sshared = carve<int32_t>(p, 2 * max_shared);
    if ((size_t)(p - (char *)w->star_block) > bytes) return GBP_E_HIP;
    for (auto &S : w->ss)  // (epoch 0 is never a launch's: seq starts at 1)
      if (hipMemset(S.sfin, 0, 4 * 64) != hipSuccess ||
          hipMemset(S.scnt, 0, 8 * (size_t)items) != hipSuccess)
        return GBP_E_HIP;
    if (!keep_shared.empty() &&
        hipMemcpy(w->sshared, keep_shared.data(), 4 * keep_shared.size(), hipMemcpyHostToDevice) != hipSuccess)
      return GBP_E_HIP;
    w->star_max_pairs = max_pairs;
    w->star_max_shared = max_shared;
  }
  if (!w->star_stream) {
    // the workspace's own (a device-wide stream would make one planner's joins
    // wait for another's replays), CU-masked to the last n/8 CUs, the ones
    // la_stream leaves free: a masked stream has a hardware queue of its own,
    // while a plain one shares one of the process's GPU_MAX_HW_QUEUES (4)
    // round-robin — with the caller's stream the replay then ran in line with
    // the connects it should overlap (config 5: 52 vs 66 M pair checks/s with
    // 8 queues)
    int xcc = 0;
    if (hipDeviceGetAttribute(&xcc, hipDeviceAttributeNumberOfXccs, w->device) != hipSuccess) xcc = 0;
    const int n = w->num_cus, lo = xcc >= 2 ? n - n / xcc : n;
    std::vector<uint32_t> mask((n + 31) / 32, 0u);
    for (int c = lo; c < n; c++) mask[c / 32] |= 1u << (c % 32);
    const hipError_t e = (lo > 0 && lo < n)
                             ? hipExtStreamCreateWithCUMask(&w->star_stream, (uint32_t)mask.size(),
                                                            mask.data())
                             : hipStreamCreateWithFlags(&w->star_stream, hipStreamNonBlocking);
    if (e != hipSuccess ||
        hipEventCreateWithFlags(&w->star_e6, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->star_e5, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->star_rdone[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->star_rdone[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&w->star_sdone, hipEventDisableTiming) != hipSuccess) {
      w->star = 0;
      return GBP_E_HIP;
    }
  }
  w->star = 1;
  w->star_delta = delta;
  return GBP_OK;
}

int gbp_plan_stage_timing(gbp_plan_ws *w, int enable) {
  if (!w) return GBP_E_BAD_HANDLE;
  Guard g(w->device);
  if (enable && !w->ntring) {
    w->tring = new (std::nothrow) gbp_plan_ws::TimedHalf[256];
    if (!w->tring) return GBP_E_ALLOC;
    w->ntring = 256;
    for (size_t i = 0; i < w->ntring; i++)
      for (auto &e : w->tring[i].ev)
        if (hipEventCreate(&e) != hipSuccess) return GBP_E_HIP;
  }
  w->timing = enable != 0;
  return GBP_OK;
}

int gbp_plan_stage_times(gbp_plan_ws *w, double *us, int n, int64_t *halves, int reset) {
  if (!w) return GBP_E_BAD_HANDLE;
  if (!us || n < 5) return GBP_E_INVALID_ARG;
  Guard g(w->device);
  timing_collect(w, false);
  for (int k = 0; k < std::min(n, 7); k++) us[k] = w->tsum[k];
  if (halves) *halves = w->tcount;
  if (reset) {
    for (double &x : w->tsum) x = 0;
    w->tcount = 0;
  }
  return GBP_OK;
}

int gbp_plan_reset(gbp_plan_ws *w, int64_t extend_counter, gbp_stream stream) {
  if (!w) return GBP_E_BAD_HANDLE;
  Guard g(w->device);
  hipLaunchKernelGGL(k_plan_reset, dim3(1), dim3(1), 0, (hipStream_t)stream, w->st, extend_counter,
                     w->la);
  HIPCHK_P(hipGetLastError());
  return GBP_OK;
}

int gbp_plan_status_read(gbp_plan_ws *w, gbp_plan_status *out, gbp_stream stream) {
  if (!w) return GBP_E_BAD_HANDLE;
  if (!out) return GBP_E_INVALID_ARG;
  Guard g(w->device);
  HIPCHK_P(hipMemcpyAsync(out, w->st, sizeof *out, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK_P(hipStreamSynchronize((hipStream_t)stream));
  return GBP_OK;
}

int gbp_plan_half_dev(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, gbp_tree *O, int32_t half,
                      int direction, int64_t batch, uint64_t seed, uint64_t target_stream,
                      int64_t target_index_base, int adaptive, int first_stage,
                      gbp_stream stream) {
  if (!t || !w || !tree_ok(T) || !tree_ok(O)) return GBP_E_BAD_HANDLE;
  if (batch < 1 || batch > w->bmax || first_stage < 0 || first_stage > (w->star ? 7 : 5) ||
      (direction != GBP_FORWARD && direction != GBP_REVERSE) || T == O)
    return GBP_E_INVALID_ARG;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  const int rc = t->storage == GBP_STORAGE_F32
                     ? enqueue_stages<float>(t, w, T, O, half, direction, batch, seed, target_stream,
                                             target_index_base, adaptive, first_stage, 5, s)
                     : enqueue_stages<double>(t, w, T, O, half, direction, batch, seed,
                                              target_stream, target_index_base, adaptive,
                                              first_stage, 5, s);
  if (w->star) {  // the replay and ranking on star_stream end before the caller's stream goes on
    HIPCHK_P(hipEventRecord(w->star_sdone, w->star_stream));
    HIPCHK_P(hipStreamWaitEvent(s, w->star_sdone, 0));
  }
  return rc;
}

int gbp_plan_halves_dev(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *Ta, gbp_tree *Tb,
                        int32_t first_half, int32_t n_halves, int64_t batch, uint64_t seed,
                        uint64_t stream_a, uint64_t stream_b, int adaptive, int first_stage,
                        gbp_stream stream) {
  if (!t || !w || !tree_ok(Ta) || !tree_ok(Tb)) return GBP_E_BAD_HANDLE;
  if (batch < 1 || batch > w->bmax || first_stage < 0 || first_stage > (w->star ? 7 : 5) ||
      n_halves < 0 || first_half < 0 || Ta == Tb)
    return GBP_E_INVALID_ARG;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  // the look-ahead search (LaHalf, la_launch): half h+1's draws do not depend
  // on the trees unless the sampling is direction-biased, and its search
  // needs only O as it stands before half h's connects, so both run on
  // la_stream beside half h; half h+1 starts with k_la_commit
  static const bool la_off = [] {  // GBP_LA_OFF=1: the inline sequence (A/B, diagnostics)
    const char *e = getenv("GBP_LA_OFF");
    return e && *e && *e != '0';
  }();
  // (RRT* too: its insertion rewires the extended tree's parents and g, not
  // its vertices, and the connects still append to O after the snapshot)
  const bool ahead = !la_off && !t->sampling.state_flag && !t->sampling.action_flag &&
                     t->storage == GBP_STORAGE_F32;  // (k_nn_mfma<float> draws)
  bool searched = false, used = false;
  int rc = GBP_OK;
  if (first_stage != 0)  // a resume: the halted half and the gated ones after it ran nothing
    for (size_t i = 0; i < w->ntring; i++)
      if (w->tring[i].pending && w->tring[i].half >= first_half) w->tring[i].pending = false;
  for (int32_t i = 0; i < n_halves && !rc; i++) {
    const int32_t h = first_half + i;
    const int k = h & 1;
    gbp_tree *T = k ? Tb : Ta, *O = k ? Ta : Tb;
    const int dir = k ? GBP_REVERSE : GBP_FORWARD;
    const uint64_t ts = k ? stream_b : stream_a;
    const int64_t tb = (int64_t)(h >> 1) * batch;
    const int fs = i == 0 ? first_stage : 0;
    LaHalf L;
    L.searched = searched;
    L.launch_next = ahead && i + 1 < n_halves && (searched || fs <= 2);
    L.draw_after = ahead && i + 2 < n_halves;
    L.stream_a = stream_a;
    L.stream_b = stream_b;
    rc = t->storage == GBP_STORAGE_F32
             ? enqueue_stages<float>(t, w, T, O, h, dir, batch, seed, ts, tb, adaptive, fs, 5, s, &L)
             : enqueue_stages<double>(t, w, T, O, h, dir, batch, seed, ts, tb, adaptive, fs, 5, s, &L);
    searched = L.launch_next;
    used = used || L.launch_next;
  }
  // nothing of the call stays on la_stream or star_stream past the caller's
  // stream (a host that reads the status, reserves or destroys after this sees
  // it finished).  la_done already follows this call's last look-ahead launch
  // (re-recording it on the device-wide la_stream would also wait for other
  // workspaces' searches: ADVICE r05)
  if (used) HIPCHK_P(hipStreamWaitEvent(s, w->la_done, 0));
  if (w->star) {
    HIPCHK_P(hipEventRecord(w->star_sdone, w->star_stream));
    HIPCHK_P(hipStreamWaitEvent(s, w->star_sdone, 0));
  }
  return rc;
}

int gbp_extend_tree_dev(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, int64_t n,
                        const double *targets, const int32_t *n_dev, int direction, int adaptive,
                        uint64_t seed, int64_t extend_base, int32_t *result, int32_t *new_vertex,
                        gbp_stream stream) {
  if (!t || !w || !tree_ok(T)) return GBP_E_BAD_HANDLE;
  if (n < 0 || n > w->bmax || (n > 0 && !targets) ||
      (direction != GBP_FORWARD && direction != GBP_REVERSE))
    return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  select_targets(w, 0);
  hipLaunchKernelGGL(k_extend_setup, dim3(grid_for(8 * n, TB, t->num_cus * 4)), dim3(TB), 0, s,
                     w->st, n, n_dev, extend_base, targets, w->targets, w->tqh);
  int rc = t->storage == GBP_STORAGE_F32
               ? enqueue_stages<float>(t, w, T, nullptr, 0, direction, n, seed, 0, 0, adaptive, 2,
                                       3, s)
               : enqueue_stages<double>(t, w, T, nullptr, 0, direction, n, seed, 0, 0, adaptive, 2,
                                        3, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_extend_out, dim3(grid_for(n, TB, t->num_cus * 4)), dim3(TB), 0, s, w->st, n,
                     w->eres, w->evtx, result, new_vertex);
  HIPCHK_P(hipGetLastError());
  return GBP_OK;
}

int gbp_extend_tree_finish_dev(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, int64_t n,
                               int direction, int32_t *result, int32_t *new_vertex,
                               gbp_stream stream) {
  if (!t || !w || !tree_ok(T)) return GBP_E_BAD_HANDLE;
  if (n < 0 || n > w->bmax) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  int rc = t->storage == GBP_STORAGE_F32
               ? enqueue_stages<float>(t, w, T, nullptr, 0, direction, n, 0, 0, 0, 0, 3, 3, s)
               : enqueue_stages<double>(t, w, T, nullptr, 0, direction, n, 0, 0, 0, 0, 3, 3, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_extend_out, dim3(grid_for(n, TB, t->num_cus * 4)), dim3(TB), 0, s, w->st, n,
                     w->eres, w->evtx, result, new_vertex);
  HIPCHK_P(hipGetLastError());
  return GBP_OK;
}

int gbp_extend_tree_host(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, int64_t n,
                         const double *targets, int direction, int adaptive, uint64_t seed,
                         int64_t extend_base, int32_t *result, int32_t *new_vertex,
                         int64_t *n_resolved) {
  if (!t || !w || !tree_ok(T)) return GBP_E_BAD_HANDLE;
  if (n < 0 || n > w->bmax || (n > 0 && (!targets || !result))) return GBP_E_INVALID_ARG;
  if (n_resolved) *n_resolved = 0;
  if (n == 0) return GBP_OK;
  Guard g(t->device);
  hipStream_t s = t->host_stream;
  int64_t cnt = 0;
  int rc = gbp_tree_size(T, &cnt, s);
  if (!rc && cnt + n > T->cap) rc = gbp_tree_reserve(T, std::max<int64_t>(2 * T->cap, cnt + n), s);
  if (rc) return rc;
  void *buf = nullptr;
  HIPCHK_P(hipMalloc(&buf, (size_t)n * (64 + 8) + 512));
  char *p = (char *)buf;
  double *dt = carve<double>(p, 8 * n);
  int32_t *dr = carve<int32_t>(p, n), *dv = carve<int32_t>(p, n);
  rc = h2d(dt, targets, 8 * n, s);
  if (!rc) rc = gbp_plan_reset(w, 0, s);
  if (!rc)
    rc = gbp_extend_tree_dev(t, w, T, n, dt, nullptr, direction, adaptive, seed, extend_base, dr,
                             dv, s);
  gbp_plan_status st;
  if (!rc) rc = gbp_plan_status_read(w, &st, s);
  if (!rc && st.halt) {
    int resume = -1;
    rc = gbp_plan_resolve_host(t, w, T, nullptr, direction, n, adaptive, &resume, n_resolved, s);
    if (!rc) rc = gbp_extend_tree_finish_dev(t, w, T, n, direction, dr, dv, s);
  }
  if (!rc) rc = d2h(result, dr, n, s);
  if (!rc && new_vertex) rc = d2h(new_vertex, dv, n, s);
  if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_tree_nearest_dev(gbp_plan_ws *w, gbp_tree *T, int64_t n, const double *queries,
                         int32_t *index, gbp_stream stream) {
  if (!w || !tree_ok(T)) return GBP_E_BAD_HANDLE;
  if (n < 0 || n > w->bmax || (n > 0 && (!queries || !index))) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  Guard g(w->device);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_set_queries, dim3(1), dim3(1), 0, s, w->st, (int32_t)n);
  return nn_launch<float>(w, &w->st->n_targets, queries, nullptr, T, index, w->num_cus, s, nullptr, nullptr,
                   nullptr, nullptr, nullptr, true);
}

int gbp_plan_resolve_host(gbp_terrain *t, gbp_plan_ws *w, gbp_tree *T, gbp_tree *O, int direction,
                          int64_t batch, int adaptive, int *resume_stage, int64_t *n_resolved,
                          gbp_stream stream) {
  if (!t || !w || !tree_ok(T)) return GBP_E_BAD_HANDLE;
  if (!resume_stage) return GBP_E_INVALID_ARG;
  Guard g(t->device);
  hipStream_t s = (hipStream_t)stream;
  gbp_plan_status st;
  int rc = gbp_plan_status_read(w, &st, stream);
  if (rc) return rc;
  *resume_stage = -1;
  int64_t k = 0;
  select_targets(w, st.halt_half >= 0 ? st.halt_half : 0);  // the halted half's target set
  if (st.halt & GBP_PLAN_HALT_STAR_PAIRS) {
    // nothing to re-decide: the caller has grown the insertion sets
    // (gbp_plan_star_config); the half redoes its stage 6
    if (2 * (int64_t)st.star_pairs > 2 * w->star_max_pairs) return GBP_E_SHAPE;
    *resume_stage = 6;
  } else if (st.halt & GBP_PLAN_HALT_TARGETS) {
    // isValidState(s_rand, STANCE) of the half's draws (rrt_connect.cpp:254)
    if (batch < 1 || batch > w->bmax) return GBP_E_INVALID_ARG;
    std::vector<uint32_t> fl(batch);
    if ((rc = d2h(fl.data(), w->cflag, batch, s))) return rc;
    HIPCHK_P(hipStreamSynchronize(s));
    for (int64_t i = 0; i < batch; i++) {
      if (!(fl[i] & GBP_F_FRAGILE)) continue;
      double q[8];
      if ((rc = d2h(q, w->cand + 8 * i, 8, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      gbp_host::Acc acc;
      const bool v = gbp_host::is_valid_state(t->host, q, GBP_STANCE, acc);
      fl[i] = acc.flags | (v ? GBP_F_VALID : 0u) | GBP_F_RESOLVED;
      if ((rc = h2d(w->cflag + i, &fl[i], 1, s))) return rc;
      k++;
    }
    *resume_stage = 1;
  } else if (st.halt & GBP_PLAN_HALT_EXTEND) {
    // newConfig + acceptance (rrt.cpp:20-101) of every extend with a FRAGILE
    // executed candidate, on the device's own candidate actions
    const int64_t n = st.n_targets;
    std::vector<uint32_t> ef(n);
    if ((rc = d2h(ef.data(), w->ef, n, s))) return rc;
    HIPCHK_P(hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; i++) {
      if (!(ef[i] & GBP_F_FRAGILE)) continue;
      int32_t nn = 0;
      double tg[8], sn0[8], act[10 * GBP_NUM_GEN_STATES];
      if ((rc = d2h(&nn, w->nn + i, 1, s)) || (rc = d2h(tg, w->targets + 8 * i, 8, s)) ||
          (rc = d2h(act, w->ca + 10 * GBP_NUM_GEN_STATES * i, 10 * GBP_NUM_GEN_STATES, s)))
        return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      if ((rc = d2h(sn0, T->v + 8 * (int64_t)nn, 8, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      const double best0 = gbp_host::state_distance(sn0, tg);
      double best = best0, s_test[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_test = 0, s_new[8];
      uint32_t fl = 0;
      int found = -1;
      for (int j = 0; j < GBP_NUM_GEN_STATES; j++) {
        uint32_t f = 0;
        const bool v = gbp_host::pair_check(t->host, sn0, act + 10 * j, direction, adaptive, s_test,
                                            &t_test, &f, nullptr);
        fl |= f & (GBP_F_VALID | GBP_F_OOD | GBP_F_NAN | GBP_F_LIMIT);
        if (v) {
          found = j;
          break;
        }
      }
      int32_t r = GBP_TRAPPED;
      if (found >= 0) {
        const double cur = gbp_host::state_distance(s_test, tg);
        if (cur < best) {
          best = cur;
          memcpy(s_new, s_test, sizeof s_new);
          r = cur <= GOAL_BOUNDS ? GBP_REACHED : GBP_ADVANCED;
          if ((rc = h2d(w->esn + 8 * i, s_new, 8, s)) ||
              (rc = h2d(w->ean + 10 * i, act + 10 * found, 10, s)))
            return rc;
        }
      }
      const uint32_t fr = fl | GBP_F_RESOLVED;
      if ((rc = h2d(w->eres + i, &r, 1, s)) || (rc = h2d(w->echo + i, &found, 1, s)) ||
          (rc = h2d(w->ef + i, &fr, 1, s)))
        return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      k++;
    }
    *resume_stage = 3;
  } else if (st.halt & GBP_PLAN_HALT_CONNECT) {
    // RRTConnectClass::attemptConnect (rrt_connect.cpp:20-91) of every
    // connection with a FRAGILE level, recursion replayed on the host
    if (!tree_ok(O)) return GBP_E_BAD_HANDLE;
    const int64_t n = st.n_added, base = st.added_base;
    const int cdir = direction == GBP_FORWARD ? GBP_REVERSE : GBP_FORWARD;
    std::vector<uint32_t> kf(n);
    if ((rc = d2h(kf.data(), w->kf, n, s))) return rc;
    HIPCHK_P(hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; i++) {
      if (!(kf[i] & GBP_F_FRAGILE)) continue;
      int32_t j = 0;
      double se[8], sq[8], sn[8] = {0, 0, 0, 0, 0, 0, 0, 0}, an[10];
      if ((rc = d2h(&j, w->nno + i, 1, s)) || (rc = d2h(sq, T->v + 8 * (base + i), 8, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      if ((rc = d2h(se, O->v + 8 * (int64_t)j, 8, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      const double t_s = gbp_host::pose_distance(sq, se) / V_NOM;
      uint32_t f = 0;
      const int32_t r = gbp_host::attempt_connect(t->host, se, sq, t_s, sn, an, cdir, adaptive,
                                                  GBP_CONNECT_MAX_DEPTH, &f);
      const uint32_t fr = f | GBP_F_RESOLVED;
      if ((rc = h2d(w->kres + i, &r, 1, s)) || (rc = h2d(w->kan + 10 * i, an, 10, s)) ||
          (rc = h2d(w->kf + i, &fr, 1, s)))
        return rc;
      if (r != GBP_TRAPPED && (rc = h2d(w->ksn + 8 * i, sn, 8, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      k++;
    }
    *resume_stage = 5;
  } else if (st.halt & GBP_PLAN_HALT_STAR) {
    // the RRT* insertion's connect checks (their pair checks, rows of stage 6)
    const int64_t n = st.star_rows;
    std::vector<uint32_t> rf(n);
    const gbp_plan_ws::StarSet &S = w->ss[st.halt_half & 1];
    if (n && (rc = d2h(rf.data(), S.srf, n, s))) return rc;
    HIPCHK_P(hipStreamSynchronize(s));
    for (int64_t i = 0; i < n; i++) {
      if (!(rf[i] & GBP_F_FRAGILE)) continue;
      double sv[8], av[10], sn[8], tn = 0;
      if ((rc = d2h(sv, S.srs + 8 * i, 8, s)) || (rc = d2h(av, S.sra + 10 * i, 10, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      uint32_t f = 0;
      const bool v = gbp_host::pair_check(t->host, sv, av, direction, adaptive, sn, &tn, &f, nullptr);
      const uint32_t fr = (f & ~GBP_F_FRAGILE) | (v ? GBP_F_VALID : 0u) | GBP_F_RESOLVED;
      if ((rc = h2d(S.srf + i, &fr, 1, s))) return rc;
      HIPCHK_P(hipStreamSynchronize(s));
      k++;
    }
    *resume_stage = 7;
  }
  if (*resume_stage >= 0) {
    st.halt = 0;
    if (!st.done) st.gate_seq = ~0ull;
    st.stat_fragile_resolved += k;
    if ((rc = h2d(w->st, &st, 1, s))) return rc;
    HIPCHK_P(hipStreamSynchronize(s));
  }
  if (n_resolved) *n_resolved = k;
  return GBP_OK;
}

}  // extern "C"
