// gbp_engine.hip — HIP kernels (gfx950, wave64) + the C ABI of include/gbp.h.
//
// Kernels:
//   K1 k_height / k_normal        batched FastTerrainMap lookups
//   K2 k_validate_direct          one lane per state-action pair
//   K2 k_validate_persistent      persistent waves; every lane evaluates ONE
//                                 sampled state per step and refills from a
//                                 global work counter as soon as its pair is
//                                 decided, so a wave never idles behind one
//                                 long-lived attempt (divergence is the cost
//                                 centre: most pairs die in 1-3 samples, a few
//                                 run ~19, SURVEY §7 "Divergence")
//   K3 k_sample_states / k_sample_actions / k_extend_prep / k_extend_select
//   K5 k_nearest                  (distance, index) lexicographic argmin
// MFMA is not used: there is no dense contraction on this path.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <cstring>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <new>
#include <vector>

#include "gbp.h"
#include "gbp_device.h"
#include "gbp_lane.h"
#include "gbp_um_order.h"
#include "gbp_internal.h"
#include "host/gbp_host_check.h"

using namespace gbp;

namespace {

constexpr uint64_t EXTEND_STREAM = GBP_EXTEND_STREAM;
constexpr int WAVE = 64;

// CM == 1: the coordinate vectors are staged in LDS (bracket fix-up and the
// bilinear x1/x2/y1/y2 then never touch global memory); CM == 2 computes
// them (gbp_device.h coord)
template <class ZT>
__device__ __forceinline__ TerrainView<ZT> stage_coords(const TerrainView<ZT> &T0, double *smem) {
  for (int i = threadIdx.x; i < T0.nx; i += blockDim.x) smem[i] = T0.x[i];
  for (int i = threadIdx.x; i < T0.ny; i += blockDim.x) smem[T0.nx + i] = T0.y[i];
  TerrainView<ZT> T = T0;
  T.x = smem;
  T.y = smem + T0.nx;
  __syncthreads();
  return T;
}

// LDS bytes of stage_coords for this terrain
// (rounded up to 16 B so the attempt rows behind it stay 16-B aligned)
inline size_t stage_bytes(int nx, int ny) { return sizeof(double) * (size_t)((nx + ny + 1) & ~1); }

// ============================================================================
// K1: batched terrain queries
// ============================================================================
// one probe per point: a single bracket pair and one cell fetch serve both
// getGroundHeight and heightIsNan; coordinates per CM (gbp_device.h coord).
template <class ZT, int CM>
__global__ __launch_bounds__(256) void k_height(TerrainView<ZT> T0, int64_t n,
                                                const double2 *__restrict__ xy,
                                                double *__restrict__ h,
                                                uint8_t *__restrict__ is_nan,
                                                uint8_t *__restrict__ ood) {
  extern __shared__ double k1_smem[];
  const TerrainView<ZT> T = CM == 1 ? stage_coords(T0, k1_smem) : T0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double2 p = xy[i];
    Probe<ZT> pr;
    probe<ZT, CM>(T, p.x, p.y, pr);
    double v;
    bool near = false;
    const bool ok = probe_height<ZT, CM>(T, pr, p.x, p.y, v, near);  // getGroundHeight
    const int r = probe_nan(pr);                              // heightIsNan
    if (h) h[i] = ok ? v : __builtin_nan("");
    if (is_nan) is_nan[i] = r != 0 ? 1 : 0;                   // UB (-1) reported as 1, like ood
    if (ood) ood[i] = (!ok || r < 0) ? 1 : 0;
  }
}

template <class ZT>
__global__ void k_normal(TerrainView<ZT> T, int64_t n, const double *__restrict__ xy,
                         double *__restrict__ nrm, uint8_t *__restrict__ ood) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double v[3];
    const bool ok = surface_normal(T, xy[2 * i], xy[2 * i + 1], v);
    nrm[3 * i] = v[0];
    nrm[3 * i + 1] = v[1];
    nrm[3 * i + 2] = v[2];
    if (ood) ood[i] = ok ? 0 : 1;
  }
}

template <class ZT>
__global__ void k_valid_states(TerrainView<ZT> T, int64_t n, const double *__restrict__ states,
                               const uint8_t *__restrict__ phase, int phase_all,
                               uint8_t *__restrict__ valid, uint32_t *__restrict__ flags,
                               uint32_t *__restrict__ counts) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double s[8];
#pragma unroll
    for (int k = 0; k < 8; k++) s[k] = states[8 * i + k];
    Acc acc{0, 0, 0};
    const bool v = is_valid_state(T, s, phase ? phase[i] : phase_all, acc);
    if (valid) valid[i] = v;
    if (flags) flags[i] = acc.flags | (v ? GBP_F_VALID : 0u);
    if (counts) counts[i] = (acc.G & 0xFFFFu) | (acc.V << 16);
  }
}

// ============================================================================
// K2 (direct): one lane per pair, the reference loops as written
// ============================================================================
// W = minimum waves per SIMD requested from the register allocator
// (__launch_bounds__ 2nd argument): 1 -> up to 512 VGPR+AGPR, 2 -> 256, 4 -> 128.
extern __shared__ double gbp_smem[];

template <class ZT, bool ADAPTIVE, int W, int CM>
__global__ __launch_bounds__(256, W) void k_validate_direct(
    TerrainView<ZT> T0, int64_t n, const double *__restrict__ S, const double *__restrict__ A,
    const uint8_t *__restrict__ dir, int dir_all, uint8_t *__restrict__ valid,
    double *__restrict__ s_new, double *__restrict__ t_new, uint32_t *__restrict__ flags,
    uint32_t *__restrict__ counts) {
  const TerrainView<ZT> T = CM == 1 ? stage_coords(T0, gbp_smem) : T0;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s[8], a[10], sn[8];
#pragma unroll
  for (int k = 0; k < 8; k++) s[k] = S[8 * i + k];
#pragma unroll
  for (int k = 0; k < 10; k++) a[k] = A[10 * i + k];
  double tn = 0;
  Acc acc{0, 0, 0};
  uint32_t f = 0;
  const int d = dir ? dir[i] : dir_all;
  const bool v = (d == GBP_FORWARD) ? pair_forward<ZT, ADAPTIVE>(T, s, a, sn, tn, acc, f)
                                    : pair_reverse<ZT, ADAPTIVE>(T, s, a, sn, tn, acc, f);
  f |= acc.flags | (v ? GBP_F_VALID : 0u);
  if (valid) valid[i] = v;
  if (s_new && (f & GBP_F_SNEW_SET)) {
#pragma unroll
    for (int k = 0; k < 8; k++) s_new[8 * i + k] = sn[k];
  }
  if (t_new && (f & GBP_F_TNEW_SET)) t_new[i] = tn;
  flags[i] = f;
  if (counts) counts[i] = (acc.G & 0xFFFFu) | (acc.V << 16);
}

// ============================================================================
// K2 (persistent): per-sample state machine with lane re-packing
// ============================================================================
// (lane state machine: gbp_lane.h)


// deferred s_new (round 4): a deciding lane queues (attempt, kind, parameter)
// in its wave's LDS ring instead of forming its s_new closed form under the
// deciding lanes' divergent mask in every step; once 64 are queued the wave
// forms all 64 converged (attempt rows re-read from L2) — once per 64
// decisions instead of once per step (~15 decisions per step and wave at
// config 3)
struct SnewRec {
  int idx, kind;
  double p;
};
constexpr int SN_RING = 2 * 64;  // entries per wave: < 64 left + up to 64 queued in a step

// -DGBP_XWAVE (A/B variant): the workgroup-level helper
// exchange.  Waves pair up (w, w ^ 1).  A wave whose own work is done does
// not exit while its partner still runs: it becomes 64 more helpers of the
// partner's owners.  Per step the partner (in its tail) publishes its owners'
// (stage, t, ts, V) in its box and raises seq; the helper wave evaluates the
// samples helpers n_idle .. n_idle + 63 would (same slot / owner rule, rows
// read from the partner's LDS rows), writes the result words and raises ack;
// the partner consumes them after its own helpers', in slot order.
struct XBox {
  int seq, ack, fin, n_idle;
  unsigned long long act;
  int st[64];
  uint32_t vb[64], r0[64], r1[64];
  double t[64], ts[64];
};

// (diagnostic build, -DGBP_LOOP_PROF: cycles per phase of the persistent loop,
// per wave, read by gbp_loop_prof_read; tools/loop_prof.py)
#ifdef GBP_LOOP_PROF
__device__ unsigned long long gbp_loop_prof[8192 * 12];
#define LP_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define LP_ADD(k, a, b) lp[k] += (b) - (a)
#else
#define LP_T(v)
#define LP_ADD(k, a, b)
#endif

template <class ZT, bool ADAPTIVE, int W, int CM, bool ONE>
__global__ __launch_bounds__(512, W) void k_validate_persistent(
    TerrainView<ZT> T0, int n, const double *__restrict__ S, const double *__restrict__ A,
    const uint8_t *__restrict__ dir, int dir_all, uint8_t *__restrict__ valid,
    double *__restrict__ s_new, double *__restrict__ t_new, uint32_t *__restrict__ flags,
    uint32_t *__restrict__ counts, const int *__restrict__ n_dev, int helpers, int xcd_map) {
#ifndef GBP_LDS_TERRAIN
  const TerrainView<ZT> T = CM == 1 ? stage_coords(T0, gbp_smem) : T0;
#else
  // A/B variant (upper bound of LDS terrain tiles): the
  // whole x-pair height array staged in LDS behind the s_new rings (only
  // terrains small enough: the host checks the fit), every gather from LDS
  TerrainView<ZT> T = CM == 1 ? stage_coords(T0, gbp_smem) : T0;
  {
    ZT *zl = (ZT *)((SnewRec *)(gbp_smem + (CM == 1 ? (T0.nx + T0.ny + 1) & ~1 : 0) +
                                (size_t)blockDim.x * SA_ROW) +
                    (blockDim.x / WAVE) * SN_RING);
    const int nz = 2 * (T0.nx - 1) * T0.ny;  // ZT elements (even: 8-B aligned pairs)
    typedef ZT zpair __attribute__((ext_vector_type(2)));
    for (int i = threadIdx.x; i < nz / 2; i += blockDim.x)
      ((zpair *)zl)[i] = ((const zpair *)T0.z)[i];
    __syncthreads();
#ifndef GBP_LDS_TERRAIN_STAGE_ONLY
    T.z = zl;
#endif
  }
#endif
  if (n_dev) n = *n_dev;  // batch size produced on the device (planner loop)
  const int lane = threadIdx.x & (WAVE - 1);
  const unsigned long long lt_mask = (1ull << lane) - 1ull;
  double *const SA = gbp_smem + (CM == 1 ? (T0.nx + T0.ny + 1) & ~1 : 0);  // attempt rows
  double *const wave_rows = SA + (size_t)(threadIdx.x & ~(WAVE - 1)) * SA_ROW;
  SnewRec *const ring = (SnewRec *)(SA + (size_t)blockDim.x * SA_ROW) + (threadIdx.x / WAVE) * SN_RING;
  int ring_n = 0;  // wave-uniform
  // s_new of the ring's first cnt entries, one per lane (converged)
  auto flush = [&](int cnt) {
    if (lane < cnt) {
      const SnewRec r = ring[lane];
      double sv[8], av[10], o[8];
#pragma unroll
      for (int k = 0; k < 8; k++) sv[k] = S[8 * (size_t)r.idx + k];
#pragma unroll
      for (int k = 0; k < 10; k++) av[k] = A[10 * (size_t)r.idx + k];
      // one closed form for every kind: sample_state at FWD_STANCE is
      // apply_stance's expression tree (same operands, same bits)
      sample_state(sv, av,
                   r.kind == SN_STANCE_S ? ST_FWD_STANCE
                                         : (r.kind == SN_FLIGHT_B ? ST_FWD_LAND : ST_REV_STANCE),
                   r.p, o);
#pragma unroll
      for (int k = 0; k < 8; k++) s_new[8 * (size_t)r.idx + k] = o[k];
    }
  };
#ifdef GBP_XWAVE
  XBox *const xbox = (XBox *)((SnewRec *)(SA + (size_t)blockDim.x * SA_ROW) + (blockDim.x / WAVE) * SN_RING);
  const int wv = threadIdx.x / WAVE;
  XBox *const mybox = xbox + wv;
  XBox *const pbox = xbox + (wv ^ 1);
  const bool has_partner = (wv ^ 1) < (int)(blockDim.x / WAVE);
  double *const partner_rows = SA + (size_t)((wv ^ 1) * WAVE) * SA_ROW;
  if (lane == 0) {
    mybox->seq = 0;
    mybox->ack = 0;
    mybox->fin = 0;
  }
  __syncthreads();
  int myseq = 0, served = 0;
  bool fin_sent = false;
#endif
  Lane L;
  L.s = SA + (size_t)threadIdx.x * SA_ROW;
  L.a = L.s + 8;
  L.stage = ST_IDLE;
  // work source: a fixed contiguous slice [cur, end) per wave, handed out to
  // the wave's idle lanes in order (no atomics).  Dynamic dequeues (one or
  // eight device-scope heads, chunked, per-workgroup LDS queues; round 4: the
  // last 15-60 % of a batch in chunks from 64 counters) were measured no
  // faster and removed.
  unsigned int cur, end;
  {
    const unsigned int waves = gridDim.x * (blockDim.x / WAVE);
    // xcd_map: workgroup b runs on XCD b % 8 (round-robin dispatch); numbering
    // the slices XCD-major gives each XCD one contiguous eighth of the batch,
    // so a batch ordered by position keeps each XCD's L2 on its own stripe
    const unsigned int wg = (xcd_map && (gridDim.x & 7u) == 0)
                                ? (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3)
                                : blockIdx.x;
    const unsigned int wid = wg * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    cur = (unsigned int)(((unsigned long long)n * wid) / waves);
    end = (unsigned int)(((unsigned long long)n * (wid + 1)) / waves);
  }
#ifdef GBP_LOOP_PROF
  unsigned long long lp[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  lp[8] = __builtin_amdgcn_s_memrealtime();
  LP_T(lp_start);
#endif
  for (;;) {
    LP_T(t0);
    const bool need = L.stage == ST_IDLE;
    unsigned long long m = __ballot(need);
    if (m && cur < end) {
      const unsigned int take = min(end - cur, (unsigned int)__popcll(m));
      const unsigned int rank = (unsigned int)__popcll(m & lt_mask);
      const bool mine = need && rank < take;
      if (mine) {
        const unsigned int i = cur + rank;
        L.idx = (int)i;
#pragma unroll
        for (int k = 0; k < 8; k++) L.s[k] = S[8 * (size_t)i + k];
#pragma unroll
        for (int k = 0; k < 10; k++) L.a[k] = A[10 * (size_t)i + k];
        L.f = 0;
        L.acc = Acc{0, 0, 0};
        L.snew_kind = SN_NONE;
        L.tnew_set = 0;
        const int d = dir ? dir[i] : dir_all;
        enter_stage(L, d == GBP_FORWARD ? ST_FWD_STANCE : ST_REV_FLIGHT);
      }
      cur += take;
    }
    const unsigned long long act = __ballot(L.stage != ST_IDLE);
#ifdef GBP_XWAVE
    // this wave's work is done: serve the partner's requests until it is done
    bool serve = false;
    if (!act) {
      if (!has_partner) break;
      if (!fin_sent) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&mybox->fin, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        fin_sent = true;
      }
      int pseq, pfin;
      for (;;) {
        pseq = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&pbox->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        pfin = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&pbox->fin, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (pseq != served || pfin) break;
        __builtin_amdgcn_s_sleep(1);
      }
      if (pseq == served) break;  // the partner finished with no request pending
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      served = pseq;
      serve = true;
    }
#else
    if (!act) break;
#endif
    LP_T(t1);
    LP_ADD(0, t0, t1);
    const bool owner = L.stage != ST_IDLE;
    asm volatile("" ::: "memory");  // re-read attempt rows per step (no long live ranges)
    // ---- the sample each lane evaluates this step --------------------------
    // Normally a lane evaluates its own attempt's next sample.  In a wave's
    // tail (no work left to refill idle lanes) the idle lanes become helpers:
    // helper j of owner r evaluates the owner's sample `slot` steps ahead,
    // assuming the samples in between pass (advance_on_success, across stage
    // boundaries: stance -> flight -> landing on the all-pass path); the
    // owner then consumes the results in order and stops at the first
    // failure or decision, so exactly the reference's samples are counted.
    const int n_act = __popcll(act);
    const bool tail = helpers && n_act < WAVE;  // every idle lane is exhausted here
    int st = L.stage, slot = 0;
    const double *ps = L.s;  // the attempt row this lane samples
    double t_eval = owner ? stage_time(L) : 0.0;
    uint32_t vbase = L.acc.V;
    bool has = owner;
#ifdef GBP_XWAVE
    // a tail step with the partner free: publish the owners' loop state
    bool xhelp = false;
    if (tail && !serve && has_partner) {
      xhelp = __builtin_amdgcn_readfirstlane(
                  __hip_atomic_load(&pbox->fin, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0;
      if (xhelp) {
        mybox->st[lane] = L.stage;
        mybox->t[lane] = L.t;
        mybox->ts[lane] = L.ts;
        mybox->vb[lane] = L.acc.V;
        if (lane == 0) {
          mybox->act = act;
          mybox->n_idle = WAVE - n_act;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        myseq++;
        if (lane == 0) __hip_atomic_store(&mybox->seq, myseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if (serve) {
      // helper n_idle + lane of the partner's owners (the rule of the tail below)
      const unsigned long long pact = pbox->act;
      const int pn = __popcll(pact);
      const int j = pbox->n_idle + lane;
      const int src = nth_set_bit(pact, j % pn);
      slot = 1 + j / pn;
      ps = partner_rows + src * SA_ROW;
      st = pbox->st[src];
      double t = pbox->t[src], ts = pbox->ts[src];
      vbase = pbox->vb[src];
      has = true;
      for (int k = 0; k < slot && has; k++) has = advance_on_success<ADAPTIVE>(st, ps + 8, t, ts);
      t_eval = sample_time(st, ps + 8, t);
    } else
#endif
    if (tail) {
      const unsigned long long idle = ~act;
      const int j = __popcll(idle & lt_mask);
      const int src = owner ? lane : nth_set_bit(act, j % n_act);
      slot = owner ? 0 : 1 + j / n_act;
      ps = wave_rows + src * SA_ROW;  // the owner's attempt row
      st = __shfl(L.stage, src);
      double t = __shfl(L.t, src), ts = __shfl(L.ts, src);
      vbase = __shfl(L.acc.V, src);
      if (!owner) {
        has = true;
        for (int k = 0; k < slot && has; k++) has = advance_on_success<ADAPTIVE>(st, ps + 8, t, ts);
        t_eval = sample_time(st, ps + 8, t);
      }
    }
    LP_T(t2);
    LP_ADD(1, t1, t2);
    Acc acc_s{0, vbase + (uint32_t)slot, 0};
    bool ok = false;
    if (has) {
      double sc[8];
      sample_state(ps, ps + 8, st, t_eval, sc);
      // ONE (a template parameter, so the kernel holds one bracket form and
      // its registers): the terrain's one-step guess is exact on both axes
      ok = is_valid_state<ZT, CM, ONE>(T, sc, stage_phase(st), acc_s);
    }
    LP_T(t3);
    LP_ADD(2, t2, t3);
#ifdef GBP_XWAVE
    if (serve) {  // the results, then the acknowledgement
      pbox->r0[lane] = (acc_s.flags & 0xFFFFu) | (ok ? 1u << 16 : 0u) | (has ? 1u << 17 : 0u) |
                       ((acc_s.V - (vbase + (uint32_t)slot)) << 18);
      pbox->r1[lane] = acc_s.G;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&pbox->ack, served, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
#endif
    bool decided = false;
    if (owner) {  // the lane's own sample
      L.acc.G += acc_s.G;
      L.acc.V = acc_s.V;
      L.acc.flags |= acc_s.flags;
      decided = (acc_s.flags & GBP_F_LIMIT) ? true : transition<ADAPTIVE>(L, ok);
    }
    if (tail) {  // consume helper results in slot order
      const unsigned long long idle = ~act;
      const int n_idle = WAVE - n_act;
#ifdef GBP_XWAVE
      // the partner's 64 helpers come after this wave's own (helpers n_idle ..)
      int n_help = n_idle;
      if (xhelp) {
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                   &mybox->ack, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) != myseq)
          __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        n_help += WAVE;
      }
#else
      const int n_help = n_idle;
#endif
      const uint32_t w0 = (acc_s.flags & 0xFFFFu) | (ok ? 1u << 16 : 0u) | (has ? 1u << 17 : 0u) |
                          ((acc_s.V - (vbase + (uint32_t)slot)) << 18);
      const uint32_t w1 = acc_s.G;
      const int my_rank = __popcll(act & lt_mask);
      bool chain = owner && !decided && ok;
      const int kmax = (n_help + n_act - 1) / n_act;
      for (int k = 1; k <= kmax; k++) {
        // every owner's chain has ended (a failure or a decision): the rest of
        // the helpers' results are not consumed (config 3 0.1315 -> 0.1206 ms,
        // config 2 0.0622 -> 0.0506 ms: the loop ran n_idle / n_act rounds of
        // shuffles and transitions whatever the chains did)
        if (!__ballot(chain)) break;
        const int j = (k - 1) * n_act + my_rank;
        const bool exists = owner && j < n_help;
        const int src = (exists && j < n_idle) ? nth_set_bit(idle, j) : lane;
        uint32_t r0 = __shfl(w0, src), r1 = __shfl(w1, src);
#ifdef GBP_XWAVE
        if (exists && j >= n_idle) {
          r0 = mybox->r0[j - n_idle];
          r1 = mybox->r1[j - n_idle];
        }
#endif
        if (chain && exists && ((r0 >> 17) & 1u)) {
          L.acc.G += r1;
          L.acc.V += (r0 >> 18) & 1u;
          L.acc.flags |= r0 & 0xFFFFu;
          const bool okk = (r0 >> 16) & 1u;
          decided = (r0 & GBP_F_LIMIT) ? true : transition<ADAPTIVE>(L, okk);
          chain = !decided && okk;
        } else {
          chain = false;
        }
      }
    }
    asm volatile("" ::: "memory");
    LP_T(t4);
    LP_ADD(3, t3, t4);
#ifdef GBP_LOOP_PROF
    lp[6] += tail ? 1 : 0;
    lp[7] += 1;
#endif
    const bool fin = owner && decided;
#ifdef GBP_SNEW_IMMEDIATE
    // A/B variant: the deciding lane forms s_new from its LDS row at once
    // (round 3's form; no ring, no re-read of the rows)
    if (fin && s_new && L.snew_kind != SN_NONE) {
      double o[8];
      sample_state(L.s, L.a,
                   L.snew_kind == SN_STANCE_S ? ST_FWD_STANCE
                                              : (L.snew_kind == SN_FLIGHT_B ? ST_FWD_LAND : ST_REV_STANCE),
                   L.snew_p, o);
#pragma unroll
      for (int k = 0; k < 8; k++) s_new[8 * (size_t)L.idx + k] = o[k];
    }
    const bool queue = false;
#else
    const bool queue = fin && s_new && L.snew_kind != SN_NONE;
#endif
    if (fin) {
      const size_t i = (size_t)L.idx;
      uint32_t f = L.f | L.acc.flags;
      if (L.snew_kind != SN_NONE) f |= GBP_F_SNEW_SET;
      if (L.tnew_set) f |= GBP_F_TNEW_SET;
      if (valid) valid[i] = (f & GBP_F_VALID) ? 1 : 0;
      if (t_new && L.tnew_set) t_new[i] = L.tnew;
      flags[i] = f;
      if (counts) counts[i] = (L.acc.G & 0xFFFFu) | (L.acc.V << 16);
    }
    const unsigned long long qm = __ballot(queue);
    if (qm) {
      if (queue) ring[ring_n + __popcll(qm & lt_mask)] = SnewRec{L.idx, L.snew_kind, L.snew_p};
      ring_n += __popcll(qm);
      if (ring_n >= WAVE) {
        flush(WAVE);
        ring_n -= WAVE;
        SnewRec r;
        if (lane < ring_n) r = ring[WAVE + lane];
        if (lane < ring_n) ring[lane] = r;
      }
    }
    if (fin) L.stage = ST_IDLE;
    LP_T(t5);
    LP_ADD(4, t4, t5);
  }
  if (ring_n) flush(ring_n);
#ifdef GBP_LOOP_PROF
  LP_T(lp_end);
  lp[5] = lp_end - lp_start;
  lp[9] = __builtin_amdgcn_s_memrealtime();
  {
    unsigned int hw;  // HW_ID: the wave's SIMD / CU / SE
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    lp[10] = hw;
    unsigned int xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    lp[11] = xcc;
  }
  const unsigned int gw = blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
  if (lane == 0 && gw < 8192)
    for (int k = 0; k < 12; k++) gbp_loop_prof[12 * gw + k] = lp[k];
#endif
}

// ============================================================================
// K3: samplers and the batched extend
// ============================================================================
// s_from / s_to of the direction-biased draws (rrt_connect.cpp:248-252)
struct DirPair {
  double from[8], to[8];
};

template <class ZT>
__global__ void k_sample_states(TerrainView<ZT> T, int64_t n, uint64_t seed, uint64_t stream_id,
                                int64_t index_base, int require_phase, int max_tries,
                                double *__restrict__ states, int32_t *__restrict__ tries,
                                gbp_sampling cfg, DirPair dp) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double q[8];
    int got = -1;
    const int mt = max_tries > 0 ? max_tries : 1;
    for (int k = 0; k < mt; k++) {
      sample_state_cfg_try(T, cfg, dp.from, dp.to, seed, stream_id, index_base + i, k, q);
      if (require_phase < 0) { got = k + 1; break; }
      Acc acc{0, 0, 0};
      if (is_valid_state(T, q, require_phase, acc)) { got = k + 1; break; }
    }
#pragma unroll
    for (int k = 0; k < 8; k++) states[8 * i + k] = q[k];
    if (tries) tries[i] = got;
  }
}

__global__ void k_sample_actions(int64_t n, const double *__restrict__ normals, uint64_t seed,
                                 uint64_t stream_id, int64_t index_base,
                                 double *__restrict__ actions) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double nv[3] = {normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]};
    double a[10];
    sample_action(nv, seed, stream_id, index_base + i, a);
#pragma unroll
    for (int k = 0; k < 10; k++) actions[10 * i + k] = a[k];
  }
}

// getRandomAction(surf_norm, direction, flag, p, s, s_near) for n draws
// (gbp_sample_actions_dir_dev)
__global__ void k_sample_actions_dir(int64_t n, const double *__restrict__ normals,
                                     const double *__restrict__ s, const double *__restrict__ s_near,
                                     const uint8_t *__restrict__ dir, int dir_all, gbp_sampling cfg,
                                     uint64_t seed, uint64_t stream_id, int64_t index_base,
                                     double *__restrict__ actions) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double nv[3] = {normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]};
    double a[10];
    sample_action_cfg(nv, cfg, dir ? dir[i] : dir_all, s + 8 * i, s_near + 8 * i, seed, stream_id,
                      index_base + i, a);
#pragma unroll
    for (int k = 0; k < 10; k++) actions[10 * i + k] = a[k];
  }
}

// one thread per (extend i, candidate j): candidate action j of extend i is
// getRandomAction(getSurfaceNormal(target_i), direction, flag, p, target_i,
// s_near_i) (rrt.cpp:34, :49) from stream (seed, EXTD, (base+i)*8+j)
template <class ZT>
__global__ void k_extend_prep(TerrainView<ZT> T, int64_t n, const double *__restrict__ s_near,
                              const double *__restrict__ target, const uint8_t *__restrict__ dir,
                              int dir_all, uint64_t seed, int64_t extend_base,
                              double *__restrict__ cand_s, double *__restrict__ cand_a,
                              uint8_t *__restrict__ cand_dir, gbp_sampling cfg) {
  const int64_t m = n * GBP_NUM_GEN_STATES;
  for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < m;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = c / GBP_NUM_GEN_STATES;
    const int j = (int)(c - i * GBP_NUM_GEN_STATES);
    double nv[3];
    surface_normal(T, target[8 * i], target[8 * i + 1], nv);  // rrt.cpp:25
    double a[10];
    const int d = dir ? dir[i] : dir_all;
    sample_action_cfg(nv, cfg, d, target + 8 * i, s_near + 8 * i, seed, EXTEND_STREAM,
                      (extend_base + i) * 8 + j, a);
#pragma unroll
    for (int k = 0; k < 10; k++) cand_a[10 * c + k] = a[k];
#pragma unroll
    for (int k = 0; k < 8; k++) cand_s[8 * c + k] = s_near[8 * i + k];
    cand_dir[c] = (uint8_t)d;
  }
}

// rrt.cpp:20-70 selection + rrt.cpp:84-101 acceptance
__global__ void k_extend_select(int64_t n, const double *__restrict__ s_near,
                                const double *__restrict__ target,
                                const double *__restrict__ cand_a,
                                const double *__restrict__ cand_snew,
                                const uint32_t *__restrict__ cand_flags,
                                const uint32_t *__restrict__ cand_counts,
                                int32_t *__restrict__ result, int32_t *__restrict__ chosen,
                                double *__restrict__ s_new, double *__restrict__ a_new,
                                uint32_t *__restrict__ counts, uint32_t *__restrict__ ext_flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double sn[8], tg[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      sn[k] = s_near[8 * i + k];
      tg[k] = target[8 * i + k];
    }
    int found = -1;
    uint32_t G = 0, V = 0, ef = 0;
    for (int j = 0; j < GBP_NUM_GEN_STATES; j++) {
      const int64_t c = i * GBP_NUM_GEN_STATES + j;
      G += GBP_COUNT_G(cand_counts[c]);
      V += GBP_COUNT_V(cand_counts[c]);
      ef |= cand_flags[c] & (GBP_F_VALID | GBP_F_OOD | GBP_F_NAN | GBP_F_FRAGILE | GBP_F_LIMIT);
      if (cand_flags[c] & GBP_F_VALID) {
        found = j;
        break;
      }
    }
    const double d0 = state_distance(sn, tg);
    double best = d0;
    double st[8];
    if (found >= 0) {
      const int64_t c = i * GBP_NUM_GEN_STATES + found;
#pragma unroll
      for (int k = 0; k < 8; k++) st[k] = cand_snew[8 * c + k];
      const double cur = state_distance(st, tg);
      if (cur < best) {
        best = cur;
#pragma unroll
        for (int k = 0; k < 8; k++) s_new[8 * i + k] = st[k];
#pragma unroll
        for (int k = 0; k < 10; k++) a_new[10 * i + k] = cand_a[10 * c + k];
      }
    }
    int r;
    if (best == state_distance(sn, tg)) r = GBP_TRAPPED;
    else r = (state_distance(st, tg) <= GOAL_BOUNDS) ? GBP_REACHED : GBP_ADVANCED;
    result[i] = r;
    if (chosen) chosen[i] = found;
    if (counts) counts[i] = (G & 0xFFFFu) | (V << 16);
    if (ext_flags) ext_flags[i] = ef;
  }
}

// ============================================================================
// K5: nearest neighbour, one workgroup per query
// ============================================================================
__device__ __forceinline__ void lex_min(double &d, int &i, double d2, int i2) {
  if (d2 < d || (d2 == d && i2 < i)) {
    d = d2;
    i = i2;
  }
}

__global__ __launch_bounds__(256) void k_nearest(int64_t n_query, const double *__restrict__ q,
                                                 int64_t n_vert, const double *__restrict__ v,
                                                 int32_t *__restrict__ idx,
                                                 double *__restrict__ dist) {
  __shared__ double sd[256 / WAVE];
  __shared__ int si[256 / WAVE];
  for (int64_t qi = blockIdx.x; qi < n_query; qi += gridDim.x) {
    double qq[8];
#pragma unroll
    for (int k = 0; k < 8; k++) qq[k] = q[8 * qi + k];
    double best = INFINITY;
    int bi = 0x7FFFFFFF;
    for (int64_t j = threadIdx.x; j < n_vert; j += blockDim.x) {
      double vv[8];
#pragma unroll
      for (int k = 0; k < 8; k++) vv[k] = v[8 * j + k];
      const double c = state_distance(qq, vv);  // stateDistance(q, vertex), planner_class.cpp:193
      if (c < best) {  // strict <, increasing j: lowest index among equals
        best = c;
        bi = (int)j;
      }
    }
#pragma unroll
    for (int off = WAVE / 2; off > 0; off >>= 1) {
      const double d2 = __shfl_down(best, off);
      const int i2 = __shfl_down(bi, off);
      lex_min(best, bi, d2, i2);
    }
    const int w = threadIdx.x / WAVE;
    if ((threadIdx.x & (WAVE - 1)) == 0) {
      sd[w] = best;
      si[w] = bi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int k = 1; k < (int)(blockDim.x / WAVE); k++) lex_min(best, bi, sd[k], si[k]);
      if (bi == 0x7FFFFFFF) bi = 0;  // nothing < INFINITY: the reference keeps index 0
      idx[qi] = bi;
      if (dist) dist[qi] = best;
    }
    __syncthreads();
  }
}

// Many queries against a large tree: 256 queries per workgroup (one per
// thread, held in registers) and the vertices streamed through LDS in tiles
// of 256, so each vertex is read from L2 once per 256 queries instead of once
// per query.  Same distance, same strict-< scan in ascending index order.
__global__ __launch_bounds__(256) void k_nearest_tiled(int64_t n_query,
                                                       const double *__restrict__ q,
                                                       int64_t n_vert,
                                                       const double *__restrict__ v,
                                                       int32_t *__restrict__ idx,
                                                       double *__restrict__ dist) {
  __shared__ double tile[256 * 8];
  const int64_t qi = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const bool live = qi < n_query;
  double qq[8];
#pragma unroll
  for (int k = 0; k < 8; k++) qq[k] = live ? q[8 * qi + k] : 0.0;
  double best = INFINITY;
  int bi = 0;  // nothing < INFINITY: the reference keeps index 0
  for (int64_t j0 = 0; j0 < n_vert; j0 += 256) {
    const int cnt = (int)min<int64_t>(256, n_vert - j0);
    __syncthreads();
    for (int e = threadIdx.x; e < cnt * 8; e += blockDim.x) tile[e] = v[8 * j0 + e];
    __syncthreads();
    for (int j = 0; j < cnt; j++) {
      const double c = state_distance(qq, tile + 8 * j);
      if (c < best) {
        best = c;
        bi = (int)(j0 + j);
      }
    }
  }
  if (live) {
    idx[qi] = bi;
    if (dist) dist[qi] = best;
  }
}

// PlannerClass::neighborhoodDist (planner_class.cpp:173-182): the vertices
// with 0 < stateDistance(q, v) <= radius, in the order the reference's vertex
// map (keys 0..n_vert-1) iterates them (gbp_um_order.h), position p holding
// key um_key_at(p, n_vert).  One workgroup per query; out[q][0..max_out)
// holds the first max_out neighbours, count[q] the total (may exceed max_out).
__global__ __launch_bounds__(256) void k_neighbors(int64_t n_query, const double *__restrict__ q,
                                                   int64_t n_vert, const double *__restrict__ v,
                                                   double radius, int max_out,
                                                   int32_t *__restrict__ out,
                                                   int32_t *__restrict__ count) {
  __shared__ int wave_cnt[256 / WAVE];
  const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int64_t qi = blockIdx.x; qi < n_query; qi += gridDim.x) {
    double qq[8];
#pragma unroll
    for (int k = 0; k < 8; k++) qq[k] = q[8 * qi + k];
    int base = 0;
    const int m = n_vert > 0 ? um_epoch(n_vert) : 0;
    for (int64_t p0 = 0; p0 < n_vert; p0 += blockDim.x) {
      const int64_t p = p0 + threadIdx.x;
      bool hit = false;
      int64_t j = 0;
      if (p < n_vert) {
        j = um_key_at(p, n_vert, m);
        const double d = state_distance(qq, v + 8 * j);
        hit = (d <= radius) && (d > 0);
      }
      const unsigned long long m = __ballot(hit);
      if (lane == 0) wave_cnt[w] = __popcll(m);
      __syncthreads();
      int off = base;
      int total = 0;
      for (int k = 0; k < (int)(blockDim.x / WAVE); k++) {
        if (k < w) off += wave_cnt[k];
        total += wave_cnt[k];
      }
      if (hit) {
        const int pos = off + __popcll(m & lt);
        if (pos < max_out) out[qi * (int64_t)max_out + pos] = (int32_t)j;
      }
      base += total;
      __syncthreads();
    }
    if (threadIdx.x == 0) count[qi] = base;
  }
}

// PlannerClass::neighborhoodN (planner_class.cpp:151-171): the n_nearest
// vertices of smallest stateDistance(q, v), in the order the reference pops
// its min-heap of std::pair<double, int> (std::greater): ascending distance,
// equal distances by ascending index.  A NaN distance orders after every
// number (the reference's heap order is then unspecified).  One wave per
// query: lane l holds the l-th smallest (distance, index) seen so far; the
// tree streams past in chunks of 64 vertices (one coalesced 64-B row per
// lane); a chunk with no candidate below the current n-th key is skipped on
// one ballot, otherwise it is sorted across the lanes (bitonic network on
// shuffles) and merged into the list (min against the reversed chunk, then
// a bitonic merge) — the "k-nearest wavefront scan" of SURVEY config 5.
__device__ __forceinline__ bool knn_less(double da, int ia, double db, int ib) {
  return da < db || (da == db && ia < ib);
}
// one compare-exchange stage with lane ^ j: keep the smaller key iff `lo`
__device__ __forceinline__ void knn_cx(double &kd, int &ki, double &od, int j, bool lo) {
  const double pd = __shfl_xor(kd, j);
  const int pi = __shfl_xor(ki, j);
  const double po = __shfl_xor(od, j);
  const bool take = lo ? knn_less(pd, pi, kd, ki) : knn_less(kd, ki, pd, pi);
  if (take) {
    kd = pd;
    ki = pi;
    od = po;
  }
}

// YAW: the cost_add_yaw distance of neighborhoodN (planner_class.cpp:157-158,
// planning_utils.h:146-155): poseDistance(q, v) * lw + stateYawDistance(q, v)
// * yw, the yaws given (glibc atan2, formed by the caller)
template <bool YAW>
__global__ __launch_bounds__(256) void k_knn(int64_t n_query, const double *__restrict__ q,
                                             int64_t n_vert, const double *__restrict__ v, int nk,
                                             int32_t *__restrict__ out, double *__restrict__ dist,
                                             const double *__restrict__ qyaw,
                                             const double *__restrict__ vyaw, double lw, double yw) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / WAVE);
  for (int64_t qi = blockIdx.x * (int64_t)(blockDim.x / WAVE) + threadIdx.x / WAVE; qi < n_query;
       qi += waves) {
    double qq[8];
#pragma unroll
    for (int k = 0; k < 8; k++) qq[k] = q[8 * qi + k];
    // the list: key (kd = the distance with NaN as +inf, ki) and the distance itself
    double kd = INFINITY, od = __builtin_nan("");
    int ki = 0x7FFFFFFF;
    for (int64_t j0 = 0; j0 < n_vert; j0 += WAVE) {
      const int64_t j = j0 + lane;
      double cd = INFINITY, co = __builtin_nan("");
      int ci = 0x7FFFFFFF;
      if (j < n_vert) {
        if constexpr (YAW)
          co = pose_distance(qq, v + 8 * j) * lw + yaw_distance(qyaw[qi], vyaw[j]) * yw;
        else
          co = state_distance(qq, v + 8 * j);
        cd = isnan(co) ? INFINITY : co;
        ci = (int)j;
      }
      const double td = __shfl(kd, nk - 1);
      const int ti = __shfl(ki, nk - 1);
      if (!__ballot(knn_less(cd, ci, td, ti))) continue;
      // sort the chunk ascending (bitonic network, 21 stages)
#pragma unroll
      for (int k = 2; k <= WAVE; k <<= 1)
#pragma unroll
        for (int jj = k >> 1; jj > 0; jj >>= 1) {
          const bool up = (lane & k) == 0;
          knn_cx(cd, ci, co, jj, ((lane & jj) == 0) == up);
        }
      // the 64 smallest of list + chunk: lane l against the chunk's lane 63 - l
      // (a bitonic sequence), then one bitonic merge
      {
        const double rd = __shfl(cd, WAVE - 1 - lane);
        const int ri = __shfl(ci, WAVE - 1 - lane);
        const double ro = __shfl(co, WAVE - 1 - lane);
        if (knn_less(rd, ri, kd, ki)) {
          kd = rd;
          ki = ri;
          od = ro;
        }
      }
#pragma unroll
      for (int jj = WAVE >> 1; jj > 0; jj >>= 1) knn_cx(kd, ki, od, jj, (lane & jj) == 0);
    }
    if (lane < nk) {
      const bool real = ki != 0x7FFFFFFF;
      out[qi * nk + lane] = real ? ki : -1;
      if (dist) dist[qi * nk + lane] = real ? od : __builtin_nan("");
    }
  }
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
namespace {

// coordinate mode of the hot kernels (gbp_device.h coord): LDS-staged vectors
// when they fit (measured 1-2 % ahead of computing them at 1024^2), else the
// verified affine form (e.g. 4096^2, whose vectors leave no LDS for the
// attempt rows), else global memory
int coord_mode(const gbp_terrain *t, bool lds_ok) {
  if (lds_ok) return 1;
  return (t->opt_affine && t->affine) ? 2 : 0;
}

// the validate kernels' coordinate mode: LDS only if the vectors fit next to
// the attempt rows with room for the W workgroups of 256 lanes that share a CU
// (160 KB per CU; the direct kernel has no rows)
int validate_coord_mode(const gbp_terrain *t, bool direct) {
  // the attempt rows and s_new rings are the persistent kernel's alone
  // (launch_validate_w allocates neither for the direct kernel)
  const size_t rows =
      direct ? 0 : (sizeof(double) * SA_ROW + sizeof(SnewRec) * SN_RING / WAVE) * (size_t)t->opt_block;
  const size_t per_cu = std::max<int64_t>(1, t->opt_waves * 256 / t->opt_block) *
                        (stage_bytes(t->nx, t->ny) + rows);
  const bool lds_ok = t->opt_lds_coords && stage_bytes(t->nx, t->ny) + rows <= t->lds_max &&
                      (direct || per_cu <= 160 * 1024);
  // the persistent kernel's LDS / computed modes are instantiated with the
  // straight-line bracket only: a terrain whose one-step guess is not exact
  // on both axes reads its vectors from global memory (general search)
  if (!direct && !(t->one_x && t->one_y)) return 0;
  return coord_mode(t, lds_ok);
}

template <class ZT, bool AD, int W, int CM, bool ONE>
int launch_validate_w(gbp_terrain *t, int64_t n, const double *s, const double *a,
                      const uint8_t *dir, int dir_all, uint8_t *valid, double *s_new,
                      double *t_new, uint32_t *flags, uint32_t *counts, hipStream_t st,
                      const int *n_dev) {
  const TerrainView<ZT> T = view<ZT>(t);
  const int block = (int)t->opt_block;
  const size_t coords = CM == 1 ? stage_bytes(t->nx, t->ny) : 0;
  const size_t rows = sizeof(double) * SA_ROW * (size_t)block;  // persistent kernel only
  const int64_t chunk = (int64_t)1 << 30;
  for (int64_t off = 0; off < n; off += chunk) {
    const int64_t m = std::min<int64_t>(n - off, chunk);
    const uint8_t *d = dir ? dir + off : nullptr;
    uint8_t *v = valid ? valid + off : nullptr;
    double *sn = s_new ? s_new + 8 * off : nullptr;
    double *tn = t_new ? t_new + off : nullptr;
    uint32_t *c = counts ? counts + off : nullptr;
    if (t->opt_kernel == GBP_KERNEL_DIRECT && !n_dev) {
      // the direct form inlines the state check at five call sites: it gets the
      // whole register file (W = 1) whatever the persistent kernel's budget is
      const int db = std::min(block, 256);  // k_validate_direct: __launch_bounds__(256)
      const unsigned g = (unsigned)((m + db - 1) / db);
      hipLaunchKernelGGL((k_validate_direct<ZT, AD, 1, CM == 2 ? 0 : CM>), dim3(g), dim3(db), coords, st, T, m,
                         s + 8 * off, a + 10 * off, d, dir_all, v, sn, tn, flags + off, c);
    } else {
      // persistent: one workgroup per resident slot (opt_waves waves per SIMD;
      // W, the register budget, allows at least that many); LDS: the
      // coordinate vectors (CM 1), the attempt rows, the s_new rings
      const int64_t resident = (int64_t)t->num_cus * std::max<int64_t>(1, t->opt_waves * 256 / block);
      // every resident slot as long as each wave gets an attempt: a batch
      // smaller than the resident lanes still spreads over every CU, its
      // waves starting with idle lanes that help from the first step
      // (65,536 attempts: 0.084 -> 0.072 ms; 262,144: unchanged)
      const int64_t g = std::max<int64_t>(1, std::min<int64_t>(resident, (m + WAVE - 1) / WAVE));
      const size_t ring = sizeof(SnewRec) * SN_RING * (size_t)(block / WAVE);
#ifdef GBP_LDS_TERRAIN
      const size_t zb = sizeof(ZT) * 2 * (size_t)(t->nx - 1) * t->ny;
      if (coords + rows + ring + zb > t->lds_max) return GBP_E_SHAPE;  // the A/B variant only
#elif defined(GBP_XWAVE)
      const size_t zb = sizeof(XBox) * (size_t)(block / WAVE);  // the helper exchange's boxes
#else
      const size_t zb = 0;
#endif
      hipLaunchKernelGGL((k_validate_persistent<ZT, AD, W, CM, ONE>), dim3((unsigned)g), dim3(block),
                         coords + rows + ring + zb, st, T, (int)m, s + 8 * off, a + 10 * off, d, dir_all, v, sn, tn,
                         flags + off, c, n_dev, (int)t->opt_helpers,
                         (int)t->opt_xcd_map);
    }
    HIPCHK(hipGetLastError());
  }
  return GBP_OK;
}

template <class ZT>
int launch_validate(gbp_terrain *t, int64_t n, const double *s, const double *a,
                    const uint8_t *dir, int dir_all, int adaptive, uint8_t *valid,
                    double *s_new, double *t_new, uint32_t *flags, uint32_t *counts,
                    hipStream_t st, const int *n_dev = nullptr) {
#define GBP_LVW(AD, W, CM, ONE)                                                              \
  launch_validate_w<ZT, AD, W, CM, ONE>(t, n, s, a, dir, dir_all, valid, s_new, t_new, flags,  \
                                        counts, st, n_dev)
#define GBP_LV(AD, W)                                                                        \
  (cm == 2 ? GBP_LVW(AD, W, 2, true)                                                         \
   : cm == 1 ? GBP_LVW(AD, W, 1, true)                                                       \
             : (one ? GBP_LVW(AD, W, 0, true) : GBP_LVW(AD, W, 0, false)))
  const int64_t w = t->opt_waves;
  // coordinates computed when the affine form is exact; else in LDS only if
  // they fit next to the attempt rows, with room for the W workgroups of 256
  // lanes that share a CU (160 KB per CU); else read from global memory
  const int cm = validate_coord_mode(t, t->opt_kernel == GBP_KERNEL_DIRECT && !n_dev);
  const bool one = t->one_x && t->one_y;  // straight-line brackets (modes 1, 2 imply it)
  // W = 1 and 2 give the same allocation (the kernel needs < 256 VGPRs)
  if (adaptive) return w >= 4 ? GBP_LV(true, 4) : (w == 3 ? GBP_LV(true, 3) : GBP_LV(true, 2));
  return w >= 4 ? GBP_LV(false, 4) : (w == 3 ? GBP_LV(false, 3) : GBP_LV(false, 2));
#undef GBP_LV
#undef GBP_LVW
}

bool valid_handle(const gbp_terrain *t) { return t != nullptr && t->d_z != nullptr; }

// The device guesses a bracket as (int)((v - d[0]) * inv) clamped to [0, n-2]
// (gbp_device.h bracket_guess); this host copy uses the same IEEE operations
// (no contraction in this TU).  The guess is monotone in v, so checking both
// ends of every cell [d[i], d[i+1]) proves |guess - bracket| <= 1 everywhere.
int guess_host(int n, double d0, double inv, double v) {
  const int i = (int)((v - d0) * inv);
  return i < 0 ? 0 : (i > n - 2 ? n - 2 : i);
}

int one_step_exact(const double *d, int n, double inv) {
  if (!(inv > 0) || !std::isfinite(inv)) return 0;
  for (int i = 0; i + 1 < n; i++) {
    if (!(d[i] < d[i + 1])) return 0;  // empty cells: keep the general search
    const int lo = guess_host(n, d[0], inv, d[i]);
    const int hi = guess_host(n, d[0], inv, std::nextafter(d[i + 1], -INFINITY));
    if (lo < i - 1 || hi > i + 1) return 0;
  }
  return 1;
}

// Is d[i] == a + h * (double)(i - base) bit for bit for every i?  Tried with
// base 0 (a = d[0]) and base n-1 (a = d[n-1], grid_map's reversed cell
// centres) and h within a few ulps of the end-to-end and first/last spacings.
// The device evaluates the same expression (no contraction in either TU).
bool affine_exact(const double *d, int n, double a, double h, int base) {
  for (int i = 0; i < n; i++) {
    const double v = a + h * (double)(i - base);
    if (memcmp(&v, &d[i], sizeof v) != 0) return false;
  }
  return true;
}

// The seed of recip_area: 1 / (mean cell area), adopted only if two Newton
// steps from it reproduce 1.0 / (dx * dy) bit for bit for EVERY pair of the
// distinct x and y spacings of the terrain (the device evaluates the same
// FMAs; products and differences are uncontracted in both TUs).  0 = divide.
double verified_rcp_seed(const double *x, int nx, const double *y, int ny) {
  if (nx < 2 || ny < 2) return 0.0;
  auto spacings = [](const double *d, int n) {
    std::vector<double> v;
    for (int i = 0; i + 1 < n; i++) v.push_back(d[i + 1] - d[i]);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end(), [](double a, double b) {
              return memcmp(&a, &b, sizeof a) == 0;
            }), v.end());
    return v;
  };
  const std::vector<double> sx = spacings(x, nx), sy = spacings(y, ny);
  if ((double)sx.size() * (double)sy.size() > 4e6) return 0.0;
  const double seed = 1.0 / (((x[nx - 1] - x[0]) / (double)(nx - 1)) *
                             ((y[ny - 1] - y[0]) / (double)(ny - 1)));
  if (!std::isfinite(seed) || !(seed > 0)) return 0.0;
  for (double dx : sx)
    for (double dy : sy) {
      const double d = dx * dy;
      const double q = 1.0 / d, r = recip_newton(d, seed);
      if (memcmp(&q, &r, sizeof q) != 0) return 0.0;
    }
  return seed;
}

bool affine_fit(const double *d, int n, double *a, double *h, int *base) {
  if (n < 2) return false;
  const double cands[3] = {(d[n - 1] - d[0]) / (double)(n - 1), d[1] - d[0], d[n - 1] - d[n - 2]};
  for (int b = 0; b < 2; b++) {
    const int bs = b ? n - 1 : 0;
    const double av = d[bs];
    for (double c : cands) {
      if (!(c > 0) || !std::isfinite(c)) continue;
      double hv = c;
      for (int k = 0; k < 4; k++) hv = std::nextafter(hv, -INFINITY);
      for (int k = 0; k < 9; k++, hv = std::nextafter(hv, INFINITY)) {
        if (affine_exact(d, n, av, hv, bs)) {
          *a = av;
          *h = hv;
          *base = bs;
          return true;
        }
      }
    }
  }
  return false;
}

// host-pointer entry points: one synchronous staging round trip through the
// handle's workspace on its private stream (used by the C++ adapters that
// re-export the reference API).
struct Stage {
  gbp_terrain *t;
  char *base;
  size_t off = 0;
  template <class T>
  T *take(size_t count) {
    off = (off + 255) & ~(size_t)255;
    T *p = (T *)(base + off);
    off += count * sizeof(T);
    return p;
  }
};
size_t rnd(size_t b) { return (b + 255) & ~(size_t)255; }

}  // namespace

__attribute__((visibility("hidden"))) int gbp_internal_validate_dev_n(
    gbp_terrain *t, int64_t n_max, const int *n_dev, const double *s, const double *a,
    const uint8_t *dir, int dir_all, int adaptive, uint8_t *valid, double *s_new, double *t_new,
    uint32_t *flags, uint32_t *counts, hipStream_t st) {
  if (n_max <= 0) return GBP_OK;
  if (t->storage == GBP_STORAGE_F32)
    return launch_validate<float>(t, n_max, s, a, dir, dir_all, adaptive, valid, s_new, t_new,
                                  flags, counts, st, n_dev);
  return launch_validate<double>(t, n_max, s, a, dir, dir_all, adaptive, valid, s_new, t_new,
                                 flags, counts, st, n_dev);
}

extern "C" {

#ifdef GBP_LOOP_PROF
// per wave: refill, lane setup / helper plan, sample + isValidState, transition
// + helper consumption, outputs + s_new ring, whole loop (cycles); tail
// iterations; iterations
int gbp_loop_prof_read(unsigned long long *out, int n_waves) {
  if (!out || n_waves < 0 || n_waves > 8192) return GBP_E_INVALID_ARG;
  if (hipDeviceSynchronize() != hipSuccess) return GBP_E_HIP;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gbp_loop_prof), sizeof(unsigned long long) * 12 * n_waves) !=
      hipSuccess)
    return GBP_E_HIP;
  return GBP_OK;
}
#endif

int gbp_version(void) { return 200; /* 0.2.0: extend flags, FRAGILE re-decision, trees */ }

const char *gbp_status_string(int status) {
  switch (status) {
    case GBP_OK: return "ok";
    case GBP_E_INVALID_ARG: return "invalid argument";
    case GBP_E_BAD_HANDLE: return "bad handle";
    case GBP_E_ALLOC: return "device allocation failed";
    case GBP_E_HIP: return "HIP runtime error";
    case GBP_E_SHAPE: return "bad shape";
    case GBP_E_NO_DEVICE: return "no HIP device";
    case GBP_E_UNSUPPORTED: return "unsupported";
    default: return "unknown status";
  }
}

int gbp_device_count(int *count) {
  if (!count) return GBP_E_INVALID_ARG;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *count = c;
  return c > 0 ? GBP_OK : GBP_E_NO_DEVICE;
}

int gbp_device_alloc(int device, size_t bytes, void **ptr) {
  if (!ptr) return GBP_E_INVALID_ARG;
  DeviceGuard g(device);
  if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess) return GBP_E_ALLOC;
  return GBP_OK;
}

int gbp_device_free(void *ptr) {
  if (ptr) HIPCHK(hipFree(ptr));
  return GBP_OK;
}

int gbp_memcpy_h2d(void *dst, const void *src, size_t bytes, gbp_stream stream) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return GBP_OK;
}

int gbp_memcpy_d2h(void *dst, const void *src, size_t bytes, gbp_stream stream) {
  HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return GBP_OK;
}

int gbp_stream_synchronize(gbp_stream stream) {
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return GBP_OK;
}

int gbp_terrain_create(int device, int nx, int ny, const double *x, const double *y,
                       const double *z, const double *dx, const double *dy, const double *dz,
                       int storage, gbp_terrain **out) {
  if (!out || !x || !y || !z) return GBP_E_INVALID_ARG;
  *out = nullptr;
  if (nx < 2 || ny < 2) return GBP_E_SHAPE;
  if ((dx == nullptr) != (dy == nullptr) || (dx == nullptr) != (dz == nullptr))
    return GBP_E_INVALID_ARG;
  for (int i = 0; i + 1 < nx; i++)
    if (!(x[i] <= x[i + 1])) return GBP_E_INVALID_ARG;  // ascending (fast_terrain_map.cpp:101-108)
  for (int i = 0; i + 1 < ny; i++)
    if (!(y[i] <= y[i + 1])) return GBP_E_INVALID_ARG;
  const size_t cells = (size_t)nx * ny;
  if (storage == GBP_STORAGE_AUTO) {
    storage = GBP_STORAGE_F32;
    for (size_t i = 0; i < cells; i++) {
      const double v = z[i];
      if (!std::isnan(v) && (double)(float)v != v) {
        storage = GBP_STORAGE_F64;
        break;
      }
    }
  } else if (storage != GBP_STORAGE_F32 && storage != GBP_STORAGE_F64) {
    return GBP_E_INVALID_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GBP_E_NO_DEVICE;
  if (device < 0 || device >= ndev) return GBP_E_INVALID_ARG;
  DeviceGuard g(device);
  gbp_terrain *t = new (std::nothrow) gbp_terrain();
  if (!t) return GBP_E_ALLOC;
  t->device = device;
  t->nx = nx;
  t->ny = ny;
  t->storage = storage;
  t->bounds[0] = x[0];
  t->bounds[1] = x[nx - 1];
  t->bounds[2] = y[0];
  t->bounds[3] = y[ny - 1];
  t->xNm = x[nx - 2];
  t->yNm = y[ny - 2];
  t->inv_hx = (x[nx - 1] > x[0]) ? (double)(nx - 1) / (x[nx - 1] - x[0]) : 0.0;
  t->inv_hy = (y[ny - 1] > y[0]) ? (double)(ny - 1) / (y[ny - 1] - y[0]) : 0.0;
  t->one_x = one_step_exact(x, nx, t->inv_hx);
  t->one_y = one_step_exact(y, ny, t->inv_hy);
  t->affine = affine_fit(x, nx, &t->ax, &t->hx, &t->bx) && affine_fit(y, ny, &t->ay, &t->hy, &t->by);
  t->rcp_seed = verified_rcp_seed(x, nx, y, ny);
  t->host.nx = nx;
  t->host.ny = ny;
  t->host.x.assign(x, x + nx);
  t->host.y.assign(y, y + ny);
  t->host.z.resize(cells);
  for (size_t i = 0; i < cells; i++)  // exactly what the device holds
    t->host.z[i] = storage == GBP_STORAGE_F32 ? (double)(float)z[i] : z[i];
  (void)hipDeviceGetAttribute(&t->num_cus, hipDeviceAttributeMultiprocessorCount, device);
  if (t->num_cus <= 0) t->num_cus = 256;
  int rc = GBP_OK;
  auto fail = [&](int code) {
    gbp_terrain_destroy(t);
    return code;
  };
  if (hipMalloc((void **)&t->d_x, sizeof(double) * nx) != hipSuccess) return fail(GBP_E_ALLOC);
  if (hipMalloc((void **)&t->d_y, sizeof(double) * ny) != hipSuccess) return fail(GBP_E_ALLOC);
  if (hipMemcpy(t->d_x, x, sizeof(double) * nx, hipMemcpyHostToDevice) != hipSuccess)
    return fail(GBP_E_HIP);
  if (hipMemcpy(t->d_y, y, sizeof(double) * ny, hipMemcpyHostToDevice) != hipSuccess)
    return fail(GBP_E_HIP);
  // heights as x-pairs (gbp_device.h TerrainView)
  const size_t zcount = 2 * ((size_t)nx - 1) * (size_t)ny;
  auto zsrc = [&](size_t k) {
    const size_t c = k >> 1, ix = c / (size_t)ny, iy = c % (size_t)ny;
    return z[(ix + (k & 1)) * (size_t)ny + iy];
  };
  if (storage == GBP_STORAGE_F32) {
    std::vector<float> zf(zcount);
    for (size_t i = 0; i < zcount; i++) zf[i] = (float)zsrc(i);
    if (hipMalloc(&t->d_z, sizeof(float) * zcount) != hipSuccess) return fail(GBP_E_ALLOC);
    if (hipMemcpy(t->d_z, zf.data(), sizeof(float) * zcount, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GBP_E_HIP);
  } else {
    std::vector<double> zd(zcount);
    for (size_t i = 0; i < zcount; i++) zd[i] = zsrc(i);
    if (hipMalloc(&t->d_z, sizeof(double) * zcount) != hipSuccess) return fail(GBP_E_ALLOC);
    if (hipMemcpy(t->d_z, zd.data(), sizeof(double) * zcount, hipMemcpyHostToDevice) != hipSuccess)
      return fail(GBP_E_HIP);
  }
  if (dx) {
    const double *src[3] = {dx, dy, dz};
    double **dst[3] = {&t->d_dx, &t->d_dy, &t->d_dz};
    for (int k = 0; k < 3; k++) {
      if (hipMalloc((void **)dst[k], sizeof(double) * cells) != hipSuccess)
        return fail(GBP_E_ALLOC);
      if (hipMemcpy(*dst[k], src[k], sizeof(double) * cells, hipMemcpyHostToDevice) != hipSuccess)
        return fail(GBP_E_HIP);
    }
  }
  {
    int lm = 0;
    if (hipDeviceGetAttribute(&lm, hipDeviceAttributeMaxSharedMemoryPerBlock, device) ==
            hipSuccess && lm > 0)
      t->lds_max = (size_t)lm;
  }
  if (hipStreamCreateWithFlags(&t->host_stream, hipStreamNonBlocking) != hipSuccess)
    return fail(GBP_E_HIP);
  (void)gbp_internal_la_stream(device, t->num_cus);  // ahead of any planner's clock
  (void)rc;
  *out = t;
  return GBP_OK;
}

int gbp_terrain_destroy(gbp_terrain *t) {
  if (!t) return GBP_E_BAD_HANDLE;
  DeviceGuard g(t->device);
  if (t->host_stream) (void)hipStreamSynchronize(t->host_stream);
  (void)hipDeviceSynchronize();  // cand_ws may be in use on any caller stream
  void *ptrs[] = {t->d_x, t->d_y, t->d_z, t->d_dx, t->d_dy, t->d_dz, t->ws};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (auto &w : t->cand_ws)
    if (w.ptr) (void)hipFree(w.ptr);
  if (t->host_stream) (void)hipStreamDestroy(t->host_stream);
  delete t;
  return GBP_OK;
}

int gbp_terrain_info(const gbp_terrain *t, int *nx, int *ny, int *storage, double bounds[4],
                     int *device) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (nx) *nx = t->nx;
  if (ny) *ny = t->ny;
  if (storage) *storage = t->storage;
  if (bounds) memcpy(bounds, t->bounds, sizeof t->bounds);
  if (device) *device = t->device;
  return GBP_OK;
}

int gbp_terrain_set_option(gbp_terrain *t, int key, int64_t value) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  switch (key) {
    case GBP_OPT_KERNEL:
      if (value != GBP_KERNEL_DIRECT && value != GBP_KERNEL_PERSISTENT) return GBP_E_INVALID_ARG;
      t->opt_kernel = value;
      return GBP_OK;
    case GBP_OPT_BLOCK:
      if (value < 64 || value > 512 || value % 64) return GBP_E_INVALID_ARG;
      t->opt_block = value;
      return GBP_OK;
    case GBP_OPT_WAVES:
      if (value < 1 || value > 4) return GBP_E_INVALID_ARG;
      t->opt_waves = value;
      return GBP_OK;
    case GBP_OPT_LDS_COORDS:
      t->opt_lds_coords = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_HELPERS:
      t->opt_helpers = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_AFFINE_COORDS:
      t->opt_affine = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_XCD_MAP:
      t->opt_xcd_map = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_FAST_RCP:
      t->opt_fast_rcp = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_NN_STATS:
      t->opt_nn_stats = value ? 1 : 0;
      return GBP_OK;
    case GBP_OPT_FRAGILE_EPS:  // in 1e-15 units; never below the default margin
      if (value < 1000 || value > 1000000000000000LL) return GBP_E_INVALID_ARG;
      t->fragile_eps = (double)value * 1e-15;
      return GBP_OK;
    default:
      return GBP_E_INVALID_ARG;
  }
}

int gbp_terrain_get_option(const gbp_terrain *t, int key, int64_t *value) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (!value) return GBP_E_INVALID_ARG;
  switch (key) {
    case GBP_OPT_KERNEL: *value = t->opt_kernel; return GBP_OK;
    case GBP_OPT_BLOCK: *value = t->opt_block; return GBP_OK;
    case GBP_OPT_WAVES: *value = t->opt_waves; return GBP_OK;
    case GBP_OPT_LDS_COORDS: *value = t->opt_lds_coords; return GBP_OK;
    case GBP_OPT_HELPERS: *value = t->opt_helpers; return GBP_OK;
    case GBP_OPT_AFFINE_COORDS: *value = t->opt_affine; return GBP_OK;
    case GBP_OPT_XCD_MAP: *value = t->opt_xcd_map; return GBP_OK;
    case GBP_OPT_FAST_RCP: *value = t->opt_fast_rcp ? (t->rcp_seed != 0.0 ? 1 : 0) : 0; return GBP_OK;
    case GBP_OPT_NN_STATS: *value = t->opt_nn_stats; return GBP_OK;
    case GBP_OPT_FRAGILE_EPS: *value = (int64_t)std::llround(t->fragile_eps * 1e15); return GBP_OK;
    case GBP_OPT_COORD_MODE:  // what the validate kernel of the current options uses
      *value = validate_coord_mode(t, t->opt_kernel == GBP_KERNEL_DIRECT);
      return GBP_OK;
    default: return GBP_E_INVALID_ARG;
  }
}

// ---- K1 --------------------------------------------------------------------
int gbp_height_batch_dev(gbp_terrain *t, int64_t n, const double *xy, double *height,
                         uint8_t *is_nan, uint8_t *ood, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && !xy)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  if (((uintptr_t)xy) % 16) return GBP_E_INVALID_ARG;  // xy is read as double2
  const size_t cbytes = stage_bytes(t->nx, t->ny);
  const bool lds = t->opt_lds_coords && cbytes <= t->lds_max;
  // enough workgroups to cover the LDS staging cost many times over
  const unsigned grid = grid_for(n, 256, t->num_cus * 8);
  const double2 *p = (const double2 *)xy;
  hipStream_t st = (hipStream_t)stream;
  const int cm = coord_mode(t, lds);
#define GBP_K1(ZT, CM)                                                                      \
  hipLaunchKernelGGL((k_height<ZT, CM>), dim3(grid), dim3(256), CM == 1 ? cbytes : 0, st, \
                     view<ZT>(t), n, p, height, is_nan, ood)
  if (t->storage == GBP_STORAGE_F32) {
    if (cm == 2) GBP_K1(float, 2);
    else if (cm == 1) GBP_K1(float, 1);
    else GBP_K1(float, 0);
  } else {
    if (cm == 2) GBP_K1(double, 2);
    else if (cm == 1) GBP_K1(double, 1);
    else GBP_K1(double, 0);
  }
#undef GBP_K1
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_normal_batch_dev(gbp_terrain *t, int64_t n, const double *xy, double *normal,
                         uint8_t *ood, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!xy || !normal))) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  const unsigned grid = grid_for(n, 256, t->num_cus * 16);
  if (t->storage == GBP_STORAGE_F32)
    hipLaunchKernelGGL(k_normal<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<float>(t), n, xy, normal, ood);
  else
    hipLaunchKernelGGL(k_normal<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<double>(t), n, xy, normal, ood);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_valid_states_dev(gbp_terrain *t, int64_t n, const double *states, const uint8_t *phase,
                         int phase_all, uint8_t *valid, uint32_t *flags, uint32_t *counts,
                         gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && !states)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  const unsigned grid = grid_for(n, 256, t->num_cus * 16);
  if (t->storage == GBP_STORAGE_F32)
    hipLaunchKernelGGL(k_valid_states<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<float>(t), n, states, phase, phase_all, valid, flags, counts);
  else
    hipLaunchKernelGGL(k_valid_states<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<double>(t), n, states, phase, phase_all, valid, flags, counts);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

// ---- K2: the hot path ---------------------------------------------------------
int gbp_validate_pairs_dev(gbp_terrain *t, int64_t n, const double *s, const double *a,
                           const uint8_t *direction, int direction_all, int adaptive,
                           uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                           uint32_t *counts, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!s || !a || !flags))) return GBP_E_INVALID_ARG;
  if (!direction && direction_all != GBP_FORWARD && direction_all != GBP_REVERSE)
    return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  if (t->storage == GBP_STORAGE_F32)
    return launch_validate<float>(t, n, s, a, direction, direction_all, adaptive, valid, s_new,
                                  t_new, flags, counts, (hipStream_t)stream);
  return launch_validate<double>(t, n, s, a, direction, direction_all, adaptive, valid, s_new,
                                 t_new, flags, counts, (hipStream_t)stream);
}

// ---- K3 ---------------------------------------------------------------------
namespace {
int launch_sample_states(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                         int64_t index_base, int require_phase, int max_tries, double *states,
                         int32_t *tries, const gbp_sampling &cfg, const DirPair &dp,
                         gbp_stream stream) {
  DeviceGuard g(t->device);
  const unsigned grid = grid_for(n, 256, t->num_cus * 16);
  if (t->storage == GBP_STORAGE_F32)
    hipLaunchKernelGGL(k_sample_states<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<float>(t), n, seed, stream_id, index_base, require_phase, max_tries,
                       states, tries, cfg, dp);
  else
    hipLaunchKernelGGL(k_sample_states<double>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       view<double>(t), n, seed, stream_id, index_base, require_phase, max_tries,
                       states, tries, cfg, dp);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

bool sampling_ok(const gbp_sampling &c) {
  return !(c.state_flag && std::isnan(c.state_p)) && !(c.action_flag && std::isnan(c.action_p));
}
}  // namespace

int gbp_sample_states_dev(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                          int64_t index_base, int require_phase, int max_tries, double *states,
                          int32_t *tries, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && !states)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  return launch_sample_states(t, n, seed, stream_id, index_base, require_phase, max_tries, states,
                              tries, gbp_sampling{}, DirPair{}, stream);
}

int gbp_terrain_set_sampling(gbp_terrain *t, const gbp_sampling *cfg) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (cfg && !sampling_ok(*cfg)) return GBP_E_INVALID_ARG;
  t->sampling = cfg ? *cfg : gbp_sampling{};
  return GBP_OK;
}

int gbp_terrain_get_sampling(const gbp_terrain *t, gbp_sampling *cfg) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (!cfg) return GBP_E_INVALID_ARG;
  *cfg = t->sampling;
  return GBP_OK;
}

int gbp_sample_states_dir_dev(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                              int64_t index_base, const gbp_sampling *cfg, const double *s_from,
                              const double *s_to, double *states, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!states || !s_from || !s_to))) return GBP_E_INVALID_ARG;
  if (cfg && !sampling_ok(*cfg)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DirPair dp;
  memcpy(dp.from, s_from, sizeof dp.from);
  memcpy(dp.to, s_to, sizeof dp.to);
  return launch_sample_states(t, n, seed, stream_id, index_base, -1, 1, states, nullptr,
                              cfg ? *cfg : t->sampling, dp, stream);
}

int gbp_sample_actions_dir_dev(gbp_terrain *t, int64_t n, const double *normals, const double *s,
                               const double *s_near, const uint8_t *direction, int direction_all,
                               const gbp_sampling *cfg, uint64_t seed, uint64_t stream_id,
                               int64_t index_base, double *actions, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!normals || !s || !s_near || !actions))) return GBP_E_INVALID_ARG;
  if (!direction && direction_all != GBP_FORWARD && direction_all != GBP_REVERSE)
    return GBP_E_INVALID_ARG;
  if (cfg && !sampling_ok(*cfg)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  hipLaunchKernelGGL(k_sample_actions_dir, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, n, normals, s, s_near, direction, direction_all,
                     cfg ? *cfg : t->sampling, seed, stream_id, index_base, actions);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_sample_actions_dev(int64_t n, const double *normals, uint64_t seed, uint64_t stream_id,
                           int64_t index_base, double *actions, gbp_stream stream) {
  if (n < 0 || (n > 0 && (!normals || !actions))) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  hipLaunchKernelGGL(k_sample_actions, dim3(grid_for(n, 256, 4096)), dim3(256), 0,
                     (hipStream_t)stream, n, normals, seed, stream_id, index_base, actions);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_extend_batch_dev(gbp_terrain *t, int64_t n, const double *s_near, const double *target,
                         const uint8_t *direction, int direction_all, int adaptive, uint64_t seed,
                         int64_t extend_base, int32_t *result, int32_t *chosen, double *s_new,
                         double *a_new, uint32_t *counts, uint32_t *flags, gbp_stream stream) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!s_near || !target || !result || !s_new || !a_new)))
    return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  DeviceGuard g(t->device);
  hipStream_t st = (hipStream_t)stream;
  const int64_t m = n * GBP_NUM_GEN_STATES;
  // candidate workspace: s (8) + a (10) + s_new (8) doubles, flags + counts u32, dir u8
  const size_t need = (size_t)m * (26 * sizeof(double) + 2 * sizeof(uint32_t) + 1) + 256;
  gbp_terrain::StreamWs *w = nullptr;
  for (auto &e : t->cand_ws)
    if (e.stream == st) w = &e;
  if (!w) {
    t->cand_ws.push_back({st, nullptr, 0});
    w = &t->cand_ws.back();
  }
  // a grown workspace may still be read by this stream's earlier launches:
  // ensure_ws frees the old one only after the stream has drained it
  if (w->bytes < need) HIPCHK(hipStreamSynchronize(st));
  int rc = ensure_ws(&w->ptr, &w->bytes, need);
  if (rc) return rc;
  char *p = (char *)w->ptr;
  double *cs = (double *)p; p += (size_t)m * 8 * sizeof(double);
  double *ca = (double *)p; p += (size_t)m * 10 * sizeof(double);
  double *csn = (double *)p; p += (size_t)m * 8 * sizeof(double);
  uint32_t *cf = (uint32_t *)p; p += (size_t)m * sizeof(uint32_t);
  uint32_t *cc = (uint32_t *)p; p += (size_t)m * sizeof(uint32_t);
  uint8_t *cd = (uint8_t *)p;
  const unsigned grid = grid_for(m, 256, t->num_cus * 16);
  if (t->storage == GBP_STORAGE_F32)
    hipLaunchKernelGGL(k_extend_prep<float>, dim3(grid), dim3(256), 0, st, view<float>(t), n,
                       s_near, target, direction, direction_all, seed, extend_base, cs, ca, cd,
                       t->sampling);
  else
    hipLaunchKernelGGL(k_extend_prep<double>, dim3(grid), dim3(256), 0, st, view<double>(t), n,
                       s_near, target, direction, direction_all, seed, extend_base, cs, ca, cd,
                       t->sampling);
  HIPCHK(hipGetLastError());
  rc = gbp_validate_pairs_dev(t, m, cs, ca, cd, 0, adaptive, nullptr, csn, nullptr, cf, cc,
                              stream);
  if (rc) return rc;
  hipLaunchKernelGGL(k_extend_select, dim3(grid_for(n, 256, t->num_cus * 16)), dim3(256), 0, st,
                     n, s_near, target, ca, csn, cf, cc, result, chosen, s_new, a_new, counts, flags);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

// ---- K5 ---------------------------------------------------------------------
int gbp_nearest_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                          const double *vertices, int32_t *index, double *dist,
                          gbp_stream stream) {
  if (n_query < 0 || n_vert < 0 || (n_query > 0 && (!queries || !index))) return GBP_E_INVALID_ARG;
  if (n_vert > 0x7FFFFFFE) return GBP_E_SHAPE;
  if (n_query == 0) return GBP_OK;
  if (n_vert > 0 && !vertices) return GBP_E_INVALID_ARG;
  if (n_query >= 512 && n_vert >= 256) {  // many queries: vertex tiles shared through LDS
    const unsigned grid = (unsigned)((n_query + 255) / 256);
    hipLaunchKernelGGL(k_nearest_tiled, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_query,
                       queries, n_vert, vertices, index, dist);
  } else {  // few queries: one workgroup scans the tree per query
    const unsigned grid = (unsigned)std::min<int64_t>(n_query, 65535);
    hipLaunchKernelGGL(k_nearest, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_query,
                       queries, n_vert, vertices, index, dist);
  }
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_neighbors_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                            const double *vertices, double radius, int max_out, int32_t *out,
                            int32_t *count, gbp_stream stream) {
  if (n_query < 0 || n_vert < 0 || max_out < 0 || (n_query > 0 && (!queries || !count)) ||
      (max_out > 0 && n_query > 0 && !out))
    return GBP_E_INVALID_ARG;
  if (n_vert > 0x7FFFFFFE) return GBP_E_SHAPE;
  if (n_query == 0) return GBP_OK;
  if (n_vert > 0 && !vertices) return GBP_E_INVALID_ARG;
  const unsigned grid = (unsigned)std::min<int64_t>(n_query, 65535);
  hipLaunchKernelGGL(k_neighbors, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_query, queries,
                     n_vert, vertices, radius, max_out, out, count);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_vertex_map_order(int64_t n, int32_t *out) {
  if (n < 0 || n > 0x7FFFFFFF || (n > 0 && !out)) return GBP_E_INVALID_ARG;
  if (n == 0) return GBP_OK;
  const int m = um_epoch(n);
  for (int64_t p = 0; p < n; p++) out[p] = (int32_t)um_key_at(p, n, m);
  return GBP_OK;
}

int gbp_vertex_map_rank(int64_t key, int64_t n, int64_t *rank) {
  if (n < 1 || n > 0x7FFFFFFF || key < 0 || key >= n || !rank) return GBP_E_INVALID_ARG;
  *rank = um_rank(key, n);
  return GBP_OK;
}

int gbp_knn_batch_dev(int64_t n_query, const double *queries, int64_t n_vert,
                      const double *vertices, int n_nearest, int32_t *out, double *dist,
                      gbp_stream stream) {
  if (n_query < 0 || n_vert < 0 || n_nearest < 1 || n_nearest > GBP_KNN_MAX ||
      (n_query > 0 && (!queries || !out)))
    return GBP_E_INVALID_ARG;
  if (n_vert > 0x7FFFFFFE) return GBP_E_SHAPE;
  if (n_query == 0) return GBP_OK;
  if (n_vert > 0 && !vertices) return GBP_E_INVALID_ARG;
  const unsigned grid = (unsigned)std::min<int64_t>((n_query + 3) / 4, 65535);
  hipLaunchKernelGGL(k_knn<false>, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_query, queries,
                     n_vert, vertices, n_nearest, out, dist, nullptr, nullptr, 0.0, 0.0);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

int gbp_knn_yaw_batch_dev(int64_t n_query, const double *queries, const double *query_yaw,
                          int64_t n_vert, const double *vertices, const double *vertex_yaw,
                          double length_weight, double yaw_weight, int n_nearest, int32_t *out,
                          double *dist, gbp_stream stream) {
  if (n_query < 0 || n_vert < 0 || n_nearest < 1 || n_nearest > GBP_KNN_MAX ||
      (n_query > 0 && (!queries || !query_yaw || !out)))
    return GBP_E_INVALID_ARG;
  if (n_vert > 0x7FFFFFFE) return GBP_E_SHAPE;
  if (n_query == 0) return GBP_OK;
  if (n_vert > 0 && (!vertices || !vertex_yaw)) return GBP_E_INVALID_ARG;
  const unsigned grid = (unsigned)std::min<int64_t>((n_query + 3) / 4, 65535);
  hipLaunchKernelGGL(k_knn<true>, dim3(grid), dim3(256), 0, (hipStream_t)stream, n_query, queries,
                     n_vert, vertices, n_nearest, out, dist, query_yaw, vertex_yaw, length_weight,
                     yaw_weight);
  HIPCHK(hipGetLastError());
  return GBP_OK;
}

// ---- host-pointer convenience entry points (see the Stage helper above) ----------

#define H2D(dst, src, bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st))
#define D2H(dst, src, bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st))

int gbp_height_batch_host(gbp_terrain *t, int64_t n, const double *xy, double *height,
                          uint8_t *is_nan, uint8_t *ood) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(16 * n) + rnd(8 * n) + 2 * rnd(n) + 1024);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *dxy = S.take<double>(2 * n), *dh = S.take<double>(n);
  uint8_t *dn = S.take<uint8_t>(n), *dood = S.take<uint8_t>(n);
  H2D(dxy, xy, 16 * n);
  rc = gbp_height_batch_dev(t, n, dxy, dh, dn, dood, st);
  if (rc) return rc;
  if (height) D2H(height, dh, 8 * n);
  if (is_nan) D2H(is_nan, dn, n);
  if (ood) D2H(ood, dood, n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_normal_batch_host(gbp_terrain *t, int64_t n, const double *xy, double *normal,
                          uint8_t *ood) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!normal) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(16 * n) + rnd(24 * n) + rnd(n) + 1024);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *dxy = S.take<double>(2 * n), *dn = S.take<double>(3 * n);
  uint8_t *dood = S.take<uint8_t>(n);
  H2D(dxy, xy, 16 * n);
  rc = gbp_normal_batch_dev(t, n, dxy, dn, dood, st);
  if (rc) return rc;
  D2H(normal, dn, 24 * n);
  if (ood) D2H(ood, dood, n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_valid_states_host(gbp_terrain *t, int64_t n, const double *states, const uint8_t *phase,
                          int phase_all, uint8_t *valid, uint32_t *flags, uint32_t *counts) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes,
                     rnd(64 * n) + 2 * rnd(n) + 2 * rnd(4 * n) + 2048);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *ds = S.take<double>(8 * n);
  uint8_t *dp = S.take<uint8_t>(n), *dv = S.take<uint8_t>(n);
  uint32_t *df = S.take<uint32_t>(n), *dc = S.take<uint32_t>(n);
  H2D(ds, states, 64 * n);
  if (phase) H2D(dp, phase, n);
  rc = gbp_valid_states_dev(t, n, ds, phase ? dp : nullptr, phase_all, dv, df, dc, st);
  if (rc) return rc;
  std::vector<uint32_t> fl(flags ? 0 : n);
  uint32_t *flags_h = flags ? flags : fl.data();
  if (valid) D2H(valid, dv, n);
  D2H(flags_h, df, 4 * n);
  if (counts) D2H(counts, dc, 4 * n);
  HIPCHK(hipStreamSynchronize(st));
  return gbp_resolve_fragile_states_host(t, n, states, phase, phase_all, valid, flags_h, counts,
                                         nullptr);
}

int gbp_validate_pairs_host(gbp_terrain *t, int64_t n, const double *s, const double *a,
                            const uint8_t *direction, int direction_all, int adaptive,
                            uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                            uint32_t *counts) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!s || !a) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes,
                     rnd(64 * n) + rnd(80 * n) + rnd(64 * n) + rnd(8 * n) + 2 * rnd(n) +
                         2 * rnd(4 * n) + 4096);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *ds = S.take<double>(8 * n), *da = S.take<double>(10 * n);
  double *dsn = S.take<double>(8 * n), *dtn = S.take<double>(n);
  uint8_t *dd = S.take<uint8_t>(n), *dv = S.take<uint8_t>(n);
  uint32_t *df = S.take<uint32_t>(n), *dc = S.take<uint32_t>(n);
  H2D(ds, s, 64 * n);
  H2D(da, a, 80 * n);
  if (direction) H2D(dd, direction, n);
  // in/out semantics: untouched outputs keep the caller's contents
  if (s_new) H2D(dsn, s_new, 64 * n);
  if (t_new) H2D(dtn, t_new, 8 * n);
  rc = gbp_validate_pairs_dev(t, n, ds, da, direction ? dd : nullptr, direction_all, adaptive,
                              dv, dsn, dtn, df, dc, st);
  if (rc) return rc;
  std::vector<uint32_t> fl(flags ? 0 : n);
  uint32_t *flags_h = flags ? flags : fl.data();
  // the caller's s_new / t_new: a FRAGILE attempt the host re-decides gets
  // back the caller's contents wherever the host check does not assign them
  std::vector<double> sn0(s_new ? 8 * n : 0), tn0(t_new ? n : 0);
  if (s_new) memcpy(sn0.data(), s_new, 64 * n);
  if (t_new) memcpy(tn0.data(), t_new, 8 * n);
  if (valid) D2H(valid, dv, n);
  if (s_new) D2H(s_new, dsn, 64 * n);
  if (t_new) D2H(t_new, dtn, 8 * n);
  D2H(flags_h, df, 4 * n);
  if (counts) D2H(counts, dc, 4 * n);
  HIPCHK(hipStreamSynchronize(st));
  for (int64_t i = 0; i < n; i++) {
    if (!(flags_h[i] & GBP_F_FRAGILE)) continue;
    if (s_new) memcpy(s_new + 8 * i, sn0.data() + 8 * i, 64);
    if (t_new) t_new[i] = tn0[i];
  }
  return gbp_resolve_fragile_host(t, n, s, a, direction, direction_all, adaptive, valid, s_new,
                                  t_new, flags_h, counts, nullptr);
}

int gbp_extend_batch_host(gbp_terrain *t, int64_t n, const double *s_near, const double *target,
                          const uint8_t *direction, int direction_all, int adaptive,
                          uint64_t seed, int64_t extend_base, int32_t *result, int32_t *chosen,
                          double *s_new, double *a_new, uint32_t *counts, uint32_t *flags) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!s_near || !target || !result || !s_new || !a_new) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes,
                     3 * rnd(64 * n) + rnd(80 * n) + rnd(n) + 4 * rnd(4 * n) + 4096);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *dsn = S.take<double>(8 * n), *dtg = S.take<double>(8 * n);
  double *dnew = S.take<double>(8 * n), *danew = S.take<double>(10 * n);
  uint8_t *dd = S.take<uint8_t>(n);
  int32_t *dr = S.take<int32_t>(n), *dch = S.take<int32_t>(n);
  uint32_t *dc = S.take<uint32_t>(n), *df = S.take<uint32_t>(n);
  H2D(dsn, s_near, 64 * n);
  H2D(dtg, target, 64 * n);
  H2D(dnew, s_new, 64 * n);
  H2D(danew, a_new, 80 * n);
  if (direction) H2D(dd, direction, n);
  rc = gbp_extend_batch_dev(t, n, dsn, dtg, direction ? dd : nullptr, direction_all, adaptive,
                            seed, extend_base, dr, dch, dnew, danew, dc, df, st);
  if (rc) return rc;
  std::vector<int32_t> ch(chosen ? 0 : n);
  std::vector<uint32_t> cnt(counts ? 0 : n), fl(flags ? 0 : n);
  int32_t *chosen_h = chosen ? chosen : ch.data();
  uint32_t *counts_h = counts ? counts : cnt.data();
  uint32_t *flags_h = flags ? flags : fl.data();
  D2H(result, dr, 4 * n);
  D2H(chosen_h, dch, 4 * n);
  D2H(s_new, dnew, 64 * n);
  D2H(a_new, danew, 80 * n);
  D2H(counts_h, dc, 4 * n);
  D2H(flags_h, df, 4 * n);
  HIPCHK(hipStreamSynchronize(st));
  // decisions that hinge on a trig-sensitive margin: re-decided with glibc
  return gbp_extend_resolve_host(t, n, s_near, target, direction, direction_all, adaptive, seed,
                                 extend_base, result, chosen_h, s_new, a_new, counts_h, flags_h,
                                 nullptr);
}

int gbp_sample_states_host(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                           int64_t index_base, int require_phase, int max_tries, double *states,
                           int32_t *tries) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!states) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(64 * n) + rnd(4 * n) + 1024);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *ds = S.take<double>(8 * n);
  int32_t *dt = S.take<int32_t>(n);
  rc = gbp_sample_states_dev(t, n, seed, stream_id, index_base, require_phase, max_tries, ds, dt,
                             st);
  if (rc) return rc;
  D2H(states, ds, 64 * n);
  if (tries) D2H(tries, dt, 4 * n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_sample_states_dir_host(gbp_terrain *t, int64_t n, uint64_t seed, uint64_t stream_id,
                               int64_t index_base, const gbp_sampling *cfg, const double *s_from,
                               const double *s_to, double *states) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!states || !s_from || !s_to) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(64 * n) + 1024);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *ds = S.take<double>(8 * n);
  rc = gbp_sample_states_dir_dev(t, n, seed, stream_id, index_base, cfg, s_from, s_to, ds, st);
  if (rc) return rc;
  D2H(states, ds, 64 * n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_sample_actions_dir_host(gbp_terrain *t, int64_t n, const double *normals, const double *s,
                                const double *s_near, const uint8_t *direction, int direction_all,
                                const gbp_sampling *cfg, uint64_t seed, uint64_t stream_id,
                                int64_t index_base, double *actions) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!normals || !s || !s_near || !actions) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(24 * n) + 2 * rnd(64 * n) + rnd(n) + rnd(80 * n) + 2048);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *dn = S.take<double>(3 * n), *ds = S.take<double>(8 * n), *dsn = S.take<double>(8 * n);
  uint8_t *dd = S.take<uint8_t>(n);
  double *da = S.take<double>(10 * n);
  H2D(dn, normals, 24 * n);
  H2D(ds, s, 64 * n);
  H2D(dsn, s_near, 64 * n);
  if (direction) H2D(dd, direction, n);
  rc = gbp_sample_actions_dir_dev(t, n, dn, ds, dsn, direction ? dd : nullptr, direction_all, cfg,
                                  seed, stream_id, index_base, da, st);
  if (rc) return rc;
  D2H(actions, da, 80 * n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_sample_actions_host(gbp_terrain *t, int64_t n, const double *normals, uint64_t seed,
                            uint64_t stream_id, int64_t index_base, double *actions) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n <= 0) return n == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!normals || !actions) return GBP_E_INVALID_ARG;
  DeviceGuard g(t->device);
  hipStream_t st = t->host_stream;
  int rc = ensure_ws(&t->ws, &t->ws_bytes, rnd(24 * n) + rnd(80 * n) + 1024);
  if (rc) return rc;
  Stage S{t, (char *)t->ws};
  double *dn = S.take<double>(3 * n), *da = S.take<double>(10 * n);
  H2D(dn, normals, 24 * n);
  rc = gbp_sample_actions_dev(n, dn, seed, stream_id, index_base, da, st);
  if (rc) return rc;
  D2H(actions, da, 80 * n);
  HIPCHK(hipStreamSynchronize(st));
  return GBP_OK;
}

int gbp_nearest_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                           const double *vertices, int32_t *index, double *dist) {
  if (n_query <= 0) return n_query == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!queries || !index || (n_vert > 0 && !vertices)) return GBP_E_INVALID_ARG;
  void *buf = nullptr;
  const size_t need = rnd(64 * n_query) + rnd(64 * (n_vert > 0 ? n_vert : 1)) +
                      rnd(4 * n_query) + rnd(8 * n_query) + 1024;
  if (hipMalloc(&buf, need) != hipSuccess) return GBP_E_ALLOC;
  char *p = (char *)buf;
  double *dq = (double *)p; p += rnd(64 * n_query);
  double *dv = (double *)p; p += rnd(64 * (n_vert > 0 ? n_vert : 1));
  int32_t *di = (int32_t *)p; p += rnd(4 * n_query);
  double *dd = (double *)p;
  hipStream_t st = nullptr;
  int rc = GBP_OK;
  if (hipMemcpy(dq, queries, 64 * n_query, hipMemcpyHostToDevice) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && n_vert > 0 &&
      hipMemcpy(dv, vertices, 64 * n_vert, hipMemcpyHostToDevice) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc) rc = gbp_nearest_batch_dev(n_query, dq, n_vert, dv, di, dd, st);
  if (!rc && hipMemcpy(index, di, 4 * n_query, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc && dist && hipMemcpy(dist, dd, 8 * n_query, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_neighbors_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                             const double *vertices, double radius, int max_out, int32_t *out,
                             int32_t *count) {
  if (n_query <= 0) return n_query == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!queries || !count || max_out < 0 || (max_out > 0 && !out) || (n_vert > 0 && !vertices))
    return GBP_E_INVALID_ARG;
  void *buf = nullptr;
  const size_t nout = (size_t)n_query * (size_t)max_out;
  const size_t need = rnd(64 * n_query) + rnd(64 * (n_vert > 0 ? n_vert : 1)) +
                      rnd(4 * (nout > 0 ? nout : 1)) + rnd(4 * n_query) + 1024;
  if (hipMalloc(&buf, need) != hipSuccess) return GBP_E_ALLOC;
  char *p = (char *)buf;
  double *dq = (double *)p; p += rnd(64 * n_query);
  double *dv = (double *)p; p += rnd(64 * (n_vert > 0 ? n_vert : 1));
  int32_t *dout = (int32_t *)p; p += rnd(4 * (nout > 0 ? nout : 1));
  int32_t *dc = (int32_t *)p;
  int rc = GBP_OK;
  if (hipMemcpy(dq, queries, 64 * n_query, hipMemcpyHostToDevice) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && n_vert > 0 &&
      hipMemcpy(dv, vertices, 64 * n_vert, hipMemcpyHostToDevice) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc) rc = gbp_neighbors_batch_dev(n_query, dq, n_vert, dv, radius, max_out, dout, dc, nullptr);
  if (!rc && nout > 0 && hipMemcpy(out, dout, 4 * nout, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc && hipMemcpy(count, dc, 4 * n_query, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_knn_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                       const double *vertices, int n_nearest, int32_t *out, double *dist) {
  if (n_query <= 0) return n_query == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!queries || !out || n_nearest < 1 || n_nearest > GBP_KNN_MAX || (n_vert > 0 && !vertices))
    return GBP_E_INVALID_ARG;
  void *buf = nullptr;
  const size_t nout = (size_t)n_query * (size_t)n_nearest;
  const size_t need = rnd(64 * n_query) + rnd(64 * (n_vert > 0 ? n_vert : 1)) + rnd(4 * nout) +
                      rnd(8 * nout) + 1024;
  if (hipMalloc(&buf, need) != hipSuccess) return GBP_E_ALLOC;
  char *p = (char *)buf;
  double *dq = (double *)p; p += rnd(64 * n_query);
  double *dv = (double *)p; p += rnd(64 * (n_vert > 0 ? n_vert : 1));
  int32_t *dout = (int32_t *)p; p += rnd(4 * nout);
  double *dd = (double *)p;
  int rc = GBP_OK;
  if (hipMemcpy(dq, queries, 64 * n_query, hipMemcpyHostToDevice) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && n_vert > 0 &&
      hipMemcpy(dv, vertices, 64 * n_vert, hipMemcpyHostToDevice) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc) rc = gbp_knn_batch_dev(n_query, dq, n_vert, dv, n_nearest, dout, dd, nullptr);
  if (!rc && hipMemcpy(out, dout, 4 * nout, hipMemcpyDeviceToHost) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && dist && hipMemcpy(dist, dd, 8 * nout, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

int gbp_knn_yaw_batch_host(int64_t n_query, const double *queries, int64_t n_vert,
                           const double *vertices, double length_weight, double yaw_weight,
                           int n_nearest, int32_t *out, double *dist) {
  if (n_query <= 0) return n_query == 0 ? GBP_OK : GBP_E_INVALID_ARG;
  if (!queries || !out || n_nearest < 1 || n_nearest > GBP_KNN_MAX || (n_vert > 0 && !vertices))
    return GBP_E_INVALID_ARG;
  // the yaws with glibc (planning_utils.h:135-136), as the reference forms them
  const int64_t nv = n_vert > 0 ? n_vert : 1;
  std::vector<double> qy((size_t)n_query), vy((size_t)nv, 0.0);
  for (int64_t i = 0; i < n_query; i++) qy[i] = gbp_host_yaw(queries + 8 * i);
  for (int64_t j = 0; j < n_vert; j++) vy[j] = gbp_host_yaw(vertices + 8 * j);
  void *buf = nullptr;
  const size_t nout = (size_t)n_query * (size_t)n_nearest;
  const size_t need = rnd(64 * n_query) + rnd(64 * nv) + rnd(8 * n_query) + rnd(8 * nv) +
                      rnd(4 * nout) + rnd(8 * nout) + 1024;
  if (hipMalloc(&buf, need) != hipSuccess) return GBP_E_ALLOC;
  char *p = (char *)buf;
  double *dq = (double *)p; p += rnd(64 * n_query);
  double *dv = (double *)p; p += rnd(64 * nv);
  double *dqy = (double *)p; p += rnd(8 * n_query);
  double *dvy = (double *)p; p += rnd(8 * nv);
  int32_t *dout = (int32_t *)p; p += rnd(4 * nout);
  double *dd = (double *)p;
  int rc = GBP_OK;
  if (hipMemcpy(dq, queries, 64 * n_query, hipMemcpyHostToDevice) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && hipMemcpy(dqy, qy.data(), 8 * n_query, hipMemcpyHostToDevice) != hipSuccess)
    rc = GBP_E_HIP;
  if (!rc && n_vert > 0 &&
      (hipMemcpy(dv, vertices, 64 * n_vert, hipMemcpyHostToDevice) != hipSuccess ||
       hipMemcpy(dvy, vy.data(), 8 * n_vert, hipMemcpyHostToDevice) != hipSuccess))
    rc = GBP_E_HIP;
  if (!rc)
    rc = gbp_knn_yaw_batch_dev(n_query, dq, dqy, n_vert, dv, dvy, length_weight, yaw_weight,
                               n_nearest, dout, dd, nullptr);
  if (!rc && hipMemcpy(out, dout, 4 * nout, hipMemcpyDeviceToHost) != hipSuccess) rc = GBP_E_HIP;
  if (!rc && dist && hipMemcpy(dist, dd, 8 * nout, hipMemcpyDeviceToHost) != hipSuccess)
    rc = GBP_E_HIP;
  (void)hipFree(buf);
  return rc;
}

// ---- FRAGILE attempts: the glibc re-decision (host/gbp_host_check.cpp) ------------
int gbp_resolve_fragile_host(gbp_terrain *t, int64_t n, const double *s, const double *a,
                             const uint8_t *direction, int direction_all, int adaptive,
                             uint8_t *valid, double *s_new, double *t_new, uint32_t *flags,
                             uint32_t *counts, int64_t *n_resolved) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!s || !a || !flags))) return GBP_E_INVALID_ARG;
  if (!direction && direction_all != GBP_FORWARD && direction_all != GBP_REVERSE)
    return GBP_E_INVALID_ARG;
  int64_t k = 0;
  for (int64_t i = 0; i < n; i++) {
    if (!(flags[i] & GBP_F_FRAGILE)) continue;
    double sn[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tn = 0;
    uint32_t f = 0, c = 0;
    const int d = direction ? direction[i] : direction_all;
    const bool v = gbp_host::pair_check(t->host, s + 8 * i, a + 10 * i, d, adaptive, sn, &tn, &f, &c);
    if (valid) valid[i] = v ? 1 : 0;
    if (s_new && (f & GBP_F_SNEW_SET)) memcpy(s_new + 8 * i, sn, sizeof sn);
    if (t_new && (f & GBP_F_TNEW_SET)) t_new[i] = tn;
    flags[i] = f | GBP_F_RESOLVED;
    if (counts) counts[i] = c;
    k++;
  }
  if (n_resolved) *n_resolved = k;
  return GBP_OK;
}

int gbp_resolve_fragile_states_host(gbp_terrain *t, int64_t n, const double *states,
                                    const uint8_t *phase, int phase_all, uint8_t *valid,
                                    uint32_t *flags, uint32_t *counts, int64_t *n_resolved) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!states || !flags))) return GBP_E_INVALID_ARG;
  int64_t k = 0;
  for (int64_t i = 0; i < n; i++) {
    if (!(flags[i] & GBP_F_FRAGILE)) continue;
    gbp_host::Acc acc;
    const bool v = gbp_host::is_valid_state(t->host, states + 8 * i, phase ? phase[i] : phase_all, acc);
    if (valid) valid[i] = v ? 1 : 0;
    flags[i] = acc.flags | (v ? GBP_F_VALID : 0u) | GBP_F_RESOLVED;
    if (counts) counts[i] = (acc.G & 0xFFFFu) | (acc.V << 16);
    k++;
  }
  if (n_resolved) *n_resolved = k;
  return GBP_OK;
}

// RRTClass::newConfig + extend's acceptance (rrt.cpp:20-70, :84-101) on the
// host for every extend whose executed candidates include a FRAGILE one.  The
// candidate actions are regenerated on the device from the same Philox
// stream (the engine's candidate sampler, not a host libm), then checked in
// index order with the glibc pair check.
int gbp_extend_resolve_host(gbp_terrain *t, int64_t n, const double *s_near, const double *target,
                            const uint8_t *direction, int direction_all, int adaptive,
                            uint64_t seed, int64_t extend_base, int32_t *result, int32_t *chosen,
                            double *s_new, double *a_new, uint32_t *counts, uint32_t *flags,
                            int64_t *n_resolved) {
  if (!valid_handle(t)) return GBP_E_BAD_HANDLE;
  if (n < 0 || (n > 0 && (!s_near || !target || !result || !s_new || !a_new || !flags)))
    return GBP_E_INVALID_ARG;
  int64_t k = 0;
  for (int64_t i = 0; i < n; i++) {
    if (!(flags[i] & GBP_F_FRAGILE)) continue;
    const double *tg = target + 8 * i, *sn0 = s_near + 8 * i;
    double nrm[3 * GBP_NUM_GEN_STATES], act[10 * GBP_NUM_GEN_STATES];
    double tgs[8 * GBP_NUM_GEN_STATES], sns[8 * GBP_NUM_GEN_STATES];
    int rc = gbp_normal_batch_host(t, 1, tg, nrm, nullptr);  // rrt.cpp:25 (k_extend_prep)
    if (rc) return rc;
    for (int j = 0; j < GBP_NUM_GEN_STATES; j++) {
      if (j) memcpy(nrm + 3 * j, nrm, 3 * sizeof(double));
      memcpy(tgs + 8 * j, tg, 8 * sizeof(double));
      memcpy(sns + 8 * j, sn0, 8 * sizeof(double));
    }
    const int d = direction ? direction[i] : direction_all;
    // the candidates k_extend_prep drew (the handle's sampling configuration)
    rc = gbp_sample_actions_dir_host(t, GBP_NUM_GEN_STATES, nrm, tgs, sns, nullptr, d, nullptr,
                                     seed, EXTEND_STREAM, (extend_base + i) * 8, act);
    if (rc) return rc;
    const double best0 = gbp_host::state_distance(sn0, tg);
    double best = best0, s_test[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_test = 0;
    uint32_t G = 0, V = 0, ef = 0;
    int found = -1;
    for (int j = 0; j < GBP_NUM_GEN_STATES; j++) {  // rrt.cpp:36-50
      uint32_t f = 0, c = 0;
      const bool v = gbp_host::pair_check(t->host, sn0, act + 10 * j, d, adaptive, s_test, &t_test, &f, &c);
      G += GBP_COUNT_G(c);
      V += GBP_COUNT_V(c);
      ef |= f & (GBP_F_VALID | GBP_F_OOD | GBP_F_NAN | GBP_F_LIMIT);
      if (v) {
        found = j;
        break;
      }
    }
    if (found >= 0) {  // rrt.cpp:55-61
      const double cur = gbp_host::state_distance(s_test, tg);
      if (cur < best) {
        best = cur;
        memcpy(s_new + 8 * i, s_test, sizeof s_test);
        memcpy(a_new + 10 * i, act + 10 * found, 10 * sizeof(double));
      }
    }
    // rrt.cpp:65-68 / :84-101
    result[i] = best == best0 ? GBP_TRAPPED
                              : (gbp_host::state_distance(s_new + 8 * i, tg) <= GOAL_BOUNDS
                                     ? GBP_REACHED
                                     : GBP_ADVANCED);
    if (chosen) chosen[i] = found;
    if (counts) counts[i] = (G & 0xFFFFu) | (V << 16);
    flags[i] = ef | GBP_F_RESOLVED;
    k++;
  }
  if (n_resolved) *n_resolved = k;
  return GBP_OK;
}

}  // extern "C"
