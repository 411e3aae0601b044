// gbp_lane.h — the reference's pair-check control flow as a per-sample state
// machine (planning_utils.cpp:651-876): one Lane holds one attempt's loop
// state; sample_state() forms the state the reference evaluates at a sample,
// transition() applies the reference's control flow to one isValidState
// result.  Used by the persistent validate kernel (lanes re-packed per
// sample) and by the planner's wave-per-connect kernel (the 64 lanes of a
// wave evaluate one attempt's next samples together).
#pragma once
#pragma clang fp contract(off)

#include "gbp_device.h"

namespace gbp {

enum : int {
  ST_IDLE = 0,
  ST_FWD_STANCE = GBP_STAGE_FWD_STANCE,
  ST_FWD_FLIGHT = GBP_STAGE_FWD_FLIGHT,
  ST_FWD_LAND = GBP_STAGE_FWD_LAND,
  ST_REV_FLIGHT = GBP_STAGE_REV_FLIGHT,
  ST_REV_STANCE = GBP_STAGE_REV_STANCE,
  ST_REV_START = GBP_STAGE_REV_START,
};
// deferred s_new: recomputed once at the end from (kind, param) — the same
// closed form and the same operands the reference assigned it from
enum : int { SN_NONE = 0, SN_STANCE_S = 1, SN_FLIGHT_B = 2, SN_STANCE_REV_B = 3 };

// Each lane's attempt (s[8], a[10]) lives in LDS, not in VGPRs: a row of
// SA_ROW doubles per thread (odd stride: the 64 lanes' 8-byte reads hit
// distinct bank pairs).  Freed registers keep the state check's in-flight
// lookups out of scratch; tail helpers read their owner's row directly.
constexpr int SA_ROW = 19;

struct Lane {
  double *s, *a;             // this lane's LDS row: input state and action (the
                             // take-off state of the flight / reverse-stance
                             // phases is recomputed per sample)
  double t, ts, tpre;        // sample time, adaptive step, last success time
  double snew_p, tnew;
  int stage, snew_kind;
  uint32_t f, tnew_set;
  Acc acc;
  int idx;
};

// enter a stage, skipping loops whose condition is false on entry
__device__ __forceinline__ void enter_stage(Lane &L, int st) {
  for (;;) {
    L.f = (L.f & ~GBP_F_STAGE_MASK) | stage_bits((uint32_t)st);
    L.stage = st;
    L.ts = KINEMATICS_RES;
    L.tpre = 0;
    switch (st) {
      case ST_FWD_STANCE:  // planning_utils.cpp:718
        L.t = 0;
        if (L.t <= L.a[6]) return;
        st = ST_FWD_FLIGHT;
        break;
      case ST_FWD_FLIGHT:  // :732-735
        L.t = 0;
        if (L.t < L.a[7]) return;
        st = ST_FWD_LAND;
        break;
      case ST_REV_FLIGHT:  // :842
        L.t = 0;
        if (L.t < L.a[7]) return;
        st = ST_REV_STANCE;
        break;
      case ST_REV_STANCE:  // :849-852
        L.t = L.a[6];
        if (L.t >= 0) return;
        st = ST_REV_START;
        break;
      default:  // FWD_LAND, REV_START: exactly one sample
        return;
    }
  }
}

// the state the reference evaluates at time t of a stage (the take-off state
// s_takeoff of :732 / :849 recomputed from (s, a): the same closed form and
// operands, hence the same bits).
//
// Every stage but the reverse flight needs one stance closed form
// (applyStance at t or t_s, or applyStanceReverse at t) and each of those has
// eight divisions by 6 t_s / 2 t_s.  Lanes of one wave sit in different
// stages, so the numerators are formed per stage (divergent, cheap), the
// eight divisions run ONCE for the whole wave (converged), and the stage's
// own sums finish the state — the expression trees of apply_stance /
// apply_stance_reverse (gbp_device.h), split at the quotient.
__device__ __forceinline__ void sample_state(const double *s_in, const double *a_in, int stage,
                                             double t, double *o) {
  double sv[8], a[10];
#pragma unroll
  for (int k = 0; k < 8; k++) sv[k] = s_in[k];
#pragma unroll
  for (int k = 0; k < 10; k++) a[k] = a_in[k];
  if (stage == ST_REV_FLIGHT) {  // applyFlight(s, -t)
    apply_flight(sv, -t, o);
    return;
  }
  const bool rev = (stage == ST_REV_STANCE || stage == ST_REV_START);
  const double t_s = a[6];
  double b[8];  // the state the stance form starts from
  double tt;    // its time argument
  if (rev) {
    apply_flight(sv, -a[7], b);  // s_to = applyFlight(s, -t_f)
    tt = t;
  } else {
#pragma unroll
    for (int k = 0; k < 8; k++) b[k] = sv[k];
    tt = (stage == ST_FWD_STANCE) ? t : t_s;
  }
  // numerators: applyStance (a_to - a_td) * (t*t*t) and (a_to - a_td) * t * t;
  // applyStanceReverse (a_to - a_td) * d3 and (a_to - a_td) * d2
  const double d1 = t_s - tt, d2 = t_s * t_s - tt * tt, d3 = t_s * t_s * t_s - tt * tt * tt;
  const double t3 = tt * tt * tt;
  const int ax[4] = {0, 1, 2, 8}, ao[4] = {3, 4, 5, 9};
  double n6[4], n2[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const double da = a[ao[k]] - a[ax[k]];
    n6[k] = rev ? da * d3 : da * t3;
    n2[k] = rev ? da * d2 : da * tt * tt;
  }
  // the eight divisions, once per wave
  double q6[4], q2[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    q6[k] = n6[k] / (6.0 * t_s);
    q2[k] = n2[k] / (2.0 * t_s);
  }
  if (rev) {  // planning_utils.cpp:348-364
    const double cx = b[3] - a[0] * t_s - 0.5 * (a[3] - a[0]) * t_s;
    const double cy = b[4] - a[1] * t_s - 0.5 * (a[4] - a[1]) * t_s;
    const double cz = b[5] - a[2] * t_s - 0.5 * (a[5] - a[2]) * t_s;
    const double cp = b[7] - a[8] * t_s - 0.5 * (a[9] - a[8]) * t_s;
    o[0] = b[0] - cx * d1 - 0.5 * a[0] * d2 - q6[0];
    o[1] = b[1] - cy * d1 - 0.5 * a[1] * d2 - q6[1];
    o[2] = b[2] - cz * d1 - 0.5 * a[2] * d2 - q6[2];
    o[3] = b[3] - a[0] * d1 - q2[0];
    o[4] = b[4] - a[1] * d1 - q2[1];
    o[5] = b[5] - a[2] * d1 - q2[2];
    // (the reference assigns [7] before [6]; the values are independent.  The
    // stores follow the forward branch's order so that the compiler's sinking
    // of the two branches' last stores meets one address, not a phi of two,
    // which would index the caller's state array dynamically: scratch)
    o[6] = b[6] - cp * d1 - 0.5 * a[8] * d2 - q6[3];
    o[7] = b[7] - a[8] * d1 - q2[3];
    return;
  }
  // planning_utils.cpp:262-271
  double c[8];
  c[0] = b[0] + b[3] * tt + 0.5 * a[0] * tt * tt + q6[0];
  c[1] = b[1] + b[4] * tt + 0.5 * a[1] * tt * tt + q6[1];
  c[2] = b[2] + b[5] * tt + 0.5 * a[2] * tt * tt + q6[2];
  c[3] = b[3] + a[0] * tt + q2[0];
  c[4] = b[4] + a[1] * tt + q2[1];
  c[5] = b[5] + a[2] * tt + q2[2];
  c[6] = b[6] + b[7] * tt + 0.5 * a[8] * tt * tt + q6[3];
  c[7] = b[7] + a[8] * tt + q2[3];
  if (stage == ST_FWD_STANCE) {
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = c[k];
  } else {  // ST_FWD_FLIGHT / ST_FWD_LAND: applyFlight(applyStance(s, a), t)
    apply_flight(c, t, o);
  }
}

template <bool ADAPTIVE>
__device__ __forceinline__ bool small_step(double ts) {
  return !ADAPTIVE || (KINEMATICS_RES - 0.01 <= ts && ts <= KINEMATICS_RES + 0.01);
}

__device__ __forceinline__ int stage_phase(int st) {
  return (st == ST_FWD_FLIGHT || st == ST_REV_FLIGHT) ? GBP_FLIGHT : GBP_STANCE;
}
// the sample time of a lane's current stage
__device__ __forceinline__ double stage_time(const Lane &L) {
  return L.stage == ST_FWD_LAND ? L.a[7] : (L.stage == ST_REV_START ? 0.0 : L.t);
}

// Advance (st, t, ts) the way a SUCCESSFUL sample does in transition() below,
// across stage boundaries (enter_stage's resets and skips included): the
// stage and time of the attempt's next sample if the current one passes.
// false: a passing sample decides the attempt (FWD_LAND, REV_START).  On the
// success path the sample sequence is deterministic, so tail helpers use this
// to evaluate an owner's future samples, in the same stage or a later one.
template <bool ADAPTIVE>
__device__ __forceinline__ bool advance_on_success(int &st, const double *a, double &t, double &ts) {
  switch (st) {
    case ST_FWD_STANCE:  // transition :218-230
      if (ADAPTIVE) { ts += KINEMATICS_RES; t += ts; } else { t += KINEMATICS_RES; }
      if (t <= a[6]) return true;
      st = ST_FWD_FLIGHT;  // enter_stage(FWD_FLIGHT)
      t = 0;
      ts = KINEMATICS_RES;
      if (t < a[7]) return true;
      st = ST_FWD_LAND;
      return true;
    case ST_FWD_FLIGHT:
      if (ADAPTIVE) { ts += KINEMATICS_RES; t += ts; } else { t += KINEMATICS_RES; }
      if (t < a[7]) return true;
      st = ST_FWD_LAND;
      return true;
    case ST_REV_FLIGHT:
      if (ADAPTIVE) { ts += KINEMATICS_RES; t += ts; } else { t += KINEMATICS_RES; }
      if (t < a[7]) return true;
      st = ST_REV_STANCE;  // enter_stage(REV_STANCE)
      t = a[6];
      ts = KINEMATICS_RES;
      if (t >= 0) return true;
      st = ST_REV_START;
      return true;
    case ST_REV_STANCE:
      if (ADAPTIVE) { ts += KINEMATICS_RES; t -= ts; } else { t -= KINEMATICS_RES; }
      if (t >= 0) return true;
      st = ST_REV_START;
      return true;
    default:
      return false;
  }
}

// the sample time of stage st at loop time t (stage_time for a helper's copy)
__device__ __forceinline__ double sample_time(int st, const double *a, double t) {
  return st == ST_FWD_LAND ? a[7] : (st == ST_REV_START ? 0.0 : t);
}

// the reference's control flow after one isValidState result `ok` of the
// lane's current stage; returns true when the pair is decided
template <bool ADAPTIVE>
__device__ __forceinline__ bool transition(Lane &L, bool ok) {
  const double step = ADAPTIVE ? 0.0 : KINEMATICS_RES;  // plain loops: constant increment
  switch (L.stage) {
    case ST_FWD_STANCE:
      if (!ok) {
        if (small_step<ADAPTIVE>(L.ts)) {
          L.snew_kind = SN_STANCE_S;
          L.snew_p = (1.0 - BACKUP_RATIO) * L.t;
          return true;
        }
        L.ts = KINEMATICS_RES;
        L.t = L.tpre;
        L.t += L.ts;
      } else {
        L.snew_kind = SN_STANCE_S;
        L.snew_p = L.t;
        L.tnew = L.t;
        L.tnew_set = 1;
        if (ADAPTIVE) {
          L.ts += KINEMATICS_RES;
          L.tpre = L.t;
          L.t += L.ts;
        } else {
          L.t += step;
        }
      }
      if (!(L.t <= L.a[6])) enter_stage(L, ST_FWD_FLIGHT);
      return false;
    case ST_FWD_FLIGHT:
      if (!ok) return true;
      if (ADAPTIVE) {
        L.ts += KINEMATICS_RES;
        L.tpre = L.t;
        L.t += L.ts;
      } else {
        L.t += step;
      }
      if (!(L.t < L.a[7])) enter_stage(L, ST_FWD_LAND);
      return false;
    case ST_FWD_LAND:
      if (!ok) return true;
      L.snew_kind = SN_FLIGHT_B;
      L.snew_p = L.a[7];
      L.tnew = L.a[6] + L.a[7];
      L.tnew_set = 1;
      L.f |= GBP_F_VALID;
      return true;
    case ST_REV_FLIGHT:
      if (!ok) return true;
      if (ADAPTIVE) {
        L.ts += KINEMATICS_RES;
        L.tpre = L.t;
        L.t += L.ts;
      } else {
        L.t += step;
      }
      if (!(L.t < L.a[7])) enter_stage(L, ST_REV_STANCE);
      return false;
    case ST_REV_STANCE:
      if (!ok) {
        if (small_step<ADAPTIVE>(L.ts)) {
          L.snew_kind = SN_STANCE_S;  // forward stance on the end state (:857)
          L.snew_p = L.t + BACKUP_RATIO * (L.a[6] - L.t);
          return true;
        }
        L.ts = KINEMATICS_RES;
        L.t = L.tpre;
        L.t -= L.ts;
      } else {
        L.snew_kind = SN_STANCE_REV_B;
        L.snew_p = L.t;
        L.tnew = L.a[6] - L.t;
        L.tnew_set = 1;
        if (ADAPTIVE) {
          L.ts += KINEMATICS_RES;
          L.tpre = L.t;
          L.t -= L.ts;
        } else {
          L.t -= step;
        }
      }
      if (!(L.t >= 0)) enter_stage(L, ST_REV_START);
      return false;
    default:  // ST_REV_START
      if (!ok) return true;
      L.snew_kind = SN_STANCE_REV_B;
      L.snew_p = 0;
      L.tnew = L.a[6];
      L.tnew_set = 1;
      L.f |= GBP_F_VALID;
      return true;
  }
}

// index of the n-th (0-based) set bit of m; requires n < popcount(m)
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int n) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const unsigned long long low = (1ull << w) - 1ull;
    const int c = __popcll(m & low);
    if (n >= c) {
      n -= c;
      m >>= w;
      pos += w;
    } else {
      m &= low;
    }
  }
  return pos;
}


}  // namespace gbp
