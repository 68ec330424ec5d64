// qp_common.h — device helpers shared by the gfx950 QP kernels.
//
// Every helper reproduces one reference operation bit for bit (IEEE binary64, no contraction;
// the library is built with -ffp-contract=off).  Reference behaviour: SURVEY.md §3.2, which
// fixes the operation order of libquadprog.a(QuadProg++.o) (the prebuilt solver behind
// include/QuadProgpp/QuadProg++.hh:69-72).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qpgpu.h"

namespace qpk {

constexpr double kEps = 2.220446049250313080847e-16;  // std::numeric_limits<double>::epsilon()
constexpr double kSqrt2 = 1.4142135623730951;         // sqrt(2.0), .rodata +0x1e8

__device__ __forceinline__ double dinf() { return __builtin_inf(); }

// sqrt(x) for x in [1, 2] (or NaN): the compiler's correctly rounded binary64 sqrt sequence
// (v_rsq_f64 seed, Goldschmidt / Newton refinement) without its range scaling (an ldexp by 0
// for x >= 2^-767) and its +-0 / +inf pass-through, neither of which can apply on [1, 2] —
// the same bits in ~8 fewer instructions.  tools/sqrt_probe.hip checks it against sqrt() over
// the whole interval.
__device__ __forceinline__ double sqrt_1to2(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}

// distance(a, b) — the reference's overflow-safe hypot (three branches), evaluated branch-free
// so that divergent lanes do not serialise; the selected branch computes exactly the same
// operations as the reference's.  1 + t*t lies in [1, 2] whenever the selected branch uses it
// (t = num / den with num <= den; the equal-magnitude branch discards it): sqrt_1to2.
__device__ __forceinline__ double qp_distance(double a, double b) {
  const double a1 = fabs(a), b1 = fabs(b);
  const bool gt = a1 > b1, lt = b1 > a1;
  const double num = gt ? b1 : a1;
  const double den = gt ? a1 : b1;
  const double t = num / den;
  const double h = den * sqrt_1to2(1.0 + t * t);
  return (gt || lt) ? h : a1 * kSqrt2;
}

// the same with the library sqrt() (tools/sqrt_probe.hip checks the two against each other)
__device__ __forceinline__ double qp_distance_libm(double a, double b) {
  const double a1 = fabs(a), b1 = fabs(b);
  const bool gt = a1 > b1, lt = b1 > a1;
  const double num = gt ? b1 : a1;
  const double den = gt ? a1 : b1;
  const double t = num / den;
  const double h = den * sqrt(1.0 + t * t);
  return (gt || lt) ? h : a1 * kSqrt2;
}

// ---- register-array helpers of the one-QP-per-lane kernels (qp_lane.hip, qp_pair.hip)
template <typename T>
__device__ __forceinline__ T opq_l(T v) {
  asm("" : "+v"(v));
  return v;
}

// v[i] / v[i] = x for a run-time i known to be >= LO (entries below LO are never selected)
template <int LO, int N, typename T>
__device__ __forceinline__ T lsel_lo(const T (&v)[N], int i) {
  T r = opq_l(v[LO]);
#pragma unroll
  for (int k = LO + 1; k < N; k++) r = (k == i) ? opq_l(v[k]) : r;
  return r;
}
template <int N, typename T>
__device__ __forceinline__ T lsel(const T (&v)[N], int i) {
  return lsel_lo<0>(v, i);
}

template <int LO, int N, typename T>
__device__ __forceinline__ void lput_lo(T (&v)[N], int i, T x) {
#pragma unroll
  for (int k = LO; k < N; k++) v[k] = (k == i) ? x : v[k];
}

// R storage: packed upper triangle (row-major) followed by the first subdiagonal.
template <int NM>
struct RIdx {
  static constexpr int NUP = NM * (NM + 1) / 2;
  static constexpr int SIZE = NUP + NM - 1;
  // compile-time index of R[i][j]; -1 for entries that are always zero
  static constexpr int at(int i, int j) {
    return j >= i ? i * NM - i * (i - 1) / 2 + (j - i) : (i == j + 1 ? NUP + j : -1);
  }
};

__device__ __forceinline__ bool wave_any(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }

// ---- arithmetic of the fast builds (qp_lane.hip, qp_pair.hip).  F (= the fast build and not
// the fallback body) selects the fast forms; otherwise a / b is the IEEE division and distance
// the reference's scaled form.  The fast forms are valid for operands well inside the exponent
// range: each one ANDs its own validity into the lane's `ok`, and a wave with any lane not ok
// re-solves with the IEEE forms (the SAFE body), so no branch sits inside the arithmetic.
// 1 / b: the v_rcp_f64 seed and the two Newton steps of the compiler's own division sequence,
// without its range scaling and special-case fix-up
__device__ __forceinline__ double frcp(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-b, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ bool rcp_ok(double r) {
  return __builtin_amdgcn_class(r, 0x108);  // +-normal (b zero, denormal, huge, inf or NaN fail)
}
// a / b given rb = frcp(b) (F) — a * rb
template <bool F>
__device__ __forceinline__ double ldiv_r(double a, double b, double rb, bool& ok) {
  if constexpr (F) {
    ok = ok && rcp_ok(rb);
    return a * rb;
  } else {
    return a / b;
  }
}
template <bool F>
__device__ __forceinline__ double ldiv(double a, double b, bool& ok) {
  if constexpr (F)
    return ldiv_r<true>(a, b, frcp(b), ok);
  else
    return a / b;
}
// distance(a, b) (F): sqrt(a^2 + b^2) with the [1, 2]-free form of sqrt_1to2's refinement,
// valid for a^2 + b^2 in [2^-600, 2^600] (and exactly 0 when a = b = 0, as the reference's)
template <bool F>
__device__ __forceinline__ double ldistance(double a, double b, bool& ok) {
  if constexpr (F) {
    const double s = __builtin_fma(a, a, b * b);
    const double y = __builtin_amdgcn_rsq(s);
    double g = s * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double d = __builtin_fma(-g, g, s);
    g = __builtin_fma(d, h, g);
    const bool z = (a == 0.0) && (b == 0.0);
    ok = ok && (z || (s >= 0x1p-600 && s <= 0x1p600));
    return z ? 0.0 : g;
  } else {
    return qp_distance(a, b);
  }
}

// Sequential sums over runtime-length index ranges with the operand loads batched kU at a time
// (qp_wave.hip, qp_generic.hip): all kU loads of a chunk are issued before the chunk's
// multiply-adds, so a loop over global (or LDS) operands costs one memory latency per chunk
// instead of one per element.  The adds stay strictly sequential in the reference's index
// order, so results are bit-identical to the plain loops.
// s + sum_{j=j0}^{j1-1} A(j) * B(j), j ascending (s += a*b per element).  Full chunks of kU
// issue all their loads unpredicated before the chunk's multiply-adds; the remainder is one
// predicated chunk.
template <int kU, class FA, class FB>
__device__ __forceinline__ double seq_fma_up(double s, int j0, int j1, FA A, FB B) {
  if constexpr (kU == 1) {
    for (int j = j0; j < j1; j++) s += A(j) * B(j);
    return s;
  }
  int jb = j0;
  for (; jb + kU <= j1; jb += kU) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = A(jb + u);
      vb[u] = B(jb + u);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) s += va[u] * vb[u];
  }
  if (jb < j1) {  // partial chunk: loads predicated, still one latency
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = jb + u < j1 ? A(jb + u) : 0.0;
      vb[u] = jb + u < j1 ? B(jb + u) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (jb + u < j1) s += va[u] * vb[u];
  }
  return s;
}

// seq_fma_up for operands in LDS with s starting at +0.0: the partial chunk's loads are
// unconditional (past j1 they read whatever lies there — in-bounds LDS) and its products past
// j1 are replaced by +0.0, so there is no exec-mask branch per load.  A sum that starts at
// +0.0 is never -0.0 (a sum is -0.0 only from two -0.0 operands), so adding +0.0 leaves it
// unchanged.
template <int kU, class FA, class FB>
__device__ __forceinline__ double seq_fma_up_lds(double s, int j0, int j1, FA A, FB B) {
  int jb = j0;
  for (; jb + kU <= j1; jb += kU) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = A(jb + u);
      vb[u] = B(jb + u);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) s += va[u] * vb[u];
  }
  if (jb < j1) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = A(jb + u);
      vb[u] = B(jb + u);
    }
    const int c = j1 - jb;
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const double q = va[u] * vb[u];
      s += u < c ? q : 0.0;
    }
  }
  return s;
}

// s - sum A(j) * B(j), j ascending (s -= a*b per element)
template <int kU, class FA, class FB>
__device__ __forceinline__ double seq_fms_up(double s, int j0, int j1, FA A, FB B) {
  if constexpr (kU == 1) {
    for (int j = j0; j < j1; j++) s -= A(j) * B(j);
    return s;
  }
  int jb = j0;
  for (; jb + kU <= j1; jb += kU) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = A(jb + u);
      vb[u] = B(jb + u);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) s -= va[u] * vb[u];
  }
  if (jb < j1) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = jb + u < j1 ? A(jb + u) : 0.0;
      vb[u] = jb + u < j1 ? B(jb + u) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (jb + u < j1) s -= va[u] * vb[u];
  }
  return s;
}

// s - sum A(k) * B(k), k DEscending from k1-1 down to k0 (s -= a*b per element)
template <int kU, class FA, class FB>
__device__ __forceinline__ double seq_fms_down(double s, int k0, int k1, FA A, FB B) {
  if constexpr (kU == 1) {
    for (int k = k1 - 1; k >= k0; k--) s -= A(k) * B(k);
    return s;
  }
  int kb = k1 - 1;
  for (; kb - kU + 1 >= k0; kb -= kU) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = A(kb - u);
      vb[u] = B(kb - u);
    }
#pragma unroll
    for (int u = 0; u < kU; u++) s -= va[u] * vb[u];
  }
  if (kb >= k0) {
    double va[kU], vb[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      va[u] = kb - u >= k0 ? A(kb - u) : 0.0;
      vb[u] = kb - u >= k0 ? B(kb - u) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kU; u++)
      if (kb - u >= k0) s -= va[u] * vb[u];
  }
  return s;
}

// Ordering point for LDS hand-offs between lanes of ONE wavefront.  A QP is always owned by
// lanes of a single wave that are converged with each other (every control decision is a
// function of replicated values), and a wave's LDS instructions execute in issue order, so a
// compiler-level fence is all that is needed (no s_barrier).
__device__ __forceinline__ void sg_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Offset of element 0 of QP b's block of E elements; element e is at +e*T.
// T = 1: QP-major (ArrayHH blocks back to back); T = 64: TILED64 (include/qpgpu.h).
template <int T>
__device__ __forceinline__ int64_t qbase(int64_t b, int E) {
  if constexpr (T == 1)
    return b * (int64_t)E;
  else
    return (b >> 6) * (int64_t)(64 * E) + (b & 63);
}
__device__ __forceinline__ int64_t qbase_rt(int64_t b, int64_t E, int T) {
  return T == 1 ? b * E : (b >> 6) * (64 * E) + (b & 63);
}

struct QpArgs {
  int n, p, m, max_steps;
  int tile;  // 1 = QP-major, 64 = TILED64
  int64_t batch;
  uint32_t flags;
  double* G;
  const double* g0;
  const double* CE;
  const double* ce0;
  const double* CI;
  const double* ci0;
  double* x;
  double* f;
  int32_t* status;
  int32_t* iters;
  // optional (NULL unless qpgpu_solve_batched_eq): the state after the equality phase, i.e. the
  // result of the same QP with CI dropped (m = 0) — x_eq / f_eq / st_eq per QP
  double* x_eq;
  double* f_eq;
  int32_t* st_eq;
  // diagnostic only (NULL in every product call): per-wave s_memtime stamps at phase
  // boundaries, kStampSlots per wave, written by lane 0.  Never feeds an output.
  uint64_t* stamps;
};
constexpr int kStampSlots = 18;
// internal QpArgs.flags bit set by the host when CI and ci0 are 16-byte aligned
constexpr uint32_t kArgAligned16 = 0x80000000u;
// internal QpArgs.flags bit: the workspace already holds the setup (qp_panel.hip) — J, x0, f0,
// c1, c2 and the Cholesky status — so the loop kernel starts at the equality phase
constexpr uint32_t kSetupDone = 0x40000000u;
// internal QpArgs.flags bit: the EXACT re-solve launch after a tolerance-mode launch — only the
// QPs whose status carries kStResolve are solved (one QP per workgroup: the others exit at once)
constexpr uint32_t kResolveOnly = 0x20000000u;
// internal QpArgs.flags bit: the workspace holds an fp32 copy of CI after the batch's per-QP
// blocks (qp_wave.hip qp_ci_shadow_kernel), which the tolerance-mode l1 scan reads first
constexpr uint32_t kArgShadow = 0x08000000u;
// Tolerance mode (n > 64 default: MFMA panel setup + tree sums) certification.  A QP one of whose
// decisions the tolerance arithmetic cannot certify against the reference's rounding is marked in
// its status word (kStResolve | reason << kStReasonShift) and re-solved by the EXACT launch, which
// writes the plain status back.  Reasons:
enum : int {
  kUncDependent = 1 << 0,   // add_constraint: |d_iq| <= 1e6 eps R_norm (rank-deficient / near-dependent column)
  kUncSetup = 1 << 1,       // panel setup: not positive definite, or pivots spread beyond 1e8
  kUncMaxIter = 1 << 2,     // the step cap fired
  kUncStepTie = 1 << 3,     // t1 and t2 within 1e-9 relative (partial vs full step)
  kUncZz = 1 << 4,          // z.z within [eps/4, 4 eps] of the reference's |z.z| > eps test
  kUncTt2 = 1 << 5,         // |t - t2| within [eps/4, 4 eps] of the full-step test
  kUncSelTie = 1 << 6,      // two most violated constraints within 1e-9 relative
  kUncPsi = 1 << 7,         // |psi| within [thr/4, 4 thr] of the stop test
  kUncFCancel = 1 << 8,     // the objective cancels: max |f| over the run > 1e4 |f|
  kUncXCancel = 1 << 9,     // x cancels: max ||x||_inf over the run > 1e4 ||x||_inf
  kUncNonFinite = 1 << 10,  // a non-finite x or f (infeasible included)
  kUncT1Tie = 1 << 11,      // two blocking constraints' u/r within 1e-9 relative
  kUncGivens = 1 << 12      // a Givens length within [eps/4, 4 eps] of the |h| < eps skip
};
constexpr int kStResolve = 0x100;
constexpr int kStReasonShift = 9;

// Per-QP device workspace of the large-QP path (n > 64, qp_wave.hip GJR + qp_panel.hip):
//   [0, OFF_R)        J, COLUMN-major: J[k][j] at j*JS + k
//   [OFF_R, OFF_H)    R row-major (R[i][j] at i*JS + j); the setup's scratch for G -> L
//   [OFF_H, OFF_G)    header: status, f0, c1, c2, (pad), x0 at HX
//   [OFF_G, PER_QP)   the Givens coefficients of a deferred add_constraint sweep while a second
//                     one is pending (qp_wave.hip, tolerance mode: 4 per rotation)
constexpr int kBigN = 256;
template <int NMAX>
struct BigWs {
  static constexpr int JS = NMAX + 1;
  static constexpr int64_t OFF_R = (int64_t)NMAX * JS;
  static constexpr int64_t OFF_H = 2 * (int64_t)NMAX * JS;
  static constexpr int HX = 8;
  static constexpr int64_t OFF_G = OFF_H + HX + NMAX;
  static constexpr int64_t PER_QP = OFF_G + 4 * (int64_t)NMAX;
};

__device__ __forceinline__ void qp_stamp(const QpArgs& a, int slot) {
  if (a.stamps) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) a.stamps[(uint64_t)blockIdx.x * kStampSlots + slot] = t;
    // start / end also on the 100 MHz constant clock (s_memtime is the shader clock of the
    // wave's XCD, neither constant-rate nor synchronised across XCDs): slots 16 / 17
    if (slot == 0 || slot == 4) {
      const uint64_t r = __builtin_amdgcn_s_memrealtime();
      if (threadIdx.x == 0) a.stamps[(uint64_t)blockIdx.x * kStampSlots + 16 + (slot == 4)] = r;
    }
  }
}

}  // namespace qpk
