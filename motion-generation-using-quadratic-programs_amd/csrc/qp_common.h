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
__device__ __forceinline__ int64_t qbase_rt(int64_t b, int E, int T) {
  return T == 1 ? b * (int64_t)E : (b >> 6) * (int64_t)(64 * E) + (b & 63);
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

// Per-QP device workspace of the large-QP path (n > 64, qp_wave.hip GJR + qp_panel.hip):
//   [0, OFF_R)        J, COLUMN-major: J[k][j] at j*JS + k
//   [OFF_R, OFF_H)    R row-major (R[i][j] at i*JS + j); the setup's scratch for G -> L
//   [OFF_H, PER_QP)   header: status, f0, c1, c2, (pad), x0 at HX
constexpr int kBigN = 256;
template <int NMAX>
struct BigWs {
  static constexpr int JS = NMAX + 1;
  static constexpr int64_t OFF_R = (int64_t)NMAX * JS;
  static constexpr int64_t OFF_H = 2 * (int64_t)NMAX * JS;
  static constexpr int HX = 8;
  static constexpr int64_t PER_QP = OFF_H + HX + NMAX;
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
