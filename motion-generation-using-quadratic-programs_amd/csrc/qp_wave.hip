// qp_wave.hip — gfx950 batched Goldfarb–Idnani solver for larger dense QPs (16 < n <= 256).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; operation order
// of the prebuilt libquadprog.a fixed in SURVEY.md §3.2).  One QP per SUBGROUP of S lanes
// (S = 32: two QPs per wavefront; S = 64: one; S = 256: a 4-wave workgroup), split as:
//   * "lead" work — the O(n) / O(iq^2) serial chains (Givens coefficients, update_r, step
//     lengths, dot products, active-set bookkeeping) — runs on lane 0 of every subgroup, so a
//     wave advances 64/S QPs' serial chains with each instruction;
//   * row-/column-parallel work — compute_d (lane = column of J), update_z and every Givens
//     row update (lane = row of J), the l1 scan s = CI^T x + ci0 (lane = constraint, CI rows
//     read coalesced from HBM/L2), the Cholesky column, the J = L^{-T} rows — is spread over
//     the subgroup's lanes.  Every parallel element keeps the reference's summation order, so
//     results are bitwise identical to the CPU restatement (oracle/qp_oracle.c).
// State lives in LDS (per QP: J and R [n][n+1], vectors, bookkeeping) with dynamic indexing;
// with GJR, J and R live in a global workspace instead (n = 256: 2 x 514 KiB per QP).  The
// lead lane exchanges scalars with its subgroup through an LDS control block.
//
// The same source built a second time with QPGPU_WAVE_FAST=1 and -ffp-contract=fast
// (qp_wave_fast.hip) is the QPGPU_FLAG_FAST kernel for the LDS variants (n <= 64, m <= 256:
// the mgqp hierarchy levels, C3): the lead's serial chains — add_constraint's |h| chain, the
// Givens coefficients of add_constraint and delete_constraint, update_r's back-substitution,
// the step lengths t1 / t2 — and the setup's divisions use one refined reciprocal per divisor
// and distance() as sqrt(a^2 + b^2) (rsq + refinement), multiply-adds fused.  Same algorithm
// and decisions; x and f within north_star's 1e-10 relative instead of bit-identical.  Every
// fast form checks that its operands are well inside the exponent range; a wave with any
// failed check re-solves with the IEEE forms.
#include <climits>
#include <cstdlib>
#include <map>
#include <mutex>

#include <type_traits>

#include "qp_common.h"

#ifndef QPGPU_WAVE_FAST
#define QPGPU_WAVE_FAST 0
#endif
#if QPGPU_WAVE_FAST
#define QPK_WAVE_NS qpk_wfast
#define QP_WAVE_KERNEL qp_wave_fast_kernel
#else
#define QPK_WAVE_NS qpk
#define QP_WAVE_KERNEL qp_wave_kernel
#endif

namespace QPK_WAVE_NS {
using namespace qpk;
constexpr bool kWaveFast = QPGPU_WAVE_FAST != 0;

// ---- the fast build's arithmetic (F = kWaveFast and not the IEEE fallback body)
// 1 / b: v_rcp_f64 + the two Newton steps of the compiler's own division sequence (without its
// range scaling and special-case fix-up); valid when the result is a normal number
__device__ __forceinline__ double wrcp(double b) {
  double y = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-b, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ bool wrcp_ok(double r) {
  return __builtin_amdgcn_class(r, 0x108);  // +-normal
}
// a / b given rb = wrcp(b) (F); a / b otherwise
template <bool F>
__device__ __forceinline__ double wdiv_r(double a, double b, double rb, bool& ok) {
  if constexpr (F) {
    ok = ok && wrcp_ok(rb);
    return a * rb;
  } else {
    return a / b;
  }
}
template <bool F>
__device__ __forceinline__ double wdiv(double a, double b, bool& ok) {
  if constexpr (F)
    return wdiv_r<true>(a, b, wrcp(b), ok);
  else
    return a / b;
}
// distance(a, b) (F): sqrt(a^2 + b^2) by v_rsq_f64 + one Goldschmidt refinement and a final
// Newton correction, valid for a^2 + b^2 in [2^-600, 2^600] (exactly 0 when a = b = 0, as the
// reference's); otherwise the reference's scaled form (qp_distance)
template <bool F>
__device__ __forceinline__ double wdist(double a, double b, bool& ok) {
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

template <int S>
__device__ __forceinline__ void grp_sync() {
  if constexpr (S > 64)
    __syncthreads();
  else
    sg_sync();
}

// Sequential sums over runtime-length index ranges with the operand loads batched kU at a time:
// all kU loads of a chunk are issued before the chunk's multiply-adds, so a loop over global
// (or LDS) operands costs one memory latency per chunk instead of one per element.  The adds
// stay strictly sequential in the reference's index order, so results are bit-identical.
// Chunk sizes: operands in global memory (CI always; J and R with GJR) batch kUG loads per
// chunk; LDS-resident operands batch kUL.
#ifndef QPGPU_WAVE_KUL
#define QPGPU_WAVE_KUL 4
#endif
// J columns of a Givens sweep loaded per chunk (LDS-resident J)
#ifndef QPGPU_WAVE_KUJ
#define QPGPU_WAVE_KUJ 4
#endif
// chunk of compute_d_z's LDS sums (J in LDS)
#ifndef QPGPU_WAVE_KUDZ
#define QPGPU_WAVE_KUDZ 8
#endif
constexpr int kUG = 8, kUL = QPGPU_WAVE_KUL;

// Value of v held by lane i of this thread's subgroup (S = 16 / 32: lane i of each 16- / 32-lane group of the wave
// serve the two QPs; S = 64: lane i).  i must be wave-uniform (a compile-time step index): two
// or four v_readlane per double, no LDS round trip.
template <int S>
__device__ __forceinline__ double sg_bcast(double v, int i) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
  const uint32_t l0 = __builtin_amdgcn_readlane(lo, i), h0 = __builtin_amdgcn_readlane(hi, i);
  if constexpr (S == 64) {
    return __builtin_bit_cast(double, ((uint64_t)h0 << 32) | l0);
  } else if constexpr (S == 16) {
    const uint32_t l1 = __builtin_amdgcn_readlane(lo, 16 + i), h1 = __builtin_amdgcn_readlane(hi, 16 + i);
    const uint32_t l2 = __builtin_amdgcn_readlane(lo, 32 + i), h2 = __builtin_amdgcn_readlane(hi, 32 + i);
    const uint32_t l3 = __builtin_amdgcn_readlane(lo, 48 + i), h3 = __builtin_amdgcn_readlane(hi, 48 + i);
    const int q = threadIdx.x >> 4;
    const uint32_t l = q == 0 ? l0 : q == 1 ? l1 : q == 2 ? l2 : l3;
    const uint32_t h = q == 0 ? h0 : q == 1 ? h1 : q == 2 ? h2 : h3;
    return __builtin_bit_cast(double, ((uint64_t)h << 32) | l);
  } else {
    static_assert(S == 32, "sg_bcast: one, two or four QPs per wave");
    const uint32_t l1 = __builtin_amdgcn_readlane(lo, 32 + i), h1 = __builtin_amdgcn_readlane(hi, 32 + i);
    const bool up = threadIdx.x >= 32;
    return __builtin_bit_cast(double, ((uint64_t)(up ? h1 : h0) << 32) | (up ? l1 : l0));
  }
}

// Subgroup argmin for S <= 64 (xor butterfly): the smallest v, ties to the smallest index — the
// result of a sequential `if (v < best)` scan in index order.  Lanes without a candidate pass
// (+inf, INT_MAX); the caller never offers +inf as a candidate.
template <int S>
__device__ __forceinline__ void sg_argmin(double& v, int& i) {
  static_assert(S <= 64, "one wave per subgroup");
#pragma unroll
  for (int o = 1; o < S; o <<= 1) {
    const double v2 = __shfl_xor(v, o, S);
    const int i2 = __shfl_xor(i, o, S);
    const bool take = (v2 < v) || (v2 == v && i2 < i);
    v = take ? v2 : v;
    i = take ? i2 : i;
  }
}

// Tolerance-mode loop kernels for the workspace variant (n > 64 after the MFMA panel setup, which
// already gives up the reference's bits for north_star's 1e-10): update_r as a wave-wide tree
// sum per row (no serial chain, no LDS round trip) and compute_d + update_z fused into one pass
// over J (lane = row, column chunks tree-reduced), so J is read once per step instead of
// 1 + (n - iq) / n times.  QPGPU_FLAG_EXACT keeps the serial, bit-exact sums.
// (Variants measured neutral or slower on C5 and removed in round 3, kept in git history:
// coefficients loaded per chunk of rotations in the J sweep, two constraints per lane in the
// l1 scan, the t1 selection across the four waves — DESIGN §5.3.)
#ifndef QPGPU_WAVE_TOLLOOP
#define QPGPU_WAVE_TOLLOOP 15  // bit 0: fused compute_d + update_z, bit 1: tree update_r,
                               // bit 2: add_constraint J sweep deferred into the next d/z pass,
                               // bit 3: two sweeps deferred, J written back every second add
#endif
// v from the lane the DPP control CTRL selects (a full-row permutation: every lane valid)
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Sum of v over the 64 lanes of this wave (all lanes active), the same value in every lane:
// symmetric butterflies inside each 16-lane row (quad xor 1, xor 2, half-row mirror, row
// mirror: every pair adds the same two operands), then the four row sums in row order
__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);  // row_half_mirror
  v += dpp_f64<0x140>(v);  // row_mirror
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
  double r[4];
#pragma unroll
  for (int k = 0; k < 4; k++)
    r[k] = __builtin_bit_cast(double, ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(hi, 16 * k) << 32) |
                                          (uint32_t)__builtin_amdgcn_readlane(lo, 16 * k));  // no sign extension
  return ((r[0] + r[1]) + r[2]) + r[3];
}

// Sixteen sums over the wave's 64 lanes at once (tolerance mode's d = J^T np, 16 columns per
// chunk): a reduce-scatter instead of sixteen full butterflies — v_permlane32_swap (lanes l, l^32),
// v_permlane16_swap (l, l^16 within each half), DPP row_mirror (i, 15-i) and row_half_mirror
// (i, 7-i) each halve the columns a lane carries while doubling the lanes summed, then two quad
// butterflies finish; ~60 instructions instead of ~370.  Lane l ends with the full sum of column
// colsum16_col(l) (the four lanes of a quad hold the same value, a + b == b + a).
__device__ __forceinline__ void swap_pl32(double& a, double& b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | (uint32_t)lo[0]);
  b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | (uint32_t)lo[1]);
}
__device__ __forceinline__ void swap_pl16(double& a, double& b) {
  const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)ua, (uint32_t)ub, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(ua >> 32), (uint32_t)(ub >> 32), false, false);
  a = __builtin_bit_cast(double, ((uint64_t)hi[0] << 32) | (uint32_t)lo[0]);
  b = __builtin_bit_cast(double, ((uint64_t)hi[1] << 32) | (uint32_t)lo[1]);
}
__device__ __forceinline__ int colsum16_col(int lane) {
  return ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane & 15) >= 8) * 2 + ((lane & 7) >= 4);
}
__device__ __forceinline__ double colsum16(double (&v)[16]) {
  const int l = threadIdx.x & 63;
  double w[8];
#pragma unroll
  for (int u = 0; u < 8; u++) {  // lanes < 32 keep columns 0..7, lanes >= 32 columns 8..15
    double a = v[u], b = v[u + 8];
    swap_pl32(a, b);
    w[u] = a + b;
  }
  double x[4];
#pragma unroll
  for (int u = 0; u < 4; u++) {  // within each half: lanes 0..15 keep slots 0..3, 16..31 slots 4..7
    double a = w[u], b = w[u + 4];
    swap_pl16(a, b);
    x[u] = a + b;
  }
  const bool lo8 = (l & 15) < 8, lo4 = (l & 7) < 4;
  double y[2];
#pragma unroll
  for (int u = 0; u < 2; u++) {  // row_mirror pairs i with 15 - i: i < 8 keeps slots 0..1
    const double keep = lo8 ? x[u] : x[u + 2], send = lo8 ? x[u + 2] : x[u];
    y[u] = keep + dpp_f64<0x140>(send);
  }
  // row_half_mirror pairs i with 7 - i: (i & 7) < 4 keeps slot 0
  double z = (lo4 ? y[0] : y[1]) + dpp_f64<0x141>(lo4 ? y[1] : y[0]);
  z += dpp_f64<0xB1>(z);  // quad xor 1
  z += dpp_f64<0x4E>(z);  // quad xor 2
  return z;
}

// Register-resident setup for the one-wave variants (S <= 64, LDS J/R, launched at one wave per
// SIMD so registers are plentiful): lane j keeps row j of G/L (Cholesky), lane r builds row r of
// J = L^{-T} by column-oriented forward substitution, and cholesky_solve runs across the lanes
// with v_readlane broadcasts.  Every element sees the reference's operations in the reference's
// order (see the block), so results are bitwise unchanged.
// (Removed in round 3 after measuring slower, kept in git history: CI columns in registers
// across the loop — C3 16.7 vs 15.4 ms, profiles/r02_s8 —, all of a lane's CI loads issued at
// once in the scan — 16.0 vs 15.3 ms, profiles/r02_s10 —, and J in registers with packed R at
// two waves per SIMD — C3 18.7 vs 14.5 ms, mgqp 1.96 vs 1.76 ms, profiles/r02_s19.)
// four QPs per wave (S = 16) for n <= 16, m <= 32 (the mgqp hierarchy levels)
#ifndef QPGPU_WAVE_S16
#define QPGPU_WAVE_S16 1
#endif
#ifndef QPGPU_WAVE_FALLTHRU
#define QPGPU_WAVE_FALLTHRU 1
#endif
#ifndef QPGPU_WAVE_RPACK
#define QPGPU_WAVE_RPACK 1
#endif
#ifndef QPGPU_WAVE_REGSETUP
#define QPGPU_WAVE_REGSETUP 1
#endif
// update_r on the lead with row i-1's row values and first chunk of its R and r entries loaded
// while row i's division is in flight, r[i+1] carried in a register, later chunks double-buffered
#ifndef QPGPU_WAVE_URPF
#define QPGPU_WAVE_URPF 1
#endif
#ifndef QPGPU_WAVE_URU
#define QPGPU_WAVE_URU 4
#endif
// the select after a scan prepared inside the scan (argmin, np gather, ci0[ip] in flight early)
#ifndef QPGPU_WAVE_PRESEL
#define QPGPU_WAVE_PRESEL 1
#endif
// per-phase clocks of the diagnostic stamps (tools/stamps_wave.py; off in the product build:
// their accumulators cost ~50 VGPRs, which the l1 scan's 16-row chunks use instead)
#ifndef QPGPU_WAVE_STAMPS
#define QPGPU_WAVE_STAMPS 0
#endif
// add_constraint's |h| chain in unmasked chunks + a one-rotation tail, qp_distance_f
#ifndef QPGPU_WAVE_HCHAIN2
#define QPGPU_WAVE_HCHAIN2 1
#endif
#ifndef QPGPU_WAVE_HCU  // rotations per unmasked chunk of the |h| chain
#define QPGPU_WAVE_HCU 8
#endif
// add_constraint's J sweep (J in LDS) in unmasked chunks + a one-rotation tail
#ifndef QPGPU_WAVE_SWEEP2
#define QPGPU_WAVE_SWEEP2 1
#endif
// CI loads per chunk of the two-constraint l1 scan (one global-memory round trip per chunk)
#ifndef QPGPU_WAVE_SCANKG
#define QPGPU_WAVE_SCANKG 16
#endif
#ifndef QPGPU_WAVE_SCANKG4  // the 128-VGPR (four waves per SIMD) instantiations
#define QPGPU_WAVE_SCANKG4 16
#endif
// diagnostic stamps only: slots 5..7 hold, instead of the equality-phase parts, the loop's
// update_r cycles, step count and sum of iq over steps (1), or add_constraint's |h| chain +
// coefficients, J sweep and R column + test cycles, equality phase and loop together (2)
// largest block LDS (bytes) for which the S < 64 variants launch their four-waves-per-SIMD
// instantiation (128 VGPRs); A/B builds lower it to send such shapes to the OCC 2 / 1 ones
#ifndef QPGPU_WAVE_OCC4_LDS
#define QPGPU_WAVE_OCC4_LDS 20480
#endif
#ifndef QPGPU_WAVE_OCC_SMALL  // the waves per SIMD that instantiation is compiled for
#define QPGPU_WAVE_OCC_SMALL 4
#endif
// waves per SIMD the workspace variant's registers are allocated for (4: 128 VGPRs, four resident
// QPs per CU; an A/B build may lower it)
#ifndef QPGPU_WAVE_GJR_OCC
#define QPGPU_WAVE_GJR_OCC 4
#endif
#ifndef QPGPU_WAVE_GJR_CAP
#define QPGPU_WAVE_GJR_CAP 0
#endif
#ifndef QPGPU_WAVE_STAMPS_DETAIL
#define QPGPU_WAVE_STAMPS_DETAIL 0
#endif
// Tolerance-mode l1 scan from an fp32 copy of CI (the workspace variant, n > 64):
// each s_i first from the half-size copy with a rigorous bound on its distance from the fp64
// sum, then the exact fp64 sum only for the constraints the select can pick; a pass whose stop
// test or candidates the bounds cannot settle scans in fp64 as before.  0 = always fp64.
#ifndef QPGPU_WAVE_SHADOW
#define QPGPU_WAVE_SHADOW 1
#endif
constexpr int kShadowCand = 16;  // most exact re-evaluations per shadow scan (else the fp64 scan)
// diagnostic counts (qpgpu_debug_shadow_stats): l1 scans that tried the fp32 copy, and those the
// bounds settled (one atomic per QP and scan, by the lead)
__device__ unsigned long long g_shadow_stats[3];  // [2]: fp64 re-evaluations (candidates)
#ifndef QPGPU_WAVE_SHADOW_U  // fp32 CI loads per constraint and chunk of the shadow scan
#define QPGPU_WAVE_SHADOW_U 32
#endif
#ifndef QPGPU_WAVE_SHADOW_KP  // a lane's constraints whose chunks load together
#define QPGPU_WAVE_SHADOW_KP 1
#endif
// per-QP control block (lead lane writes, subgroup reads after grp_sync)
struct Ctl {
  double f, t, t1, t2, ss, R_norm, c1, c2, psi, ci0ip, znp;
  // tolerance-mode certification (qp_common.h kUnc*): max |f| over the run, and the bits of
  // ||x||_inf at the end / of max ||x||_inf over the run (non-negative doubles order as integers)
  double fmax;
  unsigned long long xn, xh;
  // tolerance mode: bits of max_i ||CI[:, i]||_1 and max_i |ci0_i| (the scale of an s_i's rounding)
  unsigned long long cim, c0m;
  int iq, ip, l, status, phase, iter, steps, flags, qq, ngiv, fin;
  int unc;  // tolerance mode: kUnc* reasons this QP's decisions are not certified
  int pad[4];
};

enum : int {
  PH_DONE = 0,
  PH_SCAN = 1,   // l1
  PH_SELECT = 2, // l2
  PH_STEP = 3    // l2a
};

template <int S, int NMAX, int MMAX, bool GJR>
struct WaveCfg {
  static constexpr int QPB = S >= 64 ? 1 : 64 / S;  // QPs per block
  static constexpr int BS = S >= 64 ? S : 64;       // threads per block
  static constexpr int64_t WS_DOUBLES = GJR ? BigWs<NMAX>::PER_QP : 0;  // per QP, global workspace
};

// LDS layout of one QP, sized by the launch's (n, m) rather than the size class's (NMAX, MMAX),
// so a problem below the class bound takes only what it needs (C3, n = 30 in the n <= 32
// class: 37 KiB per two-QP block instead of 42 KiB, i.e. 4 blocks per CU instead of 3, one
// wave on every SIMD).  J and R are [n][js] with an odd row stride js, so walks down a column
// (lane = row) are LDS-bank-conflict free; with GJR they live in the workspace instead.
// Vectors: x z d np r x_old (n each), the Givens coefficients (4n, interleaved per rotation),
// u u_old (n+1 each), s (m), then int A A_old
// (n+1 each), uint8 act exc (m each) and the control block.
#ifndef QPGPU_WAVE_TOLCH
#define QPGPU_WAVE_TOLCH 16
#endif
constexpr int kTolCh = QPGPU_WAVE_TOLCH;  // columns per tree-summed chunk of the tolerance-mode d/z pass
struct WaveLay {
  int js, nr, off_r, off_x, off_z, off_d, off_np, off_rv, off_xo, off_gc, off_u, off_uo, off_s,
      off_a, off_fl, off_ctl, off_tsc, off_sp, stride;
};
__host__ __device__ inline WaveLay wave_lay(int n, int m, bool gjr, bool rpack = false) {
  WaveLay L;
  L.js = (n + 1) | 1;
  L.nr = n * (n + 1) / 2 + (n > 0 ? n - 1 : 0) + 1;
  if (rpack && !gjr) {
    // J [n][js] at 0, R packed after it, the loop's vectors, then x z d; during the setup the
    // factor L ([n][js]) overlays R and the loop's vectors
    L.off_r = n * L.js;
    L.off_np = L.off_r + L.nr;
    L.off_rv = L.off_np + n;
    L.off_xo = L.off_rv + n;
    L.off_gc = L.off_xo + n;
    L.off_u = L.off_gc + 4 * n;
    L.off_uo = L.off_u + n + 1;
    L.off_s = L.off_uo + n + 1;
    L.off_a = L.off_s + m;
    L.off_fl = L.off_a + (2 * (n + 1) + 1) / 2;
    const int end = L.off_fl + (2 * m + 7) / 8;
    L.off_x = end > L.off_r + n * L.js ? end : L.off_r + n * L.js;
    L.off_z = L.off_x + n;
    L.off_d = L.off_z + n;
    L.off_ctl = L.off_d + n;
  } else {
    L.off_r = gjr ? 0 : n * L.js;
    L.off_x = gjr ? 0 : 2 * n * L.js;
    L.off_z = L.off_x + n;
    L.off_d = L.off_z + n;
    L.off_np = L.off_d + n;
    L.off_rv = L.off_np + n;
    L.off_xo = L.off_rv + n;
    L.off_gc = L.off_xo + n;
    L.off_u = L.off_gc + 4 * n;
    L.off_uo = L.off_u + n + 1;
    L.off_s = L.off_uo + n + 1;
    L.off_a = L.off_s + m;
    L.off_fl = L.off_a + (2 * (n + 1) + 1) / 2;
    L.off_ctl = L.off_fl + (2 * m + 7) / 8;
  }
  // the workspace variant's tolerance-mode partial sums (two buffers of 4 waves x kTolCh)
  L.off_tsc = L.off_ctl + (int)((sizeof(Ctl) + 7) / 8);
  // the workspace variant's shadow scan: the n products of one exact re-evaluation, then the
  // candidate list (kShadowCand ints) and its count
  L.off_sp = L.off_tsc + (gjr ? 2 * 4 * kTolCh : 0);
  L.stride = (L.off_sp + (gjr ? n + kShadowCand / 2 + 1 : 0)) | 1;
  return L;
}
// packed-R index: R[i][j] for j >= i, the subdiagonal R[j+1][j], else a write-only slot (the
// entries below it, which the algorithm only ever shifts as zeros)
__device__ __forceinline__ int rpk(int i, int j, int n) {
  const int nup = n * (n + 1) / 2;
  return j >= i ? i * n - (i * (i - 1)) / 2 + (j - i) : (i == j + 1 ? nup + j : nup + n - 1);
}

// OCC = minimum waves per SIMD the register allocation must allow (launch-bounds hint): 1, or
// 4 for the two-QP-per-wave variants when the launch's LDS leaves room for that many (launch_wave)
// The workspace variant (GJR, 256-thread one-QP workgroups) is held to 128 VGPRs (four waves
// per SIMD = four resident QPs per CU): its loop is bound by HBM traffic, which it overlaps only
// across resident QPs (measured: two per CU 399 ms, four 323 ms for C5, profiles/r02_f).
// The solve of one block's QPs.  F: the fast build's arithmetic (wdiv / wdist / wrcp above); the
// IEEE forms otherwise (the exact build always; the fast build's fallback).  Returns false as
// soon as a fast form was not valid on some lane of the wave (checked after the equality phase,
// at every pass of the loop and before the outputs): x, f, status and iters are then not
// written, and the kernel re-solves the block with the IEEE forms — which also rewrites the
// m = 0 snapshot (x_eq / f_eq / st_eq) this attempt may have written.  (With -ffp-contract=fast
// the fallback's multiply-adds are fused too: within 1e-10, not bitwise.)
template <int S, int NMAX, int MMAX, bool GJR, int OCC, bool F>
__device__ __forceinline__ bool wave_body(const QpArgs& a, double* __restrict__ ws) {
  static_assert(!F || (!GJR && S <= 64), "the fast build covers the one-wave LDS variants");
  using C = WaveCfg<S, NMAX, MMAX, GJR>;
  bool fok = true;  // F: every fast form this lane evaluated so far was in range
  // (one-wave blocks: a ballot is the block-wide OR)
  auto any_bad = [&]() -> bool {
    if constexpr (F)
      return __builtin_amdgcn_ballot_w64(!fok) != 0;
    else
      return false;
  };
  constexpr bool kRegSetup = QPGPU_WAVE_REGSETUP && !GJR && NMAX <= S &&
                             ((S == 32 && OCC == 1) || (S == 16 && OCC <= 2));
  // R packed (upper triangle + subdiagonal) with J still in LDS: less LDS per QP, more resident
  // blocks per CU (the register setup keeps the factor L in its own overlay)
  constexpr bool kRPack = QPGPU_WAVE_RPACK && kRegSetup;
  constexpr bool kPackedR = kRPack;
  // lane-parallel selections (argmin of s for l2, of u/r for t1) for one-wave subgroups
  constexpr bool kLaneSel = S <= 64;
  // loads in flight per lane in the global-operand sums (deeper for the one-QP-per-workgroup
  // workspace variant, whose lanes have registers to spare)
  constexpr int KG = GJR ? 16 : kUG;
  extern __shared__ double lds[];
  const WaveLay Ly = wave_lay(a.n, a.m, GJR, kRPack);
  const int JS = GJR ? BigWs<NMAX>::JS : Ly.js;

  const int tid = threadIdx.x;
  const int sg = S >= 64 ? 0 : tid / S;
  const int ls = S >= 64 ? tid : tid - sg * S;
  const bool lead = (ls == 0);
  const int64_t b = (int64_t)blockIdx.x * C::QPB + sg;
  const bool live = b < a.batch;  // whole subgroups only

  double* const Q = lds + sg * Ly.stride;
  double* const Jm = GJR ? ws + (b < a.batch ? b : 0) * (int64_t)C::WS_DOUBLES : Q;
  double* const Rm = GJR ? Jm + BigWs<NMAX>::OFF_R : Q + Ly.off_r;
  double* const Lm = Rm;  // the factor L during the setup ([n][js])
  const int nv = a.n;
  double* const xv = Q + Ly.off_x;
  double* const zv = Q + Ly.off_z;
  double* const dv = Q + Ly.off_d;
  double* const npv = Q + Ly.off_np;
  double* const rv = Q + Ly.off_rv;
  double* const xo = Q + Ly.off_xo;
  // Givens coefficients of rotation g interleaved (c, s, x, applied flag) at gc[4g..4g+3], so
  // a rotation's four are one or two paired LDS accesses
  double* const gc = Q + Ly.off_gc;
#define GC_(g) gc[(g) * 4]
#define GS_(g) gc[(g) * 4 + 1]
#define GX_(g) gc[(g) * 4 + 2]
#define GF_(g) gc[(g) * 4 + 3]  // Givens step applied (1.0) / skipped (0.0)
  double* const uv = Q + Ly.off_u;
  double* const uo = Q + Ly.off_uo;
  double* const sv = Q + Ly.off_s;
  int* const Av = reinterpret_cast<int*>(Q + Ly.off_a);
  int* const Ao = Av + nv + 1;
  uint8_t* const act = reinterpret_cast<uint8_t*>(Q + Ly.off_fl);  // iai[i] == -1
  uint8_t* const exc = act + a.m;                                   // !iaexcl[i]
  Ctl* const ctl = reinterpret_cast<Ctl*>(Q + Ly.off_ctl);

  const int n = a.n, p = a.p, m = a.m, T = a.tile;
  const double inf = dinf();
  const int64_t bb = live ? b : 0;
  const double* Gb = a.G + qbase_rt(bb, n * n, T);
  const double* g0b = a.g0 + qbase_rt(bb, n, T);
  const double* CEb = a.CE + qbase_rt(bb, n * p, T);
  const double* ce0b = a.ce0 + qbase_rt(bb, p, T);
  const double* CIb = a.CI + qbase_rt(bb, n * m, T);
  const double* ci0b = a.ci0 + qbase_rt(bb, m, T);
#define EL(ptr, e) (ptr)[(int64_t)(e) * T]
  // J in LDS: row-major.  J in the workspace (GJR): column-major, so that the row-parallel work
  // (Givens sweeps, update_z, building J) reads and writes it coalesced across lanes.
#define J_(i, j) (GJR ? Jm[(j) * JS + (i)] : Jm[(i) * JS + (j)])
#define R_(i, j) Rm[kPackedR ? rpk((i), (j), n) : (i) * JS + (j)]
#define L_(i, j) Lm[(i) * JS + (j)]
  // setup already in the workspace (qp_panel.hip): start from its header
  const bool pre = GJR && (a.flags & kSetupDone);
  // certification (tolerance mode only): max |x_i| over the run into ctl->xh (kUncXCancel), an
  // LDS atomic per update (a register for it spilled the 128-VGPR workspace kernel)
  // certification: the scale of one s_i's rounding, max ||CI_i||_1 max ||x||_inf + max |ci0_i|
  [[maybe_unused]] auto sigma_s = [&]() -> double {
    const double cim = __builtin_bit_cast(double, (uint64_t)ctl->cim);
    const double c0m = __builtin_bit_cast(double, (uint64_t)ctl->c0m);
    const double xh = __builtin_bit_cast(double, (uint64_t)ctl->xh);
    return cim * xh + c0m;
  };
  auto note_x = [&](double v) {
    if (pre) {
      const double av = fabs(v);
      atomicMax(&ctl->xh, (unsigned long long)__builtin_bit_cast(uint64_t, av < dinf() ? av : 0.0));
    }
  };

  // ------------------------------------------------------------------ setup
  qp_stamp(a, 0);
  if (pre) {
    const double* H = Jm + BigWs<NMAX>::OFF_H;
    if (lead) {
      ctl->iter = 0;
      ctl->steps = 0;
      ctl->fin = 1;
      ctl->status = live ? (int)H[0] : QPGPU_QP_OK;
      ctl->f = H[1];
      ctl->c1 = H[2];
      ctl->c2 = H[3];
      ctl->R_norm = 1.0;
      // certification: a failed or badly spread panel factorization (H[4] = max / min pivot)
      ctl->unc = (ctl->status != QPGPU_QP_OK || !(H[4] <= 1e4)) ? kUncSetup : 0;
      ctl->fmax = fabs(H[1]);
      ctl->xn = ctl->xh = ctl->cim = ctl->c0m = 0ull;
      ctl->iq = 0;
      ctl->phase = live ? PH_SCAN : PH_DONE;
    }
    if (live)
      for (int i = ls; i < n; i += S) xv[i] = H[BigWs<NMAX>::HX + i];
    grp_sync<S>();
    if (live)
      for (int i = ls; i < n; i += S) note_x(xv[i]);  // (ctl->xh was cleared before the sync)
  }
  // G -> R region (becomes L), g0 -> z region
  if (live && !pre) {
    if constexpr (NMAX <= S && NMAX <= 64) {
      // lane j copies column j: every row's load issued at once (one memory latency; rows
      // coalesced across lanes), indices clamped instead of predicated — the clamped loads and
      // stores repeat row n-1 / column n-1 with the same values
      const int jc = ls < n ? ls : n - 1;
      double gv[NMAX];
#pragma unroll
      for (int i = 0; i < NMAX; i++) gv[i] = EL(Gb, (i < n ? i : n - 1) * n + jc);
#pragma unroll
      for (int i = 0; i < NMAX; i++) L_(i < n ? i : n - 1, jc) = gv[i];
    } else {
      for (int e = ls; e < n * n; e += S) {
        const int i = e / n, j = e - (e / n) * n;
        L_(i, j) = EL(Gb, e);
      }
    }
    for (int i = ls; i < n; i += S) zv[i] = EL(g0b, i);
  }
  if (lead && !pre) {
    ctl->unc = 0;
    ctl->status = QPGPU_QP_OK;
    ctl->iter = 0;
    ctl->steps = 0;
    ctl->phase = live ? PH_SCAN : PH_DONE;
    ctl->fin = 1;
  }
  grp_sync<S>();
  if constexpr (kRegSetup) {
    // cholesky_decomposition (@.text+0x2df0) with lane j holding row j of G / L in registers.
    // Step i: sum = A[i][j] - sum_{k=i-1..0} L[i][k] L[j][k] (k descending) on every lane
    // j >= i (lane i: the pivot sum with A[i][i]); L[i][i-1] comes from lane i by v_readlane,
    // the older L[i][k] and the upper G[i][j] from LDS; the pivot is broadcast, every lane takes
    // the same sqrt, and lanes j > i divide.  Column i is published lower and mirrored upper at
    // once, as the reference leaves it after row i.  The inner loops are branch-free (row
    // indices clamped; lanes and entries past n compute values nobody reads) so their loads
    // issue together.
    if (live) {
      if (lead) {
        double c1 = 0.0;
        for (int i = 0; i < n; i++) c1 += L_(i, i);
        ctl->c1 = c1;
      }
      const int j = ls;
      const bool mine = j < n;
      const int jc = mine ? j : n - 1;
      double A[NMAX];
#pragma unroll
      for (int k = 0; k < NMAX; k++) A[k] = L_(jc, k < n ? k : n - 1);
      bool fail = false;
      double bad = 0.0;
#pragma unroll
      for (int i = 0; i < NMAX; i++) {
        if (i < n && !fail) {
          const double lnew = i > 0 ? sg_bcast<S>(A[i > 0 ? i - 1 : 0], i) : 0.0;  // L[i][i-1]
          double lold[NMAX];
#pragma unroll
          for (int k = 0; k + 1 < i; k++) lold[k] = L_(i, k);
          double sum = (j == i) ? A[i] : L_(i, jc);
#pragma unroll
          for (int k = i - 1; k >= 0; k--) sum -= ((k == i - 1) ? lnew : lold[k]) * A[k];
          const double sd = sg_bcast<S>(sum, i);
          if (sd <= 0.0) {
            fail = true;
            bad = sd;
          } else {
            const double dg = sqrt(sd);
            const double v = (j == i) ? dg : wdiv<F>(sum, dg, fok);
            if (mine && j >= i) {
              A[i] = v;
              L_(j, i) = v;
              if (j > i) L_(i, j) = v;
            }
          }
          sg_sync();
        }
      }
      if (lead && fail) {
        ctl->status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
        ctl->f = bad;
      }
    }
    grp_sync<S>();
  } else {
    if (live && !pre) {
      if (lead) {
        double c1 = 0.0;
        for (int i = 0; i < n; i++) c1 += L_(i, i);
        ctl->c1 = c1;
      }
      // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored.
      for (int i = 0; i < n; i++) {
        if (lead) {
          const double sum = seq_fms_down<GJR ? kUG : kUL>(L_(i, i), 0, i, [&](int k) { return L_(i, k); },
                                          [&](int k) { return L_(i, k); });
          if (sum <= 0.0) {
            ctl->status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
            ctl->f = sum;
          } else {
            ctl->t = sqrt(sum);  // the pivot, shared with the subgroup
          }
        }
        grp_sync<S>();
        if (ctl->status != QPGPU_QP_OK) break;
        const double dg = ctl->t;
        for (int j = i + 1 + ls; j < n; j += S) {
          const double s2 = seq_fms_down<GJR ? kUG : kUL>(L_(i, j), 0, i, [&](int k) { return L_(i, k); },
                                         [&](int k) { return L_(j, k); });
          L_(j, i) = wdiv<F>(s2, dg, fok);
        }
        if (lead) L_(i, i) = dg;
        grp_sync<S>();
        for (int k = i + 1 + ls; k < n; k += S) L_(i, k) = L_(k, i);
        grp_sync<S>();
      }
    }
  }
  qp_stamp(a, 1);
  const bool chol_ok = live && ctl->status == QPGPU_QP_OK;
  if (live && !pre && (a.flags & QPGPU_FLAG_WRITE_FACTOR)) {
    double* Gw = a.G + qbase_rt(bb, n * n, T);
    for (int e = ls; e < n * n; e += S) EL(Gw, e) = L_(e / n, e - (e / n) * n);
  }
  if constexpr (kRegSetup) {
    if (chol_ok) {
      const int j = ls;
      const bool mine = j < n;
      const int jc = mine ? j : n - 1;
      // J = L^{-T}: lane r builds row r = (L^{-1} e_r)^T by column-oriented forward
      // substitution: at step q, y_q = s_q / L[q][q], then s_i -= L[i][q] y_q for i > q — for
      // each i the same subtractions in the same (q ascending) order as the reference's row
      // sums.  The reference's literal form throughout (for a finite L its first r entries are
      // +0.0 and subtract exact zeros: the skip of the LDS path changes no bits).  Column q of L
      // is row q of the mirrored upper triangle (contiguous: paired broadcast reads).  The
      // running sums sit in a window that shifts one entry per step (w[k] = s_{q+k}), so the
      // step loop stays rolled with compile-time register indices; entries past n are never
      // stored.
      double w[NMAX];
#pragma unroll
      for (int k = 0; k < NMAX; k++) w[k] = (k == j) ? 1.0 : 0.0;
      {
        for (int q = 0; q < n; q++) {
          const double* Lq = Lm + q * JS + q;  // Lq[k] = L[q+k][q] (k >= 1), Lq[0] = L[q][q]
          double lc[NMAX];
#pragma unroll
          for (int k = 0; k < NMAX; k++) lc[k] = Lq[k];
          const double y = wdiv<F>(w[0], lc[0], fok);
          if (mine) J_(j, q) = y;
#pragma unroll
          for (int k = 0; k + 1 < NMAX; k++) w[k] = w[k + 1] - lc[k + 1] * y;
          w[NMAX - 1] = 0.0;
        }
      }
      // cholesky_solve (@.text+0x31a2) across the lanes: forward y = L^{-1} g0 column-oriented
      // (lane i accumulates its row's subtractions in q order), backward x = L^{-T} y row by row
      // (lane k forms U[k][i] x_i as soon as x_i is broadcast; lane i subtracts them in i+1..n-1
      // order, the reference's; entries past n stay +0.0 and subtract nothing).  Row j of the
      // factor array holds both L[j][q] (q < j) and U[j][i] (i > j).  Divisors broadcast with
      // v_readlane.
      const double diag = L_(jc, jc);
      const double rdiag = F ? wrcp(diag) : 0.0;
      double yv = zv[jc];
      for (int q = 0; q < n; q++) {
        const double lq = L_(jc, q);
        const double yq = sg_bcast<S>(wdiv_r<F>(yv, diag, rdiag, fok), q);
        const double upd = yv - lq * yq;
        yv = (j == q) ? yq : ((j > q) ? upd : yv);
      }
      double Lr[NMAX];
#pragma unroll
      for (int k = 0; k < NMAX; k++) Lr[k] = L_(jc, k);
      double P[NMAX];
#pragma unroll
      for (int k = 0; k < NMAX; k++) P[k] = 0.0;
      double xm = 0.0;
#pragma unroll
      for (int i = NMAX - 1; i >= 0; i--) {
        double v = yv;
#pragma unroll
        for (int k = i + 1; k < NMAX; k++) v -= P[k];
        const double xi = sg_bcast<S>(wdiv_r<F>(v, diag, rdiag, fok), i);
        xm = (j == i) ? xi : xm;
        P[i] = (j < i && i < n) ? Lr[i] * xi : 0.0;
      }
      if (mine) xv[j] = -xm;
      grp_sync<S>();
      if (lead) {
        double c2 = 0.0;
        for (int i = 0; i < n; i++) c2 += J_(i, i);
        ctl->c2 = c2;
        double f = 0.0;
        for (int i = 0; i < n; i++) f += zv[i] * xv[i];
        ctl->f = 0.5 * f;
        ctl->R_norm = 1.0;
        ctl->iq = 0;
      }
      grp_sync<S>();
    }
  } else {
    if (chol_ok && !pre) {
      // J = L^{-T}: lane r builds row r = (L^{-1} e_r)^T in place (J_(r, .) is its own scratch).
      // With a finite L the first r entries are exactly +0.0 and add exact zeros later: skipped
      // (same bits).  A non-finite L takes the literal path.
      if (lead) {
        int fin = 1;
        for (int i = 0; i < n && fin; i++)
          for (int j = 0; j <= i; j++)
            if (!(fabs(L_(i, j)) < inf)) {
              fin = 0;
              break;
            }
        ctl->fin = fin;
      }
      grp_sync<S>();
      const bool skip = ctl->fin != 0;
      for (int r = ls; r < n; r += S) {
        const int i0 = skip ? r : 0;
        for (int i = 0; i < i0; i++) J_(r, i) = 0.0;
        for (int i = i0; i < n; i++) {
          const double v = seq_fms_up<GJR ? kUG : kUL>((i == r) ? 1.0 : 0.0, i0, i, [&](int j) { return L_(i, j); },
                                      [&](int j) { return J_(r, j); });
          J_(r, i) = wdiv<F>(v, L_(i, i), fok);
        }
      }
      grp_sync<S>();
      if (lead) {
        double c2 = 0.0;
        for (int i = 0; i < n; i++) c2 += J_(i, i);
        ctl->c2 = c2;
        // cholesky_solve (@.text+0x31a2): y -> d, x = -G^{-1} g0
        for (int i = 0; i < n; i++) {
          const double v = seq_fms_up<GJR ? kUG : kUL>(zv[i], 0, i, [&](int j) { return L_(i, j); },
                                      [&](int j) { return dv[j]; });
          dv[i] = wdiv<F>(v, L_(i, i), fok);
        }
        for (int i = n - 1; i >= 0; i--) {
          const double v = seq_fms_up<GJR ? kUG : kUL>(dv[i], i + 1, n, [&](int j) { return L_(i, j); },
                                      [&](int j) { return xv[j]; });
          xv[i] = wdiv<F>(v, L_(i, i), fok);
        }
        double f = 0.0;
        for (int i = 0; i < n; i++) {
          xv[i] = -xv[i];
          f += zv[i] * xv[i];
        }
        ctl->f = 0.5 * f;
        ctl->R_norm = 1.0;
        ctl->iq = 0;
      }
      grp_sync<S>();
    }
  }
  if (chol_ok) {
    // R = 0 (L no longer needed), flags
    for (int e = ls; e < (kPackedR ? Ly.nr : n * JS); e += S) Rm[e] = 0.0;
    for (int i = ls; i < m; i += S) act[i] = exc[i] = 0;
    for (int i = ls; i <= n; i += S) {
      uv[i] = 0.0;
      Av[i] = 0;
    }
    grp_sync<S>();
  }

  qp_stamp(a, 2);
  // ------------------------------------------------------------------ shared kernels
  // d = J^T np (lane = column, j ascending); z = J[:, iq:] d[iq:] (lane = row)
  // diagnostic clocks (stamps only): loop phases (scan, select, d/z, lead step, add, delete) and
  // equality-phase parts (d/z, update_r, lead t2 + x/u, add_constraint, the lead's |h| chains)
  uint64_t tph[6] = {0, 0, 0, 0, 0, 0}, teq[5] = {0, 0, 0, 0, 0}, tdet[3] = {0, 0, 0};
  auto clk = [&]() -> uint64_t { return (QPGPU_WAVE_STAMPS && a.stamps) ? __builtin_amdgcn_s_memtime() : 0; };
  // iq0 of an add_constraint whose J sweep was deferred into the next d/z pass, or -1
  // (tolerance mode, QPGPU_WAVE_TOLLOOP bit 2; the same value in every lane).  A QP can finish
  // with a sweep still pending (no violated constraint after a successful add, or the step
  // cap): its J in the workspace is then not the reference's final J.  Nothing reads J after
  // the loop in this mode — J reaches the caller only through QPGPU_FLAG_WRITE_FACTOR (G, the
  // factor, not J) and EXACT runs, and uses_panel() sends both of those to the serial path
  // (defer needs `pre`, which only the panel setup sets).  A future J export from this path
  // must first apply the pending sweep (plain_sweep with iq0 = pend).
  int pend = -1;
  constexpr bool kDefer = GJR && (QPGPU_WAVE_TOLLOOP & 4) && (QPGPU_WAVE_TOLLOOP & 1) && S == 4 * 64 && NMAX <= S;
  // Two deferred sweeps (QPGPU_WAVE_TOLLOOP bit 3): the d/z pass after an add applies the
  // pending sweep A in registers without writing J back; the next add's sweep B joins it and the
  // pass after that applies A then B (B one rotation behind A along each row) and writes the
  // final columns once — each trailing column of J is written once per two adds instead of once
  // per add.  While B is pending, A's coefficients sit in the workspace (gA) because B's occupy
  // gc.  pend2 = B's iq0 or -1; J in memory is current only with nothing pending, so
  // delete_constraint and a degenerate add first apply what is pending.
  constexpr bool kDefer2 = kDefer && (QPGPU_WAVE_TOLLOOP & 8);
  int pend2 = -1;
  [[maybe_unused]] double* const gA = GJR ? Jm + BigWs<NMAX>::OFF_G : nullptr;
  auto compute_d_z = [&](int iq) {
    {
      if constexpr (GJR && (QPGPU_WAVE_TOLLOOP & 1) && S == 4 * 64 && NMAX <= S) {
        if (pre && n >= 2 * kTolCh) {  // the same test as add_constraint's defer
          // tolerance mode: lane r holds row r of each chunk of kDC columns (column-major J:
          // coalesced), d[c] = sum_r J[r][c] np[r] as per-wave tree sums + the four wave partials
          // in wave order (LDS, double-buffered), then z[r] += J[r][c] d[c] for c >= iq from the
          // same registers.  One pass over J.  With a deferred add_constraint sweep (pend = its
          // iq0, QPGPU_WAVE_TOLLOOP bit 2) the pass applies the sweep too: columns below iq0 are
          // read as they are, then each chunk of rotations produces its final columns n-1-g in
          // registers (stored back to J) and their d and z terms, and column iq0 gets the carry.
          constexpr int kDC = kTolCh;
          const int wv = ls >> 6;
          const bool row = ls < n;
          const double npr = row ? npv[ls] : 0.0;
          double* const T = Q + Ly.off_tsc;
          double z = 0.0;
          int buf = 0;
          // d (and z) for the kDC values v of this lane's row; col(u) = their column or -1
          static_assert(kDC == 16, "colsum16 reduces 16 columns per chunk");
          const int c16 = colsum16_col(ls & 63);
          auto chunk = [&](const double* v, auto col) {
            double* const P = T + buf * (4 * kDC);
            buf ^= 1;
            double pv[kDC];
#pragma unroll
            for (int u = 0; u < kDC; u++) pv[u] = v[u] * npr;
            const double w = colsum16(pv);
            if ((ls & 3) == 0) P[wv * kDC + c16] = w;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < kDC; u++) {
              const int c = col(u);
              const double d = ((P[u] + P[kDC + u]) + P[2 * kDC + u]) + P[3 * kDC + u];
              if (ls == 0 && c >= 0) dv[c] = d;
              z += (c >= iq) ? v[u] * d : 0.0;
            }
          };
          const int ps = pend;
          const int cA = ps >= 0 ? ps : n;
          for (int c0 = 0; c0 < cA; c0 += kDC) {
            double jv[kDC];
#pragma unroll
            for (int u = 0; u < kDC; u++) jv[u] = (row && c0 + u < cA) ? J_(ls, c0 + u) : 0.0;
            chunk(jv, [&](int u) { return c0 + u < cA ? c0 + u : -1; });
          }
          if (kDefer2 && ps >= 0 && pend2 >= 0) {
            // A (coefficients in gA, rotations g = 0..ngA-1 on columns (n-2-g, n-1-g)) then B
            // (gc, pend2 = ps + 1, one rotation fewer): A's rotation g yields column n-1-g, which
            // is the t1 of B's rotation g-1 (g = 0: B's initial carry); B's rotation g-1 yields
            // the final column n-g.  The final columns are written back and both are cleared.
            const int ngA = n - 1 - ps;
            double carA = row ? J_(ls, n - 1) : 0.0, carB = 0.0;
            for (int gb = 0; gb < ngA; gb += kDC) {
              double t1v[kDC], fv[kDC];
#pragma unroll
              for (int u = 0; u < kDC; u++) t1v[u] = (row && gb + u < ngA) ? J_(ls, n - 2 - gb - u) : 0.0;
#pragma unroll
              for (int u = 0; u < kDC; u++) {
                const int g = gb + u;
                fv[u] = 0.0;
                if (g < ngA) {
                  const double c = gA[4 * g], sn = gA[4 * g + 1], xn = gA[4 * g + 2];
                  const bool f = gA[4 * g + 3] != 0.0;
                  const double t1 = t1v[u], t2 = carA;
                  const double n1 = t1 * c + t2 * sn;
                  const double eA = f ? xn * (t1 + n1) - t2 : t2;  // column n-1-g after A
                  carA = f ? n1 : t1;
                  if (g == 0) {
                    carB = eA;
                  } else {
                    const int h = g - 1;
                    const double cb = GC_(h), sb_ = GS_(h), xb = GX_(h);
                    const bool fb = GF_(h) != 0.0;
                    const double n2 = eA * cb + carB * sb_;
                    fv[u] = fb ? xb * (eA + n2) - carB : carB;  // final column n-g
                    carB = fb ? n2 : eA;
                    if (row) J_(ls, n - g) = fv[u];
                  }
                }
              }
              chunk(fv, [&](int u) { return (gb + u >= 1 && gb + u < ngA) ? n - gb - u : -1; });
            }
            if (row) {
              J_(ls, ps + 1) = carB;
              J_(ls, ps) = carA;
            }
            double cv[kDC];
#pragma unroll
            for (int u = 0; u < kDC; u++) cv[u] = u == 0 ? carB : (u == 1 ? carA : 0.0);
            chunk(cv, [&](int u) { return u == 0 ? ps + 1 : (u == 1 ? ps : -1); });
            pend = pend2 = -1;
          } else if (ps >= 0) {
            // one pending sweep: applied in registers; with two-deep deferral it stays pending
            // (J is not written back), otherwise its final columns are written now
            const bool keep = kDefer2;
            const int ng = ctl->ngiv;  // = n - 1 - ps
            double carry = row ? J_(ls, n - 1) : 0.0;
            for (int gb = 0; gb < ng; gb += kDC) {
              double t1v[kDC], fv[kDC];
#pragma unroll
              for (int u = 0; u < kDC; u++) t1v[u] = (row && gb + u < ng) ? J_(ls, n - 2 - gb - u) : 0.0;
#pragma unroll
              for (int u = 0; u < kDC; u++) {
                const int g = gb + u;
                fv[u] = 0.0;
                if (g < ng) {
                  const double c = GC_(g), sn = GS_(g), xn = GX_(g);
                  const bool f = GF_(g) != 0.0;
                  const double t1 = t1v[u], t2 = carry;
                  const double n1 = t1 * c + t2 * sn;
                  fv[u] = f ? xn * (t1 + n1) - t2 : t2;
                  carry = f ? n1 : t1;
                  if (row && !keep) J_(ls, n - 1 - g) = fv[u];
                }
              }
              chunk(fv, [&](int u) { return gb + u < ng ? n - 1 - gb - u : -1; });
            }
            if (row && !keep) J_(ls, ps) = carry;
            double cv[kDC];
#pragma unroll
            for (int u = 0; u < kDC; u++) cv[u] = u == 0 ? carry : 0.0;
            chunk(cv, [&](int u) { return u == 0 ? ps : -1; });
            if (!keep) pend = -1;
          }
          if (row) zv[ls] = z;
          grp_sync<S>();
          return;
        }
      }
      for (int c = ls; c < n; c += S)
        dv[c] = GJR ? seq_fma_up<KG>(0.0, 0, n, [&](int j) { return J_(j, c); }, [&](int j) { return npv[j]; })
                    : seq_fma_up_lds<QPGPU_WAVE_KUDZ>(0.0, 0, n, [&](int j) { return J_(j, c); }, [&](int j) { return npv[j]; });
      grp_sync<S>();
      for (int r = ls; r < n; r += S)
        zv[r] = GJR ? seq_fma_up<KG>(0.0, iq, n, [&](int j) { return J_(r, j); }, [&](int j) { return dv[j]; })
                    : seq_fma_up_lds<QPGPU_WAVE_KUDZ>(0.0, iq, n, [&](int j) { return J_(r, j); }, [&](int j) { return dv[j]; });
      grp_sync<S>();
    }
  };
  // update_r (r = R[:iq,:iq]^{-1} d[:iq], rows i descending, each s = sum_{j>i} R[i][j] r[j]
  // with j ascending).  LDS-resident R: the lead alone.  R in the workspace (GJR): wave 0 works
  // as the lead's load/multiply unit — its lanes hold row i-1's R entries (loaded while row i is
  // summed) and, once r[i] is known, write the products R[i][j] r[j] (the same single rounding
  // as the reference's `R[i][j] * r[j]`) to LDS; the lead then adds them in j order.  Called by
  // every lane of the subgroup.  Rows lo..iq-1 only: the loop passes lo = p — the equality
  // constraints' rows of r feed only their multipliers u[0..p), which nothing reads (t1, the
  // dual step's drop and the rollback use the inequalities' u; x and f never use u), and r[i]
  // for i >= p does not depend on the rows below.
  auto update_r = [&](int iq, int lo) {
    if constexpr (!GJR && QPGPU_WAVE_URPF) {
      // row i: s = R[i][i+1] r[i+1] + sum_{j >= i+2} R[i][j] r[j] in j order (the reference's
      // order: +0.0 first, then each product).  r[i+1] stays in a register (no LDS round trip on
      // the chain); the next row's loads (R[i-1][i-1..i+U], d[i-1], r[i+1..i+U]) are
      // unconditional (no exec-mask branch per load) and follow row i's division, before r[i]
      // is stored (issuing them ahead of row i's chain instead measured no faster).  Entries
      // past the row are read (in-bounds LDS, any value) and their products replaced by +0.0:
      // s is never -0.0 (it starts at +0.0 and a sum is -0.0 only from two -0.0 operands), so
      // adding +0.0 leaves it unchanged.
      if (lead && iq > lo) {
        constexpr int U = QPGPU_WAVE_URU;
        auto rowp = [&](int i) -> const double* {
          return kPackedR ? Rm + (i * n - (i * (i - 1)) / 2 - i) : Rm + i * JS;
        };
        double nd, nRii, nrRii, nR1, nR[U], nr[U];  // the next row's values (nrRii: F, 1 / R[i][i])
        // row i's base pointer (Ri[j] = R[i][j]), stepped per row: packed, row i-1 starts
        // n - i entries before row i (no multiplications in the loop)
        const double* Rp = rowp(iq - 1);
        auto prefetch = [&](int i) {
          const double* Ri = Rp;
          nd = dv[i];
          nRii = Ri[i];
          nrRii = F ? wrcp(nRii) : 0.0;  // off the chain: R[i][i] is known before r[i+1]
          nR1 = Ri[i + 1];
#pragma unroll
          for (int u = 0; u < U; u++) {
            nR[u] = Ri[i + 2 + u];
            nr[u] = rv[i + 2 + u];
          }
        };
        prefetch(iq - 1);
        double rn;  // r[i+1]
        {
          // row iq-1: an empty sum (+0.0)
          const double di = nd, Rii = nRii, rRii = nrRii;
          const double r = wdiv_r<F>(di - 0.0, Rii, rRii, fok);
          if (iq > 1) Rp -= kPackedR ? n - (iq - 1) : JS;
          prefetch(iq > 1 ? iq - 2 : 0);
          rv[iq - 1] = r;
          rn = r;
        }
        // rows in two runs: chunk 0 partly past the row (c = iq-i-2 < U: masked), then whole
        // (c >= U: unmasked, longer rows' further chunks with the last one masked)
        auto row = [&](int i, auto Whole) {
          const double di = nd, Rii = nRii, rRii = nrRii, R1 = nR1;
          double cR[U], cr[U];
#pragma unroll
          for (int u = 0; u < U; u++) {
            cR[u] = nR[u];
            cr[u] = nr[u];
          }
          double s = 0.0;
          s += R1 * rn;
          const int c = iq - (i + 2);  // valid entries of chunk 0
#pragma unroll
          for (int u = 0; u < U; u++) {
            const double q = cR[u] * cr[u];
            if constexpr (decltype(Whole)::value)
              s += q;
            else
              s += u < c ? q : 0.0;
          }
          if constexpr (decltype(Whole)::value) {
            if (c > U) {
              const double* Ri = Rp;
              for (int jb = i + 2 + U; jb < iq; jb += U) {
                double aR[U], ar[U];
#pragma unroll
                for (int u = 0; u < U; u++) {
                  aR[u] = Ri[jb + u];
                  ar[u] = rv[jb + u];
                }
                const int cc = iq - jb;
#pragma unroll
                for (int u = 0; u < U; u++) {
                  const double q = aR[u] * ar[u];
                  s += u < cc ? q : 0.0;
                }
              }
            }
          }
          const double r = wdiv_r<F>(di - s, Rii, rRii, fok);
          if (i > 0) Rp -= kPackedR ? n - i : JS;
          prefetch(i > 0 ? i - 1 : 0);  // r[i+1 ..] are in LDS already; r[i] is carried
          rv[i] = r;
          rn = r;
        };
        int i = iq - 2;
        for (; i >= lo && iq - i - 2 < U; i--) row(i, std::false_type{});
        for (; i >= lo; i--) row(i, std::true_type{});
      }
    } else if constexpr (!GJR) {
      if (lead)
        for (int i = iq - 1; i >= lo; i--) {
          // row i of R as a pointer (Ri[j] = R[i][j], j >= i): packed rows are contiguous too
          const double* Ri = kPackedR ? Rm + (i * n - (i * (i - 1)) / 2 - i) : Rm + i * JS;
          const double s = seq_fma_up<kUL>(0.0, i + 1, iq, [&](int j) { return Ri[j]; },
                                      [&](int j) { return rv[j]; });
          rv[i] = wdiv<F>(dv[i] - s, Ri[i], fok);
        }
    } else {
      if (ls >= 64) return;  // waves 1.. idle (they wait at the caller's grp_sync)
      constexpr int PU = (NMAX + 63) / 64;
      if constexpr (QPGPU_WAVE_TOLLOOP & 2) {
        if (pre) {
          // tolerance mode: lane l holds r[j] for j = l + 64u in registers; row i's products
          // R[i][j] r[j] (j in (i, iq)) are summed by the wave's tree (wave_sum_f64), so each row
          // costs a tree sum and a division.  Rows are fetched kRD ahead (a register ring with
          // compile-time slots) so the global loads' latency is off the chain.
          constexpr int kRD = 4;
          double rr[PU], ring[kRD][PU], rd[kRD], rg[kRD];
#pragma unroll
          for (int u = 0; u < PU; u++) rr[u] = 0.0;
          auto fetch_row = [&](int i, double* dst, double& di, double& gi) {
#pragma unroll
            for (int u = 0; u < PU; u++) {
              const int j = ls + 64 * u;
              dst[u] = (i >= 0 && j > i && j < iq) ? R_(i, j) : 0.0;
            }
            di = i >= 0 ? dv[i] : 0.0;
            gi = i >= 0 ? R_(i, i) : 1.0;
          };
#pragma unroll
          for (int k = 0; k < kRD; k++) fetch_row(iq - 1 - k, ring[k], rd[k], rg[k]);
          for (int i0 = iq - 1; i0 >= lo; i0 -= kRD) {
#pragma unroll
            for (int k = 0; k < kRD; k++) {
              const int i = i0 - k;
              if (i < lo) break;
              double rc[PU];
#pragma unroll
              for (int u = 0; u < PU; u++) rc[u] = ring[k][u];
              const double di = rd[k], gi = rg[k];
              fetch_row(i - kRD, ring[k], rd[k], rg[k]);
              double sl = 0.0;
#pragma unroll
              for (int u = 0; u < PU; u++) {
                const int j = ls + 64 * u;
                sl += (j > i && j < iq) ? rc[u] * rr[u] : 0.0;
              }
              const double ri = (di - wave_sum_f64(sl)) / gi;
#pragma unroll
              for (int u = 0; u < PU; u++)
                if (ls + 64 * u == i) rr[u] = ri;
              if (lead) rv[i] = ri;
            }
          }
          sg_sync();
          return;
        }
      }
      double* const P = gc;  // scratch (the Givens buffers are free during a step)
      double rn[PU], rc[PU];
      auto fetch = [&](int i) {
#pragma unroll
        for (int u = 0; u < PU; u++) {
          const int j = i + 1 + ls + 64 * u;
          rn[u] = (i >= 0 && j < iq) ? R_(i, j) : 0.0;
        }
      };
      fetch(iq - 1);
      for (int i = iq - 1; i >= lo; i--) {
#pragma unroll
        for (int u = 0; u < PU; u++) rc[u] = rn[u];
        fetch(i - 1);  // in flight while row i is finished
#pragma unroll
        for (int u = 0; u < PU; u++) {
          const int j = i + 1 + ls + 64 * u;
          if (j < iq) P[j] = rc[u] * rv[j];
        }
        sg_sync();
        if (lead) {
          double s = 0.0;
          int j = i + 1;
          for (; j + 4 <= iq; j += 4) {
            const double p0 = P[j], p1 = P[j + 1], p2 = P[j + 2], p3 = P[j + 3];
            s += p0;
            s += p1;
            s += p2;
            s += p3;
          }
          for (; j < iq; j++) s += P[j];
          rv[i] = (dv[i] - s) / R_(i, i);
        }
        sg_sync();
      }
    }
  };
  // the lead's two step dot products z.z and z.np, one pass (two independent chains)
  auto dot2_lead = [&](double& zz, double& znp, double* npx = nullptr) {
    double s1 = 0.0, s2 = 0.0, s3 = 0.0;
    constexpr int U = 8;  // loads of a chunk issued together (the adds stay in i order)
    // full chunks, then the last one with unconditional loads (in-bounds LDS past n) and its
    // products past n replaced by +0.0: the sums start at +0.0, so they are never -0.0 and
    // adding +0.0 leaves them unchanged
    auto chunk = [&](int ib, int c) {
      double zc[U], pc[U], xc[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        zc[u] = zv[ib + u];
        pc[u] = npv[ib + u];
        if (npx) xc[u] = xv[ib + u];
      }
#pragma unroll
      for (int u = 0; u < U; u++) {
        const double q1 = zc[u] * zc[u], q2 = zc[u] * pc[u];
        s1 += u < c ? q1 : 0.0;
        s2 += u < c ? q2 : 0.0;
        if (npx) {
          const double q3 = pc[u] * xc[u];
          s3 += u < c ? q3 : 0.0;
        }
      }
    };
    int ib = 0;
    for (; ib + U <= n; ib += U) chunk(ib, U);
    if (ib < n) chunk(ib, n - ib);
    zz = s1;
    znp = s2;
    if (npx) *npx = s3;
  };
  // add_constraint (@.text+0x21fd), split in three:
  //  1. the lead runs the serial part of the d-chain.  Rotation g (j = n-1-g) computes
  //     h = distance(d[j-1], d[j]), and distance() reads magnitudes only, while the rotated d[j-1]
  //     is +-h; so the chain of h values needs nothing but the previous |h| (or, after a skipped
  //     |h| < eps step, the untouched d[j-1]).  The lead records h (gx) and applied/skipped (gf);
  //  2. lane g rebuilds rotation g's inputs exactly as the reference sees them (d[j-1] is still
  //     the original; d[j] is the original, or +-h of rotation g-1 with the sign of
  //     d[j] / h_{g-1}) and evaluates the same cc = d[j-1]/h, ss = d[j]/h, sign flip and
  //     xny = ss/(1+cc) as the reference — every rotation in parallel, bit for bit;
  //  3. every lane applies the rotations to its rows of J in order; the lead finishes with
  //     R[:iq, iq-1] = d and the degeneracy test.  Returns through ctl->fin (1 = added).
  static_assert(S >= NMAX, "one lane per rotation");
  // Fast build, LDS variants: the |h| chain from one prefix sum of squares over the subgroup.
  // Without a skipped step, distance(a, b) = sqrt(a^2 + b^2) and the carried value is the previous
  // h, so h_g^2 = d[n-1]^2 + sum_{k<=g} d[n-2-k]^2: lane g takes its square, an inclusive scan
  // over the subgroup (log2 S shuffles) gives every h at once instead of n-1-iq dependent
  // hypots on the lead (the largest serial chain left in the equality phase: 25-28k of the mgqp
  // level's 110k cycles per wave, profiles/r04_s26).  h grows with g, so a step can be skipped
  // (|h| < eps) only if the first one is: that case and squares outside the fast forms' range
  // take the serial chain.  Within north_star's 1e-10 like the rest of the fast build.
  auto h_prefix = [&](int iq) -> bool {
    if constexpr (F && !GJR && S <= 64) {
      const int ng = iq < n - 1 ? n - 1 - iq : 0;
      const int g = ls;
      const double ag = g < ng ? dv[n - 2 - g] : 0.0;
      double v = ag * ag;
#pragma unroll
      for (int o = 1; o < S; o <<= 1) {
        const double t = __shfl_up(v, o, S);
        v += ls >= o ? t : 0.0;
      }
      const double d0 = ng > 0 ? dv[n - 1] : 0.0;
      const double P = __builtin_fma(d0, d0, v);
      const bool bad = g < ng && (!(P >= 0x1p-600 && P <= 0x1p600) || (g == 0 && P < 4.0 * kEps * kEps));
      const uint64_t bm = __builtin_amdgcn_ballot_w64(bad);
      const int sgb = (S >= 64) ? 0 : (int)(threadIdx.x & 63) & ~(S - 1);
      const uint64_t sgm = (S >= 64) ? ~0ull : ((1ull << (S & 63)) - 1) << sgb;
      if (bm & sgm) return false;  // this QP's lanes take the serial chain
      if (g < ng) {
        GX_(g) = sqrt(P);
        GF_(g) = 1.0;
      }
      if (lead) ctl->ngiv = ng;
      return true;
    } else if constexpr (GJR && S == 4 * 64) {
      // tolerance mode of the workspace variant: the same prefix sum of squares over the block
      // (a scan per wave, then the waves' totals in wave order), so the |h| chain — n-1-iq
      // dependent hypots on the lead, 7 % of the C5 loop (profiles/r06_s3) — becomes one scan and
      // one square root per lane.  A possibly skipped first step (h < 2 eps) or squares outside
      // [2^-600, 2^600] take the serial chain, as in the fast build.
      if (!pre) return false;
      const int ng = iq < n - 1 ? n - 1 - iq : 0;
      const int g = ls;
      const double ag = g < ng ? dv[n - 2 - g] : 0.0;
      double v = ag * ag;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double t = __shfl_up(v, o, 64);
        v += (ls & 63) >= o ? t : 0.0;
      }
      double* const W = Q + Ly.off_tsc;  // (not live between the d/z passes)
      if ((ls & 63) == 63) W[ls >> 6] = v;
      __syncthreads();
      const double d0 = ng > 0 ? dv[n - 1] : 0.0;
      double P = d0 * d0;
      for (int w = 0; w < (ls >> 6); w++) P += W[w];
      P += v;
      const bool bad = g < ng && (!(P >= 0x1p-600 && P <= 0x1p600) || (g == 0 && P < 4.0 * kEps * kEps) ||
                                  !(fabs(ag) <= 0x1p300));
      if (__syncthreads_or(bad)) return false;  // this QP takes the serial chain
      if (g < ng) {
        GX_(g) = sqrt(P);
        GF_(g) = 1.0;
      }
      if (lead) ctl->ngiv = ng;
      return true;
    } else {
      return false;
    }
  };
  // J's trailing columns swept in memory by a recorded set of rotations (coef: 4 per rotation,
  // as gc) — plain_sweep's arithmetic with the coefficients taken from `coef`
  [[maybe_unused]] auto sweep_coef = [&](const double* coef, int ng) {
    for (int k = ls; k < n; k += S) {
      double carry = J_(k, n - 1);
      for (int g = 0; g < ng; g++) {
        const double t1 = J_(k, n - 2 - g), t2 = carry;
        const double c = coef[4 * g], sn = coef[4 * g + 1], xn = coef[4 * g + 2];
        const bool f = coef[4 * g + 3] != 0.0;
        const double n1 = t1 * c + t2 * sn;
        J_(k, n - 1 - g) = f ? xn * (t1 + n1) - t2 : t2;
        carry = f ? n1 : t1;
      }
      J_(k, n - 1 - ng) = carry;
    }
  };
  auto add_constraint = [&]() {
    const uint64_t h0 = clk();
    if constexpr (kDefer2) {
      // a sweep is pending (its coefficients in gc): they move to the workspace before this
      // add's rotations are recorded in gc
      if (pend >= 0) {
        const int ngA = n - 1 - pend;
        for (int e = ls; e < 4 * ngA; e += S) gA[e] = gc[e];
        grp_sync<S>();
      }
    }
    const bool hp = h_prefix(ctl->iq);
    if (lead && !hp) {
      const int iq = ctl->iq;
      int ng = 0;
      if (QPGPU_WAVE_HCHAIN2 && iq < n) {
        // full chunks of U rotations without per-rotation exec-mask branches (the chunk's d
        // values loaded together), then the tail one rotation per trip; distance() with the
        // range-reduced sqrt (qp_common.h)
        double carried = dv[n - 1];
        constexpr int U = QPGPU_WAVE_HCU;
        int jb = n - 1;
        for (; jb - U >= iq; jb -= U) {
          double ac[U];
#pragma unroll
          for (int u = 0; u < U; u++) ac[u] = dv[jb - u - 1];
#pragma unroll
          for (int u = 0; u < U; u++) {
            const double a0 = ac[u];
            const double h = wdist<F>(a0, carried, fok);
            const bool skip = fabs(h) < kEps;
            GF_(ng + u) = skip ? 0.0 : 1.0;
            GX_(ng + u) = h;
            carried = skip ? a0 : h;
          }
          ng += U;
        }
        for (; jb >= iq + 1; jb--) {
          const double a0 = dv[jb - 1];
          const double h = wdist<F>(a0, carried, fok);
          const bool skip = fabs(h) < kEps;
          GF_(ng) = skip ? 0.0 : 1.0;
          GX_(ng) = h;
          carried = skip ? a0 : h;
          ng++;
        }
      } else if (iq < n) {
        double carried = dv[n - 1];
        constexpr int U = 8;  // d values of a chunk loaded together, ahead of the h chain
        for (int jb = n - 1; jb >= iq + 1; jb -= U) {
          double ac[U];
#pragma unroll
          for (int u = 0; u < U; u++) ac[u] = jb - u >= iq + 1 ? dv[jb - u - 1] : 0.0;
#pragma unroll
          for (int u = 0; u < U; u++)
            if (jb - u >= iq + 1) {
              const double a0 = ac[u];
              const double h = wdist<F>(a0, carried, fok);
              const bool skip = fabs(h) < kEps;
              GF_(ng) = skip ? 0.0 : 1.0;
              GX_(ng) = h;
              carried = skip ? a0 : h;
              ng++;
            }
        }
      }
      ctl->ngiv = ng;
    }
    grp_sync<S>();
    teq[4] += clk() - h0;
    {
      const int ng = ctl->ngiv, g = ls;
      const bool mine = g < ng;
      // branch-free: every lane evaluates both branches of the reference's rotation with its
      // index clamped (lanes past ng compute values nobody stores) and selects
      const int gm = mine ? g : 0, gp = gm > 0 ? gm - 1 : 0;
      const int j = n - 1 - gm;
      const double h = GX_(gm), cc_raw = dv[j - 1], dj = dv[j], hp = GX_(gp);
      const bool prev = gm > 0 && GF_(gp) != 0.0, app = GF_(gm) != 0.0;
      // (F: hp > 0 for an applied previous step, so dj / hp < 0 is dj < 0; only applied
      // rotations of this QP count for the range checks)
      bool rok = true;
      const bool dneg = F ? (dj < 0.0) : (dj / hp < 0.0);
      const double ss_raw = prev ? (dneg ? -hp : hp) : dj;
      const double rh = F ? wrcp(h) : 0.0;
      double ss1 = wdiv_r<F>(ss_raw, h, rh, rok), cc1 = wdiv_r<F>(cc_raw, h, rh, rok);
      const bool neg = cc1 < 0.0;
      cc1 = neg ? -cc1 : cc1;
      ss1 = neg ? -ss1 : ss1;
      const double x1 = wdiv<F>(ss1, 1.0 + cc1, rok);
      if (F && mine && app) fok = fok && rok;
      const double cc = app ? cc1 : 0.0, ss = app ? ss1 : 0.0, xny = app ? x1 : 0.0;
      const double dlast = app ? (neg ? -h : h) : cc_raw;
      grp_sync<S>();
      if (mine) {
        GC_(g) = cc;
        GS_(g) = ss;
        GX_(g) = xny;
        if (g == ng - 1) dv[n - 1 - g - 1] = dlast;  // d[iq] after the sweep
      }
    }
    grp_sync<S>();
    const uint64_t h1 = clk();
    if (QPGPU_WAVE_STAMPS_DETAIL == 2) tdet[0] += h1 - h0;
    const int iq0 = ctl->iq;
    // tolerance mode: the J sweep waits for the next d/z pass (which reads J anyway) unless the
    // constraint turns out degenerate (then delete_constraint needs the swept J right away)
    const bool defer = kDefer && pre && n >= 2 * kTolCh;
    auto plain_sweep = [&]() {
      // Row k's sweep over columns n-1 .. iq: rotation g maps (J[k][j-1], J[k][j]), j = n-1-g,
      // to (n1, xny (t1 + n1) - t2) and n1 is the next rotation's t2, so it is carried in a
      // register and the t1 loads (independent of the chain) are issued kU at a time.
      constexpr bool kGC = false;  // (coefficients per chunk in the workspace variant: removed)
      constexpr int kU = GJR ? KG : QPGPU_WAVE_KUJ;
      const int ng = ctl->ngiv;
      for (int k = ls; k < n; k += S) {
        double carry = J_(k, n - 1);
        for (int gb = 0; gb < ng; gb += kU) {
          // the chunk's J entries (and, with J in LDS, its rotation coefficients) are loaded
          // before its first store (LDS stores would otherwise fence every later load); the
          // workspace variant reads the coefficients per rotation (registers: its occupancy)
          constexpr int kUC = (GJR && !kGC) ? 1 : kU;
          double t1v[kU], cv[kUC], sw[kUC], xw[kUC];
          bool fw[kUC];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int g = gb + u;
            const bool ok = g < ng;
            t1v[u] = ok ? J_(k, n - 2 - g) : 0.0;
            if constexpr (!GJR || kGC) {
              cv[u] = ok ? GC_(g) : 0.0;
              sw[u] = ok ? GS_(g) : 0.0;
              xw[u] = ok ? GX_(g) : 0.0;
              fw[u] = ok && GF_(g) != 0.0;
            }
          }
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int g = gb + u;
            if (g < ng) {
              const int uc = (GJR && !kGC) ? 0 : u;
              if constexpr (GJR && !kGC) {
                cv[0] = GC_(g);
                sw[0] = GS_(g);
                xw[0] = GX_(g);
                fw[0] = GF_(g) != 0.0;
              }
              const double t1 = t1v[u], t2 = carry;
              const double n1 = t1 * cv[uc] + t2 * sw[uc];
              // skipped step (gf = 0): both columns unchanged
              J_(k, n - 1 - g) = fw[uc] ? xw[uc] * (t1 + n1) - t2 : t2;
              carry = fw[uc] ? n1 : t1;
            }
          }
        }
        J_(k, n - 1 - ng) = carry;
      }
    };
    if (!GJR && QPGPU_WAVE_SWEEP2 && iq0 < n) {
      // the sweep below with J in LDS: full chunks of kU rotations with no per-rotation
      // exec-mask branch (the chunk's J entries and coefficients loaded first), then the tail
      // one rotation per trip
      constexpr int kU = QPGPU_WAVE_KUJ;
      const int ng = ctl->ngiv;
      for (int k = ls; k < n; k += S) {
        double carry = J_(k, n - 1);
        int g = 0;
        for (; g + kU <= ng; g += kU) {
          double t1v[kU], cv[kU], sw[kU], xw[kU];
          bool fw[kU];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            t1v[u] = J_(k, n - 2 - g - u);
            cv[u] = GC_(g + u);
            sw[u] = GS_(g + u);
            xw[u] = GX_(g + u);
            fw[u] = GF_(g + u) != 0.0;
          }
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const double t1 = t1v[u], t2 = carry;
            const double n1 = t1 * cv[u] + t2 * sw[u];
            J_(k, n - 1 - g - u) = fw[u] ? xw[u] * (t1 + n1) - t2 : t2;
            carry = fw[u] ? n1 : t1;
          }
        }
        for (; g < ng; g++) {
          const double t1 = J_(k, n - 2 - g), t2 = carry;
          const double c = GC_(g), sn = GS_(g), xn = GX_(g);
          const bool f = GF_(g) != 0.0;
          const double n1 = t1 * c + t2 * sn;
          J_(k, n - 1 - g) = f ? xn * (t1 + n1) - t2 : t2;
          carry = f ? n1 : t1;
        }
        J_(k, n - 1 - ng) = carry;
      }
    } else if (iq0 < n && !defer) {
      plain_sweep();
    }
    grp_sync<S>();
    const uint64_t h2 = clk();
    if (QPGPU_WAVE_STAMPS_DETAIL == 2) tdet[1] += h2 - h1;
    if (iq0 < n)  // R[:iq+1, iq] = d[:iq+1], one entry per lane
      for (int i = ls; i <= iq0; i += S) R_(i, iq0) = dv[i];
    if (lead) {
      int iq = ctl->iq;
      if (iq >= n) {
        ctl->fin = 0;  // reference UB (p > n); reported as dependent
      } else {
        iq++;
        ctl->iq = iq;
        const double dd = fabs(dv[iq - 1]);
        if (pre && dd <= 1e6 * kEps * ctl->R_norm) ctl->unc |= kUncDependent;
        if (dd <= kEps * ctl->R_norm) {
          ctl->fin = 0;
        } else {
          ctl->R_norm = (ctl->R_norm < dd) ? dd : ctl->R_norm;
          ctl->fin = 1;
        }
      }
    }
    grp_sync<S>();
    if (defer && iq0 < n) {
      if (ctl->fin) {
        if (kDefer2 && pend >= 0)
          pend2 = iq0;  // = pend + 1: the d/z pass applies both and writes J back
        else
          pend = iq0;
      } else {
        // degenerate: delete_constraint needs the current J — the pending sweep (its
        // coefficients now in gA), then this one
        if (kDefer2 && pend >= 0) {
          sweep_coef(gA, n - 1 - pend);
          grp_sync<S>();
          pend = -1;
        }
        plain_sweep();
        grp_sync<S>();
      }
    }
    if (QPGPU_WAVE_STAMPS_DETAIL == 2) tdet[2] += clk() - h2;
  };
  // delete_constraint (@.text+0x26a8) of constraint l: the lead does the bookkeeping and the
  // R re-triangularisation (recording the rotations), the lanes shift R's rows and rotate
  // J's columns.
  auto delete_constraint = [&](int l) {
    if constexpr (kDefer2) {
      // J must be current: a sweep kept pending by the last d/z pass (its coefficients still in
      // gc: no add since) is applied now
      if (pend >= 0) {
        sweep_coef(gc, n - 1 - pend);
        grp_sync<S>();
        pend = -1;
      }
    }
    if (lead) {
      const int iq = ctl->iq;
      int qq = 0;
      for (int i = p; i < iq; i++)
        if (Av[i] == l) {
          qq = i;
          break;
        }
      for (int i = qq; i < iq - 1; i++) {
        Av[i] = Av[i + 1];
        uv[i] = uv[i + 1];
      }
      Av[iq - 1] = Av[iq];
      uv[iq - 1] = uv[iq];
      Av[iq] = 0;
      uv[iq] = 0.0;
      ctl->qq = qq;
    }
    grp_sync<S>();
    {
      const int iq = ctl->iq, qq = ctl->qq;
      for (int j = ls; j < n; j += S) {
        for (int i = qq; i < iq - 1; i++) R_(j, i) = R_(j, i + 1);
        if (j < iq) R_(j, iq - 1) = 0.0;
      }
    }
    grp_sync<S>();
    if (lead) {
      const int iq = --ctl->iq;
      const int qq = ctl->qq;
      int ng = 0;
      if (iq > 0) {
        for (int j = qq; j < iq; j++) {
          double cc = R_(j, j), ss = R_(j + 1, j);
          const double h = wdist<F>(cc, ss, fok);
          if (pre && fabs(h) >= 0.25 * kEps && fabs(h) <= 4.0 * kEps) ctl->unc |= kUncGivens;
          if (fabs(h) < kEps) {
            GF_(ng++) = 0.0;
            continue;
          }
          const double rh = F ? wrcp(h) : 0.0;
          cc = wdiv_r<F>(cc, h, rh, fok);
          ss = wdiv_r<F>(ss, h, rh, fok);
          R_(j + 1, j) = 0.0;
          if (cc < 0.0) {
            R_(j, j) = -h;
            cc = -cc;
            ss = -ss;
          } else {
            R_(j, j) = h;
          }
          const double xny = wdiv<F>(ss, 1.0 + cc, fok);
          for (int k = j + 1; k < iq; k++) {
            const double t1 = R_(j, k), t2 = R_(j + 1, k);
            const double r1 = t1 * cc + t2 * ss;
            R_(j, k) = r1;
            R_(j + 1, k) = xny * (t1 + r1) - t2;
          }
          GC_(ng) = cc;
          GS_(ng) = ss;
          GX_(ng) = xny;
          GF_(ng++) = 1.0;
        }
      }
      ctl->ngiv = ng;
    }
    grp_sync<S>();
    {
      // row k's sweep over columns qq .. qq+ng: rotation g maps (J[k][j], J[k][j+1]), j = qq+g,
      // to (n1, xny (n1 + t1) - t2); the second is the next rotation's t1 (carried)
      constexpr int kU = GJR ? KG : QPGPU_WAVE_KUJ;
      const int ng = ctl->ngiv, qq = ctl->qq;
      for (int k = ls; k < n; k += S) {
        double carry = J_(k, qq);
        for (int gb = 0; gb < ng; gb += kU) {
          constexpr int kUC = GJR ? 1 : kU;
          double t2v[kU], cv[kUC], sw[kUC], xw[kUC];
          bool fw[kUC];
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int g = gb + u;
            const bool ok = g < ng;
            t2v[u] = ok ? J_(k, qq + g + 1) : 0.0;
            if constexpr (!GJR) {
              cv[u] = ok ? GC_(g) : 0.0;
              sw[u] = ok ? GS_(g) : 0.0;
              xw[u] = ok ? GX_(g) : 0.0;
              fw[u] = ok && GF_(g) != 0.0;
            }
          }
#pragma unroll
          for (int u = 0; u < kU; u++) {
            const int g = gb + u;
            if (g < ng) {
              const int uc = GJR ? 0 : u;
              if constexpr (GJR) {
                cv[0] = GC_(g);
                sw[0] = GS_(g);
                xw[0] = GX_(g);
                fw[0] = GF_(g) != 0.0;
              }
              const double t1 = carry, t2 = t2v[u];
              const double n1 = t1 * cv[uc] + t2 * sw[uc];
              J_(k, qq + g) = fw[uc] ? n1 : t1;
              carry = fw[uc] ? xw[uc] * (n1 + t1) - t2 : t2;
            }
          }
        }
        J_(k, qq + ng) = carry;
      }
    }
    grp_sync<S>();
  };

  // ------------------------------------------------------------------ equality phase
  if (chol_ok) {
    // step i+1's column of CE (lane j: CE[j][i+1]) and ce0[i+1] are loaded during step i, so no
    // step waits on global memory (S >= NMAX: at most one row per lane)
    double np_next = (ls < n && p > 0) ? EL(CEb, ls * p) : 0.0;
    double c0_next = (p > 0) ? EL(ce0b, 0) : 0.0;
    for (int i = 0; i < p; i++) {
      if (ls < n) npv[ls] = np_next;
      const double c0 = c0_next;
      if (i + 1 < p) {
        np_next = ls < n ? EL(CEb, ls * p + i + 1) : 0.0;
        c0_next = EL(ce0b, i + 1);
      }
      grp_sync<S>();
      const uint64_t e0 = clk();
      compute_d_z(ctl->iq);
      const uint64_t e1 = clk();
      // (no update_r and no u[:iq] update in the equality phase: r and the equality constraints'
      // multipliers feed nothing, see update_r)
      const uint64_t e2 = clk();
      teq[0] += e1 - e0;
      teq[1] += e2 - e1;
      if (lead) {
        const int iq = ctl->iq;
        double t2 = 0.0, zz, znp, npx;
        dot2_lead(zz, znp, &npx);  // np.x in the same pass (the reference's np.x, i ascending)
        if (fabs(zz) > kEps) t2 = wdiv<F>(-npx - c0, znp, fok);
        ctl->t2 = t2;
        uv[iq] = t2;
        ctl->f += 0.5 * (t2 * t2) * znp;
        if (pre) {
          if (fabs(zz) >= 0.25 * kEps && fabs(zz) <= 4.0 * kEps) ctl->unc |= kUncZz;
          ctl->fmax = fmax(ctl->fmax, fabs(ctl->f));
        }
        Av[i] = -i - 1;
      }
      grp_sync<S>();
      {
        const double t2 = ctl->t2;
        for (int k = ls; k < n; k += S) {
          xv[k] += t2 * zv[k];
          note_x(xv[k]);
        }
      }
      const uint64_t e3 = clk();
      teq[2] += e3 - e2;
      add_constraint();
      teq[3] += clk() - e3;
      if (!ctl->fin) {
        if (lead) {
          ctl->status = QPGPU_QP_DEPENDENT;
          ctl->phase = PH_DONE;
        }
        grp_sync<S>();
        break;
      }
    }
  } else if (lead) {
    ctl->phase = PH_DONE;
  }
  grp_sync<S>();
  if (a.x_eq && live) {  // the m = 0 answer: an empty l1 scan returns right here
    const int st = ctl->status;
    if (st != QPGPU_QP_NOT_POSITIVE_DEFINITE) {
      double* xb = a.x_eq + qbase_rt(bb, n, T);
      for (int i = ls; i < n; i += S) EL(xb, i) = xv[i];
    }
    if (lead) {
      a.f_eq[b] = ctl->f;
      a.st_eq[b] = st;
    }
  }

  qp_stamp(a, 3);
  if (any_bad()) return false;  // the fast attempt's setup / equality phase went out of range
  if (GJR && pre && live) {
    // certification: the scales of the s_i's rounding (sigma_s), one extra read of CI per QP
    for (int i = ls; i < m; i += S) {
      double a1 = 0.0;
      for (int j = 0; j < n; j++) a1 += fabs(EL(CIb, j * m + i));
      const double c0 = fabs(EL(ci0b, i));
      atomicMax(&ctl->cim, (unsigned long long)__builtin_bit_cast(uint64_t, a1));
      atomicMax(&ctl->c0m, (unsigned long long)__builtin_bit_cast(uint64_t, c0));
    }
    grp_sync<S>();
  }
  // ------------------------------------------------------------------ active-set loop
  // ---- the tolerance-mode l1 scan from the fp32 copy of CI (QPGPU_WAVE_SHADOW; workspace
  // variant).  Each lane's s~_i = fl(sum_j (double)CI32[j][i] x_j) + ci0_i in j order, with a bound
  // B_i >= |s_i - s~_i| for the fp64 scan's s_i: CI32 = CI (1 + d), |d| <= 2^-24, or |CI32 - CI|
  // <= 2^-126 below fp32's normal range, and both sums' rounding (each <= (n + 1) eps' of
  // sum |CI_ij x_j| + |ci0_i|), and products below the normal range — B_i = 1.001 (5.97e-8 A_i +
  // 2e-38 sum|x| + 1e-13 |ci0_i|) + 1e-300, A_i = sum |CI32_ij x_j|.  Accepted (true) only when
  //   * every s~_i and B_i is finite,
  //   * |psi~| - E > 1.001 thr + 1e-10 sigma_s m, where psi~ sums the negative s~_i and E bounds
  //     |psi - psi~| (1.001 x the B_i of every constraint that may be negative, plus both sums'
  //     rounding, 4e-16 m sum |s~_i| over them): the fp64 psi then continues the loop and stays
  //     outside kUncPsi's window;
  //   * at most kShadowCand constraints are candidates: not active, lower bound below 0 and not
  //     above H2, the second-smallest upper bound among those — the two smallest fp64 values are
  //     among them, so the select's pick, its runner-up (kUncSelTie) and any re-select after a
  //     degenerate add (which compares against the carried ss, itself a candidate's value) come
  //     out as from the fp64 scan, the other s~_i lying above every value they are compared with.
  // The candidates get their fp64 s_i (the same products and the same j-order sum as the fp64
  // scan: the lanes form the n products, the lead adds them) into sv; the other sv entries keep
  // s~_i.  Otherwise (false) the caller scans in fp64, overwriting sv.
  constexpr bool kShadow = GJR && QPGPU_WAVE_SHADOW && S == 4 * 64 && NMAX <= S;
  bool shadow_hit = false;
  [[maybe_unused]] auto shadow_scan = [&]() -> bool {
    constexpr int KS = (MMAX + S - 1) / S;  // constraints per lane
    const float* const C32 = reinterpret_cast<const float*>(ws + a.batch * (int64_t)C::WS_DOUBLES) + bb * (int64_t)n * m;
    double* const W = Q + Ly.off_tsc;  // (not live between the d/z passes)
    double* const P = Q + Ly.off_sp;
    int* const cl = reinterpret_cast<int*>(P + n);  // [0] count, [1..kShadowCand] candidates
    if (lead) cl[0] = 0;
    double bk[KS];  // (s~_i is read back from sv)
    double lpsi = 0.0, le = 0.0, les = 0.0;
    bool lbad = false;
    // KP of a lane's constraints per pass over j (their loads of a chunk in flight together)
    constexpr int KP = QPGPU_WAVE_SHADOW_KP < KS ? QPGPU_WAVE_SHADOW_KP : KS;
    static_assert(KS % KP == 0, "constraints per lane in whole groups");
#pragma unroll
    for (int k0 = 0; k0 < KS; k0 += KP) {
      if (ls + k0 * S < m) {
        double sa[KP], Aa[KP], X = 0.0;
        int ia[KP];
#pragma unroll
        for (int q = 0; q < KP; q++) {
          sa[q] = 0.0;
          Aa[q] = 0.0;
          ia[q] = ls + (k0 + q) * S < m ? ls + (k0 + q) * S : m - 1;  // (a clamped one is discarded)
        }
        constexpr int U = QPGPU_WAVE_SHADOW_U;
        for (int jb = 0; jb < n; jb += U) {
          float c[KP][U];
#pragma unroll
          for (int q = 0; q < KP; q++)
#pragma unroll
            for (int u = 0; u < U; u++) c[q][u] = C32[(jb + u < n ? jb + u : n - 1) * m + ia[q]];
#pragma unroll
          for (int u = 0; u < U; u++)
            if (jb + u < n) {
              const double xj = xv[jb + u];
              X += fabs(xj);
#pragma unroll
              for (int q = 0; q < KP; q++) {
                const double cd = (double)c[q][u];
                sa[q] += cd * xj;
                Aa[q] += fabs(cd) * fabs(xj);
              }
            }
        }
#pragma unroll
        for (int q = 0; q < KP; q++) {
          const int i = ls + (k0 + q) * S;
          bk[k0 + q] = 0.0;
          if (i < m) {
            const double c0 = EL(ci0b, i);
            const double s = sa[q] + c0;
            const double B = 1.001 * (5.97e-8 * Aa[q] + 2e-38 * X + 1e-13 * fabs(c0)) + 1e-300;
            lbad = lbad || !(fabs(s) < inf && B < inf);
            sv[i] = s;
            exc[i] = 0;
            bk[k0 + q] = B;
            if (s - B < 0.0) {
              le += B;
              les += fabs(s);
            }
            if (s < 0.0) lpsi += s;
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < KP; q++) bk[k0 + q] = 0.0;
      }
    }
    const int w = ls >> 6;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lpsi += __shfl_xor(lpsi, o, 64);
      le += __shfl_xor(le, o, 64);
      les += __shfl_xor(les, o, 64);
    }
    const bool wbad = __builtin_amdgcn_ballot_w64(lbad) != 0;
    if ((ls & 63) == 0) {
      W[4 * w] = lpsi;
      W[4 * w + 1] = le;
      W[4 * w + 2] = les;
      W[4 * w + 3] = wbad ? 1.0 : 0.0;
    }
    grp_sync<S>();
    double psi = 0.0, E = 0.0, Es = 0.0;
    bool bad = false;
#pragma unroll
    for (int v = 0; v < S / 64; v++) {
      psi += W[4 * v];
      E += W[4 * v + 1];
      Es += W[4 * v + 2];
      bad = bad || W[4 * v + 3] != 0.0;
    }
    const double thr = (double)m * kEps * ctl->c1 * ctl->c2 * 100.0;
    if (bad || !(fabs(psi) - (1.001 * E + 4e-16 * m * Es) > 1.001 * thr + 1e-10 * sigma_s() * m)) return false;
    // the two smallest upper bounds among the constraints the select may pick
    double h1 = inf, h2 = inf;
#pragma unroll
    for (int k = 0; k < KS; k++) {
      const int i = ls + k * S;
      const double sk = i < m ? sv[i] : 0.0;
      if (i < m && sk - bk[k] < 0.0 && !act[i]) {
        const double hi = sk + bk[k];
        if (hi < h1) {
          h2 = h1;
          h1 = hi;
        } else if (hi < h2) {
          h2 = hi;
        }
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const double c1 = __shfl_xor(h1, o, 64), c2 = __shfl_xor(h2, o, 64);
      if (c1 < h1) {
        h2 = fmin(h1, c2);
        h1 = c1;
      } else {
        h2 = fmin(h2, c1);
      }
    }
    if ((ls & 63) == 0) {
      W[16 + 2 * w] = h1;
      W[17 + 2 * w] = h2;
    }
    grp_sync<S>();
    h1 = W[16];
    h2 = W[17];
#pragma unroll
    for (int v = 1; v < S / 64; v++) {
      const double c1 = W[16 + 2 * v], c2 = W[17 + 2 * v];
      if (c1 < h1) {
        h2 = fmin(h1, c2);
        h1 = c1;
      } else {
        h2 = fmin(h2, c1);
      }
    }
#pragma unroll
    for (int k = 0; k < KS; k++) {
      const int i = ls + k * S;
      const double sk = i < m ? sv[i] : 0.0;
      if (i < m && sk - bk[k] < 0.0 && !act[i] && sk - bk[k] <= h2) {
        const int pos = atomicAdd(&cl[0], 1);
        if (pos < kShadowCand) cl[1 + pos] = i;
      }
    }
    grp_sync<S>();
    const int cnt = cl[0];
    if (cnt > kShadowCand) return false;
    if (lead) atomicAdd(&g_shadow_stats[2], (unsigned long long)cnt);
    for (int c = 0; c < cnt; c++) {
      const int i = cl[1 + c];
      if (ls < n) P[ls] = EL(CIb, ls * m + i) * xv[ls];
      grp_sync<S>();
      if (lead) {
        double s = 0.0;
        for (int jb = 0; jb < n; jb += 8) {
          double v[8];
#pragma unroll
          for (int u = 0; u < 8; u++) v[u] = P[jb + u < n ? jb + u : n - 1];
#pragma unroll
          for (int u = 0; u < 8; u++)
            if (jb + u < n) s += v[u];
        }
        sv[i] = s + EL(ci0b, i);
      }
      grp_sync<S>();
    }
    return true;
  };

  // Per-subgroup state machine; a wave loops until all of its QPs are done.
  const int max_steps = a.max_steps;
  // the select that follows a scan (carried ss reset to 0): its argmin, the np gather and
  // ci0[ip] are started inside the scan, so their global loads overlap the lead's psi sum
  constexpr bool kPreSel = QPGPU_WAVE_PRESEL && kLaneSel && !GJR && MMAX <= 2 * S && NMAX <= S;
  [[maybe_unused]] double pre_sb = 0.0, pre_np = 0.0, pre_c0 = 0.0;
  [[maybe_unused]] int pre_ib = INT_MAX;
  [[maybe_unused]] bool from_scan = false;
  // A QP falls through scan -> select -> step within one pass of the loop (QPGPU_WAVE_FALLTHRU),
  // so two QPs of a wave at different phases share the later blocks instead of running them in
  // separate passes.
  while (true) {
    if (any_bad()) return false;
    int phase = ctl->phase;
    if (S < 64) {
      if (__builtin_amdgcn_ballot_w64(phase != PH_DONE) == 0) break;
    } else if (phase == PH_DONE) {
      break;
    }
    if (phase == PH_DONE) continue;  // other subgroups of this wave are still busy
    if (phase == PH_SCAN) {
      const uint64_t t0 = clk();
      // ---- l1
      if (lead) ctl->iter++;
      {
        // mark the active inequalities; keep the rollback copies of A and u (read only after a
        // degenerate add_constraint, so they may be taken whether or not the scan finds ψ = 0)
        const int iqs = ctl->iq;
        for (int i = ls; i < iqs; i += S) {
          const int ai = Av[i];
          if (i >= p) act[ai] = 1;
          Ao[i] = ai;
          uo[i] = uv[i];
        }
      }
      if constexpr (!GJR && MMAX <= 2 * S) {
        // a lane's two constraints (i0 = ls, i1 = ls + S) summed together, so each chunk of CI
        // loads covers both and a scan waits on half as many memory latencies; each sum keeps the
        // reference's j order (the second constraint's index is clamped when it does not exist,
        // its sum then discarded)
        const int i0 = ls, i1 = ls + S;
        const bool h0 = i0 < m, h1 = i1 < m;
        const int c0i = h0 ? i0 : 0, c1i = h1 ? i1 : c0i;
        const double c00 = EL(ci0b, c0i), c01 = EL(ci0b, c1i);
        constexpr int SKG = OCC >= 4 ? QPGPU_WAVE_SCANKG4 : QPGPU_WAVE_SCANKG;
        double s0 = 0.0, s1 = 0.0;
        int jb = 0;
        for (; jb + SKG <= n; jb += SKG) {
          double a0[SKG], a1[SKG], xw[SKG];
#pragma unroll
          for (int u = 0; u < SKG; u++) {
            a0[u] = EL(CIb, (jb + u) * m + c0i);
            a1[u] = EL(CIb, (jb + u) * m + c1i);
            xw[u] = xv[jb + u];
          }
#pragma unroll
          for (int u = 0; u < SKG; u++) {
            s0 += a0[u] * xw[u];
            s1 += a1[u] * xw[u];
          }
        }
        if (jb < n) {
          double a0[SKG], a1[SKG], xw[SKG];
#pragma unroll
          for (int u = 0; u < SKG; u++) {
            const int jj = jb + u < n ? jb + u : n - 1;
            a0[u] = EL(CIb, jj * m + c0i);
            a1[u] = EL(CIb, jj * m + c1i);
            xw[u] = xv[jj];
          }
#pragma unroll
          for (int u = 0; u < SKG; u++)
            if (jb + u < n) {
              s0 += a0[u] * xw[u];
              s1 += a1[u] * xw[u];
            }
        }
        const double v0 = s0 + c00, v1 = s1 + c01;
        if (h0) {
          sv[i0] = v0;
          exc[i0] = 0;
        }
        if (h1) {
          sv[i1] = v1;
          exc[i1] = 0;
        }
        if constexpr (kPreSel) {
          // the select's candidates (s < 0, not active; exclusions were just cleared) from this
          // lane's two sums in index order, then the subgroup argmin (ties: lower index)
          sg_sync();  // the other lanes' act[] marks of this scan
          double sb = inf;
          int ib = INT_MAX;
          if (h0 && v0 < 0.0 && !act[i0]) {
            sb = v0;
            ib = i0;
          }
          if (h1 && v1 < 0.0 && !act[i1] && v1 < sb) {
            sb = v1;
            ib = i1;
          }
          sg_argmin<S>(sb, ib);
          pre_sb = sb;
          pre_ib = ib;
          const int ig = ib != INT_MAX ? ib : 0;
          pre_np = EL(CIb, (ls < n ? ls : n - 1) * m + ig);
          pre_c0 = EL(ci0b, ig);
          from_scan = true;
        }
      } else {
        shadow_hit = false;
        if constexpr (kShadow) {
          if (pre && (a.flags & kArgShadow)) {
            shadow_hit = shadow_scan();
            if (lead) {
              atomicAdd(&g_shadow_stats[0], 1ull);
              if (shadow_hit) atomicAdd(&g_shadow_stats[1], 1ull);
            }
          }
        }
        if (!shadow_hit) {
          for (int i = ls; i < m; i += S) {
            const double c0 = EL(ci0b, i);  // issued with the first chunk, added last
            double s = seq_fma_up<KG>(0.0, 0, n, [&](int j) { return EL(CIb, j * m + i); },
                                  [&](int j) { return xv[j]; });
            s += c0;
            sv[i] = s;
            exc[i] = 0;
          }
        }
      }
      grp_sync<S>();
      if (lead && shadow_hit) {
        // the bounds settled the stop test (|psi| is above the threshold and outside the
        // certification window whatever the fp64 values) and the candidates hold their fp64 s
        ctl->ss = 0.0;
        ctl->ip = 0;
        ctl->phase = PH_SELECT;
      } else if (lead) {
        double psi = 0.0;
        int negc = 0;  // (certification: the negative s_i psi sums)
        constexpr int U = 8;  // loads of a chunk together, adds in i order
        auto chunk = [&](int ib, int c) {
          double sc[U];
#pragma unroll
          for (int u = 0; u < U; u++) sc[u] = sv[ib + u];  // past m: in-bounds LDS, masked
#pragma unroll
          for (int u = 0; u < U; u++) {
            psi += (u < c && sc[u] < 0.0) ? sc[u] : 0.0;
            negc += (u < c && sc[u] < 0.0) ? 1 : 0;
          }
        };
        int ib = 0;
        for (; ib + U <= m; ib += U) chunk(ib, U);
        if (ib < m) chunk(ib, m - ib);
        ctl->ss = 0.0;
        ctl->ip = 0;
        if (pre) {
          // the stop test |psi| <= thr within the rounding the two evaluations of the negative
          // s_i can differ by: each s_i by at most 1e-10 (||CI_i||_1 ||x||_inf + |ci0_i|)
          const double thr = (double)m * kEps * ctl->c1 * ctl->c2 * 100.0;
          if (fabs(fabs(psi) - thr) <= 1e-4 * thr + 1e-10 * sigma_s() * negc) ctl->unc |= kUncPsi;
        }
        if (fabs(psi) <= (double)m * kEps * ctl->c1 * ctl->c2 * 100.0) {
          ctl->phase = PH_DONE;
        } else {
          ctl->phase = PH_SELECT;
        }
      }
      for (int i = ls; i < n; i += S) xo[i] = xv[i];
      grp_sync<S>();
      tph[0] += clk() - t0;
      if (!QPGPU_WAVE_FALLTHRU) continue;
      phase = ctl->phase;
    }
    if (phase == PH_SELECT) {
      const uint64_t t0 = clk();
      // ---- l2 (ss deliberately not reset: reference quirk)
      [[maybe_unused]] double sbest = inf;
      [[maybe_unused]] int ibest = INT_MAX;
      if constexpr (kLaneSel) {
        if (kPreSel && from_scan) {
          sbest = pre_sb;
          ibest = pre_ib;
        } else {
          // each lane scans its constraints in index order, then the subgroup argmin: the same
          // (smallest s below the carried ss, first index) as the reference's sequential scan
          const double ss0 = ctl->ss;
          for (int i = ls; i < m; i += S) {
            const double v = sv[i];
            if (v < ss0 && !act[i] && !exc[i] && v < sbest) {
              sbest = v;
              ibest = i;
            }
          }
          sg_argmin<S>(sbest, ibest);
        }
      }
      // workspace variant (one QP per 256-thread block): the same selection across the block —
      // each lane scans its constraints in index order, then a butterfly per wave and the four
      // waves' results in wave order; (value, index) pairs merge by value then lower index, so
      // the result is the reference's (smallest s below the carried ss, first index) bit for bit,
      // with the runner-up value for the certification (kUncSelTie)
      [[maybe_unused]] double s2best = inf;
      if constexpr (GJR && !kLaneSel) {
        const double ss0 = ctl->ss;
        for (int i = ls; i < m; i += S) {
          const double v = sv[i];
          if (v < ss0 && !act[i] && !exc[i]) {
            if (v < sbest) {
              s2best = sbest;
              sbest = v;
              ibest = i;
            } else if (v < s2best) {
              s2best = v;
            }
          }
        }
        auto merge = [&](double c1, int j1, double c2) {
          if (c1 < sbest || (c1 == sbest && j1 < ibest)) {
            s2best = fmin(sbest, c2);
            sbest = c1;
            ibest = j1;
          } else {
            s2best = fmin(s2best, c1);
          }
        };
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          const double c1 = __shfl_xor(sbest, o, 64), c2 = __shfl_xor(s2best, o, 64);
          const int j1 = __shfl_xor(ibest, o, 64);
          merge(c1, j1, c2);
        }
        double* const W = Q + Ly.off_tsc;  // (the d/z pass's partials are not live here)
        if ((ls & 63) == 0) {
          W[3 * (ls >> 6)] = sbest;
          W[3 * (ls >> 6) + 1] = (double)ibest;
          W[3 * (ls >> 6) + 2] = s2best;
        }
        grp_sync<S>();
        if (lead) {
          sbest = W[0];
          ibest = (int)W[1];
          s2best = W[2];
          for (int w = 1; w < S / 64; w++) merge(W[3 * w], (int)W[3 * w + 1], W[3 * w + 2]);
        }
      }
      if (lead) {
        double ss = ctl->ss;
        int ip = ctl->ip;
        if constexpr (kLaneSel) {
          if (ibest != INT_MAX) {
            ss = sbest;
            ip = ibest;
          }
        } else if (GJR) {
          if (ibest != INT_MAX) {
            ss = sbest;
            ip = ibest;
            // two candidates within the rounding the two evaluations of s can differ by: a
            // decision the tolerance mode's rounding may order differently (kUncSelTie)
            if (pre && s2best < inf && s2best - sbest <= 2e-10 * sigma_s() + 1e-12 * (fabs(sbest) + fabs(s2best)))
              ctl->unc |= kUncSelTie;
          }
        } else {
          for (int i = 0; i < m; i++)
            if (sv[i] < ss && !act[i] && !exc[i]) {
              ss = sv[i];
              ip = i;
            }
        }
        ctl->ss = ss;
        ctl->ip = ip;
        if (ss >= 0.0) {
          ctl->phase = PH_DONE;
        } else {
          uv[ctl->iq] = 0.0;
          Av[ctl->iq] = ip;
          ctl->ci0ip = (kPreSel && from_scan) ? pre_c0 : EL(ci0b, ip);
          ctl->phase = PH_STEP;
        }
      }
      grp_sync<S>();
      if (ctl->phase == PH_STEP) {
        const int ip = ctl->ip;
        if (kPreSel && from_scan) {
          if (ls < n) npv[ls] = pre_np;
        } else {
          for (int j = ls; j < n; j += S) npv[j] = EL(CIb, j * m + ip);
        }
        grp_sync<S>();
      }
      from_scan = false;
      tph[1] += clk() - t0;
      if (!QPGPU_WAVE_FALLTHRU) continue;
      phase = ctl->phase;
    }
    if (phase != PH_STEP) continue;
    // ---- l2a (phase == PH_STEP)
    if (lead) {
      if (max_steps > 0 && ++ctl->steps > max_steps) {
        ctl->status = QPGPU_QP_MAX_ITER;
        ctl->phase = PH_DONE;
      }
    }
    grp_sync<S>();
    if (ctl->phase == PH_DONE) continue;
    uint64_t t0 = clk();
    compute_d_z(ctl->iq);
    uint64_t t1c = clk();
    tph[2] += t1c - t0;
    int kind = 0;  // 1 infeasible, 2 dual step, 3 full step, 4 partial step
    if (QPGPU_WAVE_STAMPS_DETAIL == 1) {
      tdet[1] += 1;
      tdet[2] += ctl->iq;
    }
    update_r(ctl->iq, p);
    if (QPGPU_WAVE_STAMPS_DETAIL == 1) tdet[0] += clk() - t1c;
    // t1 = min over active inequalities with r > 0 of u/r (first index on ties), l its constraint
    [[maybe_unused]] double t1best = inf;
    [[maybe_unused]] int kbest = INT_MAX;
    if constexpr (kLaneSel) {
      const int iq = ctl->iq;
      for (int k = p + ls; k < iq; k += S)
        if (rv[k] > 0.0) {
          const double q = wdiv<F>(uv[k], rv[k], fok);
          if (q < t1best) {
            t1best = q;
            kbest = k;
          }
        }
      sg_argmin<S>(t1best, kbest);
    }
    if (lead) {
      const int iq = ctl->iq;
      int l = 0;
      double t1 = inf;
      if constexpr (kLaneSel) {
        if (kbest != INT_MAX) {
          t1 = t1best;
          l = Av[kbest];
        }
      } else if (pre) {
        double t1b = inf;  // runner-up (kUncT1Tie)
        for (int k = p; k < iq; k++)
          if (rv[k] > 0.0) {
            const double q = uv[k] / rv[k];
            if (q < t1) {
              t1b = t1;
              t1 = q;
              l = Av[k];
            } else if (q < t1b) {
              t1b = q;
            }
          }
        if (t1b < inf && t1b - t1 <= 1e-9 * (fabs(t1) + fabs(t1b))) ctl->unc |= kUncT1Tie;
      } else {
        for (int k = p; k < iq; k++)
          if (rv[k] > 0.0 && uv[k] / rv[k] < t1) {
            t1 = uv[k] / rv[k];
            l = Av[k];
          }
      }
      double t2, zz, znp;
      dot2_lead(zz, znp);
      if (fabs(zz) > kEps) {
        t2 = wdiv<F>(-sv[ctl->ip], znp, fok);
        if (t2 < 0) t2 = inf;  // Takano Akio patch
      } else {
        t2 = inf;
      }
      const double t = (t2 < t1) ? t2 : t1;
      ctl->t = t;
      ctl->t1 = t1;
      ctl->t2 = t2;
      ctl->l = l;
      if (pre) {
        if (fabs(zz) >= 0.25 * kEps && fabs(zz) <= 4.0 * kEps) ctl->unc |= kUncZz;
        if (t1 < inf && t2 < inf && fabs(t1 - t2) <= 1e-9 * fmax(fabs(t1), fabs(t2))) ctl->unc |= kUncStepTie;
        if (fabs(t - t2) >= 0.25 * kEps && fabs(t - t2) <= 4.0 * kEps) ctl->unc |= kUncTt2;
      }
      if (t >= inf) {
        ctl->status = QPGPU_QP_INFEASIBLE;
        ctl->f = inf;
        ctl->phase = PH_DONE;
        kind = 1;
      } else if (t2 >= inf) {
        uv[iq] += t;  // u[:iq] -= t r[:iq] by the lanes below
        act[l] = 0;
        kind = 2;
      } else {
        ctl->f += t * znp * (0.5 * t + uv[iq]);
        if (pre) ctl->fmax = fmax(ctl->fmax, fabs(ctl->f));
        uv[iq] += t;
        kind = (fabs(t - t2) < kEps) ? 3 : 4;
      }
      ctl->qq = kind;  // broadcast the branch
    }
    grp_sync<S>();
    kind = ctl->qq;
    if (kind >= 2) {
      const double t = ctl->t;
      for (int k = p + ls; k < ctl->iq; k += S) uv[k] -= t * rv[k];  // (u[0..p) are never read)
      grp_sync<S>();
    }
    t0 = clk();
    tph[3] += t0 - t1c;
    if (kind == 1) continue;
    if (kind == 2) {
      delete_constraint(ctl->l);
      tph[5] += clk() - t0;
      if (lead) ctl->phase = PH_STEP;
      grp_sync<S>();
      continue;
    }
    {
      const double t = ctl->t;
      for (int k = ls; k < n; k += S) {
        xv[k] += t * zv[k];
        note_x(xv[k]);
      }
    }
    grp_sync<S>();
    if (kind == 3) {
      const uint64_t ta = clk();
      add_constraint();
      tph[4] += clk() - ta;
      if (!ctl->fin) {
        const int ip = ctl->ip;
        if (lead) exc[ip] = 1;
        grp_sync<S>();
        delete_constraint(ip);
        for (int i = ls; i < m; i += S) act[i] = 0;
        grp_sync<S>();
        for (int i = p + ls; i < ctl->iq; i += S) {
          const int ai = Ao[i];
          Av[i] = ai;
          uv[i] = uo[i];
          act[ai] = 1;
        }
        if (lead) ctl->phase = PH_SELECT;
        for (int i = ls; i < n; i += S) xv[i] = xo[i];
      } else {
        if (lead) {
          act[ctl->ip] = 1;
          ctl->phase = PH_SCAN;
        }
      }
      grp_sync<S>();
      continue;
    }
    // partial step: drop l, refresh s[ip]
    if (lead) act[ctl->l] = 0;
    grp_sync<S>();
    {
      const uint64_t td = clk();
      delete_constraint(ctl->l);
      tph[5] += clk() - td;
    }
    if (lead) {
      const double s = seq_fma_up_lds<8>(0.0, 0, n, [&](int k) { return npv[k]; },
                                [&](int k) { return xv[k]; });
      sv[ctl->ip] = s + ctl->ci0ip;
      ctl->phase = PH_STEP;
    }
    grp_sync<S>();
  }
#undef J_
#undef R_
#undef GC_
#undef GS_
#undef GX_
#undef GF_

  qp_stamp(a, 4);
  if (a.stamps && threadIdx.x == 0)
    for (int k = 0; k < 6; k++) a.stamps[(uint64_t)blockIdx.x * kStampSlots + 8 + k] = tph[k];
  if (a.stamps && threadIdx.x == 0) {
    for (int k = 0; k < 3; k++)
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 5 + k] = QPGPU_WAVE_STAMPS_DETAIL ? tdet[k] : teq[k];
    for (int k = 3; k < 5; k++) a.stamps[(uint64_t)blockIdx.x * kStampSlots + 11 + k] = teq[k];
  }
  // ------------------------------------------------------------------ outputs
  if (any_bad()) return false;
  if (GJR && pre && live) {
    // certification at the end: x's norm against its largest value over the run (cancellation),
    // non-finite results, the step cap; a QP with any reason is marked for the EXACT re-solve
    if (ls < n) {
      const double xi = fabs(xv[ls]);
      if (!(xi < inf)) atomicOr(&ctl->unc, kUncNonFinite);
      atomicMax(&ctl->xn, (unsigned long long)__builtin_bit_cast(uint64_t, xi < inf ? xi : 0.0));
    }
    grp_sync<S>();
    if (lead) {
      const double xn = __builtin_bit_cast(double, (uint64_t)ctl->xn);
      const double xh = __builtin_bit_cast(double, (uint64_t)ctl->xh);
      const double fv = ctl->f;
      int u = ctl->unc;
      if (ctl->status == QPGPU_QP_MAX_ITER) u |= kUncMaxIter;
      if (!(fabs(fv) < inf)) u |= kUncNonFinite;
      if (!(ctl->fmax <= 1e4 * fabs(fv))) u |= kUncFCancel;
      if (!(xh <= 1e4 * xn)) u |= kUncXCancel;
      ctl->unc = u;
    }
    grp_sync<S>();
  }
  if (live) {
    const int st = ctl->status;
    if (st != QPGPU_QP_NOT_POSITIVE_DEFINITE) {
      double* xb = a.x + qbase_rt(bb, n, T);
      for (int i = ls; i < n; i += S) EL(xb, i) = xv[i];
    }
    if (lead) {
      a.f[b] = ctl->f;
      const int unc = (GJR && pre) ? ctl->unc : 0;
      a.status[b] = unc ? (st | kStResolve | (unc << kStReasonShift)) : st;
      if (a.iters) a.iters[b] = ctl->iter;
    }
  }
#undef EL
  return true;
}

template <int S, int NMAX, int MMAX, bool GJR, int OCC = 1>
__global__ void __launch_bounds__(S >= 64 ? S : 64, GJR ? QPGPU_WAVE_GJR_OCC : OCC)
    QP_WAVE_KERNEL(const QpArgs a, double* __restrict__ ws) {
  if constexpr (GJR) {
    // the EXACT re-solve after a tolerance-mode launch: only the QPs marked for it (one QP per
    // workgroup, so the exit is uniform)
    if (a.flags & kResolveOnly) {
      const int64_t b = blockIdx.x;
      if (b >= a.batch || !(a.status[b] & kStResolve)) return;
    }
  }
  if constexpr (kWaveFast && !GJR && S <= 64) {
    if (!wave_body<S, NMAX, MMAX, GJR, OCC, true>(a, ws)) {
      __syncthreads();  // the fast attempt's LDS traffic is over
      wave_body<S, NMAX, MMAX, GJR, OCC, false>(a, ws);
    }
  } else {
    wave_body<S, NMAX, MMAX, GJR, OCC, false>(a, ws);
  }
}

// ------------------------------------------------------------------------------------------
template <int S, int NMAX, int MMAX, bool GJR>
static hipError_t launch_wave(const QpArgs& a, hipStream_t stream, double* ws) {
  using C = WaveCfg<S, NMAX, MMAX, GJR>;
  const int64_t blocks = (a.batch + C::QPB - 1) / C::QPB;
  size_t lds_bytes = (size_t)C::QPB * wave_lay(a.n, a.m, GJR).stride * sizeof(double);
  // Two-QP-per-wave variants: when a block's LDS leaves room for >= 2 waves per SIMD (<= 20 KiB,
  // i.e. >= 8 one-wave blocks per CU) register pressure is the occupancy limit, so launch the
  // instantiation compiled for 4 waves per SIMD (a few spilled VGPRs).  Measured: mgqp level 0
  // (10.5 KiB per block) 2.44 -> 2.32 ms; C3 (37 KiB per block, LDS-limited to one wave per SIMD)
  // keeps the unconstrained allocation (21.0 vs 22.0 ms).  The register-setup instantiations
  // (OCC 2 for S = 16, OCC 1) use the packed-R layout when QPGPU_WAVE_RPACK is on.
  if constexpr (S < 64 && !GJR) {
    if (lds_bytes <= QPGPU_WAVE_OCC4_LDS) {
      hipLaunchKernelGGL((QP_WAVE_KERNEL<S, NMAX, MMAX, GJR, QPGPU_WAVE_OCC_SMALL>), dim3((unsigned)blocks), dim3(C::BS),
                         lds_bytes, stream, a, ws);
      return hipGetLastError();
    }
    const size_t lds_p = (size_t)C::QPB * wave_lay(a.n, a.m, GJR, QPGPU_WAVE_RPACK != 0).stride * sizeof(double);
    // four-QP waves (S = 16): up to 40 KiB per block still leaves room for two waves per SIMD
    if (S == 16 && lds_bytes <= 40960) {
      hipLaunchKernelGGL((QP_WAVE_KERNEL<S, NMAX, MMAX, GJR, 2>), dim3((unsigned)blocks), dim3(C::BS),
                         lds_p, stream, a, ws);
      return hipGetLastError();
    }
    lds_bytes = lds_p;  // OCC 1 (register setup) from here on
  }
  // workspace variant (n > 64): an A/B build with -DQPGPU_WAVE_GJR_CAP=k pads the dynamic LDS so
  // at most k one-QP workgroups share a CU (fewer resident QPs = a working set that may stay in
  // the Infinity Cache).  The product build has no cap.
  if constexpr (GJR && QPGPU_WAVE_GJR_CAP > 0) {
    constexpr size_t cap = QPGPU_WAVE_GJR_CAP > 0 ? QPGPU_WAVE_GJR_CAP : 1;
    const size_t want = (size_t)163840 / cap - 1024;
    if (want > lds_bytes) lds_bytes = want;
  }
  // dynamic LDS beyond 64 KiB must be granted per kernel and device; host threads may launch
  // concurrently (include/qpgpu.h), so the record of what was granted is locked
  if (lds_bytes > 65536) {
    static std::mutex mu;
    static std::map<int, size_t> granted;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    size_t& g = granted[dev];
    if (lds_bytes > g) {
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&QP_WAVE_KERNEL<S, NMAX, MMAX, GJR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
      if (e != hipSuccess) return e;
      g = lds_bytes;
    }
  }
  hipLaunchKernelGGL((QP_WAVE_KERNEL<S, NMAX, MMAX, GJR>), dim3((unsigned)blocks), dim3(C::BS), lds_bytes,
                     stream, a, ws);
  return hipGetLastError();
}

struct WaveVariant {
  int nmax, mmax;
  int64_t ws_doubles_per_qp;
  const char* name;
  hipError_t (*launch)(const QpArgs&, hipStream_t, double*);
};

#if QPGPU_WAVE_FAST
#define QPK_WAVE_VNAME(s) "qp_wave_fast<" s ">"
#else
#define QPK_WAVE_VNAME(s) "qp_wave<" s ">"
#endif
static const WaveVariant kWaveVariants[] = {
#if QPGPU_WAVE_S16
    {16, 32, 0, QPK_WAVE_VNAME("S=16,N=16,M=32"), launch_wave<16, 16, 32, false>},
#endif
    {32, 64, 0, QPK_WAVE_VNAME("S=32,N=32,M=64"), launch_wave<32, 32, 64, false>},
    {32, 128, 0, QPK_WAVE_VNAME("S=32,N=32,M=128"), launch_wave<32, 32, 128, false>},
    {64, 128, 0, QPK_WAVE_VNAME("S=64,N=64,M=128"), launch_wave<64, 64, 128, false>},
    {64, 256, 0, QPK_WAVE_VNAME("S=64,N=64,M=256"), launch_wave<64, 64, 256, false>},
#if !QPGPU_WAVE_FAST
    {256, 1024, WaveCfg<256, 256, 1024, true>::WS_DOUBLES,
     "qp_panel<MFMA f64 16x16x4> + qp_wave<S=256,N=256,M=1024,global J/R>",
     launch_wave<256, 256, 1024, true>},
#endif
};

const WaveVariant* pick_wave(int n, int m) {
  for (const auto& v : kWaveVariants)
    if (n <= v.nmax && m <= v.mmax) return &v;
  return nullptr;
}

}  // namespace QPK_WAVE_NS

#if QPGPU_WAVE_FAST
// the fast build covers the LDS variants only (n <= 64, m <= 256); wider shapes keep the
// default path (its n > 64 form is already the 1e-10 tolerance mode)
extern "C" const char* qpk_medium_name_fast(int n, int /*p*/, int m) {
  const qpk_wfast::WaveVariant* v = qpk_wfast::pick_wave(n, m);
  return v ? v->name : nullptr;
}
extern "C" hipError_t qpk_launch_medium_fast(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                             const char** name) {
  const qpk_wfast::WaveVariant* v = qpk_wfast::pick_wave(a->n, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  return v->launch(*a, stream, nullptr);
}
#else
extern "C" const char* qpk_medium_name(int n, int /*p*/, int m) {
  const qpk::WaveVariant* v = qpk::pick_wave(n, m);
  return v ? v->name : nullptr;
}
extern "C" int qpk_medium_max_n(void) { return 256; }
extern "C" int qpk_medium_max_m(void) { return 1024; }
extern "C" hipError_t qpk_launch_panel_setup(const qpk::QpArgs* a, hipStream_t stream, double* ws);

// Workspace variants (n > 64) run the MFMA panel setup (qp_panel.hip) first unless the caller
// asked for the reference's exact operation order (QPGPU_FLAG_EXACT) or for the factor in G
// (QPGPU_FLAG_WRITE_FACTOR: the reference's bits), which the serial restatement here provides.
// Only panel-set-up launches run the tolerance-mode loop, whose deferred J sweep may still be
// pending when a QP finishes (see `pend` in qp_wave_kernel): keep both flags out of it.
static bool g_resolve = true;
static bool uses_panel(const qpk::WaveVariant* v, uint32_t flags) {
  return v->ws_doubles_per_qp > 0 && !(flags & (QPGPU_FLAG_EXACT | QPGPU_FLAG_WRITE_FACTOR));
}

// The fp32 copy of CI for the tolerance-mode shadow scan (QPGPU_WAVE_SHADOW): QP-major batches
// of the panel path, after the batch's per-QP workspace blocks, up to 16 GiB (a larger batch
// scans in fp64).  qpk_set_shadow(0) (qpgpu_debug_set_shadow) turns it off for A/B tests.
static bool g_shadow = QPGPU_WAVE_SHADOW != 0;
static int64_t shadow_bytes(const qpk::WaveVariant* v, const qpk::QpArgs* a) {
  if (!g_shadow || !uses_panel(v, a->flags) || a->tile != 1 || a->m <= 0) return 0;
  const int64_t b = (int64_t)a->n * a->m * 4 * a->batch;
  return b <= ((int64_t)16 << 30) ? (b + 255) / 256 * 256 : 0;
}
__global__ void __launch_bounds__(256) qp_ci_shadow_kernel(const double* __restrict__ ci, float* __restrict__ out,
                                                           int64_t count) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += stride) out[i] = (float)ci[i];
}

// bytes of device workspace the medium kernels need for a launch (0 = none)
extern "C" int64_t qpk_medium_workspace_bytes(const qpk::QpArgs* a) {
  const qpk::WaveVariant* v = qpk::pick_wave(a->n, a->m);
  return v ? v->ws_doubles_per_qp * 8 * a->batch + shadow_bytes(v, a) : 0;
}

extern "C" hipError_t qpk_launch_medium_ws(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                          const char** name, double* ws) {
  const qpk::WaveVariant* v = qpk::pick_wave(a->n, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  if (uses_panel(v, a->flags)) {
    hipError_t e = qpk_launch_panel_setup(a, stream, ws);
    if (e != hipSuccess) return e;
    qpk::QpArgs b = *a;
    b.flags |= qpk::kSetupDone;
    if (shadow_bytes(v, a) > 0) {
      const int64_t count = (int64_t)a->n * a->m * a->batch;
      const int64_t want = (count + 255) / 256;
      const unsigned blocks = (unsigned)(want < 16384 ? want : 16384);
      hipLaunchKernelGGL(qp_ci_shadow_kernel, dim3(blocks), dim3(256), 0, stream, a->CI,
                         reinterpret_cast<float*>(ws + a->batch * v->ws_doubles_per_qp), count);
      if ((e = hipGetLastError()) != hipSuccess) return e;
      b.flags |= qpk::kArgShadow;
    }
    e = v->launch(b, stream, ws);
    if (e != hipSuccess || !g_resolve) return e;
    // the QPs the tolerance mode could not certify (status | kStResolve) again in the reference's
    // operation order: one more launch whose other workgroups exit at once
    qpk::QpArgs c = *a;
    c.flags |= QPGPU_FLAG_EXACT | qpk::kResolveOnly;
    return v->launch(c, stream, ws);
  }
  return v->launch(*a, stream, ws);
}
// test / diagnostic hook (qpgpu_debug_set_resolve): 0 leaves the tolerance mode's marks in
// the status words and skips the EXACT re-solve
extern "C" void qpk_set_resolve(int on) { g_resolve = on != 0; }
// test / diagnostic hook (qpgpu_debug_set_shadow): 0 scans in fp64 only
extern "C" void qpk_set_shadow(int on) { g_shadow = on != 0 && QPGPU_WAVE_SHADOW != 0; }
// diagnostic (qpgpu_debug_shadow_stats): out[0] scans that tried the fp32 copy, out[1] those it
// settled, out[2] the fp64 re-evaluations of candidates they made, since the last reset;
// device-synchronous
extern "C" hipError_t qpk_shadow_stats(unsigned long long* out, int reset) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(qpk::g_shadow_stats), 3 * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    const unsigned long long z[3] = {0, 0, 0};
    e = hipMemcpyToSymbol(HIP_SYMBOL(qpk::g_shadow_stats), z, sizeof(z));
  }
  return e;
}
#endif  // QPGPU_WAVE_FAST
