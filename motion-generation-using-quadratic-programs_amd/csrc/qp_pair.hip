// qp_pair.hip — gfx950 batched Goldfarb–Idnani solver, ONE QP PER LANE PAIR: the QPGPU_FLAG_FAST
// kernel of the headline shape (C1 / C4: n = 7, p = 6, m = 14, QP-major).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; operation order
// of the prebuilt libquadprog.a fixed in SURVEY.md §3.2), as qp_lane.hip does, with two lanes
// per QP.
//
// Why pairs: qp_lane runs one QP per lane, so 65 536 QPs are exactly one wave per SIMD and every
// stall of that wave is exposed (~40 % of its cycles issue, the rest wait on memory
// or on the previous instruction).  Here lanes 2q and 2q+1 share QP q of the wave's 32: a
// 65 536-QP launch is 2 048 waves, two resident per SIMD (<= 256 VGPR+AGPR and 20 KiB of LDS
// per wave), so one wave's stalls are the other wave's issue slots.  The work divides where it
// is data-parallel and is duplicated where it is a serial chain:
//   * J rows are interleaved — lane h holds rows 2k+h — so compute_d (J^T np: one pair sum per
//     column), update_z and every Givens rotation of J run on half the rows;
//   * the constraints are interleaved too — lane h owns c = 2i+h — so the l1 scan and the l2
//     select run on half the constraints (the select exchanges the lane minima once);
//   * x, z and np are held by rows as J is; the dots z.z, z.np, np.x are pair sums, and the
//     scan assembles the whole x once per pass;
//   * the Cholesky factor, x0, R, u, r, A, the Givens coefficients, t1, t2 and every decision are
//     computed by both lanes from identical operands (a pair sum v0 + v1 is the same bits on
//     both lanes: IEEE addition commutes), so the two lanes of a QP always branch alike.
// Exchanges are DPP quad_perm moves inside the pair (no LDS round trip).  Splitting a sum over
// the pair changes its rounding against the reference's left-to-right order, so this kernel
// exists only in the fast build (-ffp-contract=fast, the fast forms of qp_common.h): x and f
// within north_star's 1e-10 relative per QP, status and l1 passes identical to the reference's
// (tests/test_gpu_parity.py).  A wave whose fast forms went out of range re-solves with the
// IEEE division and distance (the SAFE body), as qp_lane's fast build does.
#include <type_traits>

#include "qp_common.h"

// A/B knobs (tools/ab_pair.sh): CE loads kCeAhead steps ahead; the CI copy by DMA during the
// equality phase (1) or by the first scan (0).  Measured on C1 (profiles/r04_s15, r04_s16;
// kernel us): DMA from step 0 48.7, from step 3 45.6, from step 4 44.5, no DMA 43.8 (the first
// scan then reads rows 0..4 from memory, +4k cycles per wave, but the equality phase loses the
// waits on the copy: 16.1k instead of 19.5-31.6k cycles) — so 0.
#ifndef QPGPU_PAIR_CE_AHEAD
#define QPGPU_PAIR_CE_AHEAD 2
#endif
#ifndef QPGPU_PAIR_DMA
#define QPGPU_PAIR_DMA 0
#endif
// first equality step that issues a part of the CI copy (-1: the step that issues the last CE
// load, so that no CE load queues behind a copy part)
#ifndef QPGPU_PAIR_DMA_FROM
#define QPGPU_PAIR_DMA_FROM -1
#endif

namespace qpk_pair {
using namespace qpk;

constexpr int kQpw = 32;       // QPs per wave: one per lane pair
constexpr int kStage = 2560;   // LDS per wave, doubles (20 KiB: two waves per SIMD, 8 per CU)

// ---- pair exchange: the other lane of the pair (DPP quad_perm(1, 0, 3, 2))
constexpr int kSwap = 0xB1;
__device__ __forceinline__ uint32_t pswu(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kSwap, 0xf, 0xf, false);
}
__device__ __forceinline__ double psw(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = pswu((uint32_t)u), hi = pswu((uint32_t)(u >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int pswi(int v) { return (int)pswu((uint32_t)v); }
// v(lane 2q) + v(lane 2q+1), the same bits on both lanes
__device__ __forceinline__ double psum(double v) { return v + psw(v); }

// Rows of the CI copy that fit the LDS in the piece layout below
template <int NM, int MM>
constexpr int ci_rows_fit() {
  int r = 0;
  while (r < NM && ((r + 1) * MM / 2 + 1) / 2 * 128 <= kStage) r++;
  return r;
}

// One dword of every 128-B line of an NB-byte block (starting anywhere), the pair's lanes taking
// alternate lines: the cache warm-up.  retire() keeps the loads' results alive to a point well
// after they have landed, so nothing waits on them earlier.
template <int NB>
struct Touch {
  static constexpr int K = NB >= 4 ? (NB + 255) / 256 + 1 : 0;
  uint32_t v[K > 0 ? K : 1];
  __device__ __forceinline__ void load(const void* base, int h) {
    const char* c = reinterpret_cast<const char*>(base);
#pragma unroll
    for (int k = 0; k < K; k++) v[k] = *reinterpret_cast<const uint32_t*>(c + min(k * 256 + h * 128, NB - 4));
  }
  __device__ __forceinline__ void retire() const {
#pragma unroll
    for (int k = 0; k < K; k++) asm volatile("" ::"v"(v[k]));
  }
};

// The solve of one wave's 32 QPs.  SAFE: the IEEE forms of division and distance (the fallback
// of a wave whose fast forms were not valid on some lane).  Returns false as soon as that happens
// (checked after the J build, after the equality phase and after the loop): x, f, status and
// iters are not written then, and the caller re-solves the wave with SAFE.
template <int NM, int MM, int PX, bool SAFE>
__device__ __forceinline__ bool pair_body(const QpArgs& a, double* sbuf) {
  static_assert(MM % 2 == 0 && MM <= 64, "constraints interleave over the pair; bitmasks hold m <= 64");
  static_assert(PX >= 0 && PX <= NM, "p is a compile-time constant <= n");
  using RI = RIdx<NM>;
  constexpr bool F = !SAFE;
  constexpr int H = (NM + 1) / 2;  // rows per lane: local row k is row 2k + h
  constexpr int MH = MM / 2;       // constraints per lane: local i is constraint 2i + h
  constexpr int n = NM, m = MM, p = PX;
  bool fok = true;  // F: every fast form so far was valid on this lane

  const int lane = threadIdx.x;
  const int h = lane & 1;
  const int q = lane >> 1;
  const int64_t b0 = (int64_t)blockIdx.x * kQpw;
  const int64_t b = b0 + q;
  const int valid = (int)min<int64_t>(kQpw, a.batch - b0);
  const bool live = q < valid;
  const bool full = valid == kQpw;
  const int64_t bs = live ? b : b0;  // source QP of every load (idle lanes read QP b0)
  const double inf = dinf();
  // local row k exists unless n is odd and k is the odd lane's last
  const bool last_row = (NM % 2 == 0) || h == 0;
  auto has_row = [&](int k) { return k < H - 1 || last_row; };

  // ---- LDS staging of G and g0 (the wave's 32 contiguous QP blocks, LDS-DMA)
  auto copy_chunk = [&](const double* src, int nd, int off, int k) {  // doubles [k, k+128)
    const int e = k + 2 * lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(e < nd ? src + e : src),
                                     (__attribute__((address_space(3))) void*)(sbuf + off + k), 16, 0, 0);
  };
  auto stage_all = [&](const double* X, int E, int off) {
    if (full) {
      const double* src = X + b0 * (int64_t)E;
#pragma unroll 4
      for (int k = 0; k < kQpw * E; k += 128) copy_chunk(src, kQpw * E, off, k);
    } else if (live) {
      const double* src = X + b * (int64_t)E;
      for (int e = h; e < E; e += 2) sbuf[off + q * E + e] = src[e];
    }
  };
  constexpr int RB = kQpw * NM * NM;  // g0 staging offset
  static_assert(RB % 2 == 0 && RB + kQpw * NM <= kStage, "G and g0 staging exceed the LDS");

  // ---- CI rows 0..kCiRows-1 of every QP kept in LDS through the loop, in 16-B pieces: piece P
  // of QP q at doubles ((P >> 1) * 64 + 2q + (P & 1)) * 2.  Constraint 2i+h of row j is element
  // h of piece j*MH + i, so lane h's own elements sit at compile-time offsets from 4q + h.
  constexpr int kCiRows = ci_rows_fit<NM, MM>();
  constexpr int kCiPieces = kCiRows * MM / 2;
  constexpr int kCiInstr = (kCiPieces + 1) / 2;
  static_assert(kCiInstr * 128 <= kStage, "CI copy exceeds the LDS");
  double* const sbl = sbuf + 4 * q + h;
  auto ci_own_off = [](int j, int i) {  // offset from sbl of own constraint i of row j
    const int P = j * MH + i;
    return (P >> 1) * 128 + (P & 1) * 2;
  };
  auto ci_lds_at = [&](int r, int c) -> double {  // element (r, c) of this QP (runtime r, c)
    const int P = r * MH + (c >> 1);
    return sbuf[((P >> 1) * 64 + 2 * q + (P & 1)) * 2 + (c & 1)];
  };
  // p > 0: the copy by LDS-DMA during the equality phase (16-B pieces: CI 16-B aligned); p = 0:
  // the first scan writes it (qp_lane.hip measured no gain for a DMA without an equality phase)
  const bool dma = QPGPU_PAIR_DMA && PX > 0 && kCiRows > 0 && (a.flags & kArgAligned16);
  auto dma_ci_part = [&](int part, int parts) {
    const int per = (kCiInstr + parts - 1) / parts;
    const double* src = a.CI + bs * (int64_t)(NM * MM);
#pragma unroll
    for (int t = 0; t < kCiInstr; t++)
      if (t >= part * per && t < (part + 1) * per) {
        const int P = 2 * t + h < kCiPieces ? 2 * t + h : 0;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 2 * P),
                                         (__attribute__((address_space(3))) void*)(sbuf + t * 128), 16, 0, 0);
      }
  };
  // cache warm-up: one dword per 128-B line of this QP's CE, ce0 and (the rows the scans read
  // from global memory) CI rows kCiRows.. and ci0 — the pair's two lanes take alternate lines
  constexpr int kCeB = NM * PX * 8, kCe0B = PX * 8, kCiB = (NM - kCiRows) * MM * 8, kCi0B = MM * 8;
  [[maybe_unused]] Touch<kCeB> pf_ce;
  [[maybe_unused]] Touch<kCe0B> pf_ce0;
  [[maybe_unused]] Touch<kCiB> pf_ci;
  [[maybe_unused]] Touch<kCi0B> pf_ci0;
  [[maybe_unused]] Touch<kCiRows * MM * 8> pf_cil;  // without the copy by DMA: the rows it would copy

  int status = QPGPU_QP_OK;
  double fval = 0.0;
  int iter = 0;
  double xh[H];  // x, own rows
#pragma unroll
  for (int k = 0; k < H; k++) xh[k] = 0.0;
  double c1 = 0.0, c2 = 0.0;
  double Jh[H][NM];  // J, own rows
  // equality phase operands: np (own rows) and ce0 of step i, loaded kCeAhead steps ahead —
  // the first kCeAhead right after G has been read, so they arrive during the setup's compute
  // (one step ahead, every step waited a full memory latency: 39.5k instead of ~20k cycles per
  // wave, profiles/r04_s13; three or all six ahead spill registers)
  constexpr int kCeAhead = QPGPU_PAIR_CE_AHEAD;
  constexpr int PXA = PX > 0 ? PX : 1;
  [[maybe_unused]] double cea[PXA][H], c0a[PXA];
  const double* CEq = a.CE + bs * (int64_t)(NM * PX) + h * PX;  // row h of this QP's CE
  auto load_ce = [&](int i) {
#pragma unroll
    for (int k = 0; k < H; k++) {
      const double v = CEq[(has_row(k) ? 2 * k : 0) * PX + i];
      cea[i][k] = has_row(k) ? v : 0.0;
    }
    c0a[i] = a.ce0[bs * PX + i];
  };

  qp_stamp(a, 0);  // diagnostic phase clocks (tools/stamps.py; a.stamps is NULL in product calls)

  // ---------------------------------------------------------------- setup
  bool chol_ok = live;
  double bad_sum = 0.0;
  {
    double Gr[NM][NM];
    stage_all(a.G, NM * NM, 0);
    stage_all(a.g0, NM, RB);
    __syncthreads();
    double g0v[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) {
#pragma unroll
      for (int j = 0; j < NM; j++) {
        const double v = sbuf[q * NM * NM + i * NM + j];
        Gr[i][j] = live ? v : 0.0;
      }
      const double v0 = sbuf[RB + q * NM + i];
      g0v[i] = live ? v0 : 0.0;
    }
    __syncthreads();  // G read: the LDS is the CI copy's from here
    qp_stamp(a, 9);
    if constexpr (PX > 0) {
#pragma unroll
      for (int i = 0; i < PX && i < kCeAhead; i++) load_ce(i);
      pf_ce.load(a.CE + bs * (int64_t)(NM * PX), h);
      pf_ce0.load(a.ce0 + bs * PX, h);
      pf_ci.load(a.CI + bs * (int64_t)(NM * MM) + kCiRows * MM, h);
      pf_ci0.load(a.ci0 + bs * MM, h);
      if (!dma) pf_cil.load(a.CI + bs * (int64_t)(NM * MM), h);
    }
#pragma unroll
    for (int i = 0; i < NM; i++) c1 += Gr[i][i];
    // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored
#pragma unroll
    for (int i = 0; i < NM; i++) {
      if (chol_ok) {
        double sum = Gr[i][i];
#pragma unroll
        for (int k = i - 1; k >= 0; k--) sum -= Gr[i][k] * Gr[i][k];
        if (sum <= 0.0) {
          chol_ok = false;
          bad_sum = sum;
        } else {
          const double dg = sqrt(sum);
          Gr[i][i] = dg;
          const double rdg = F ? frcp(dg) : 0.0;
#pragma unroll
          for (int j = i + 1; j < NM; j++) {
            double s2 = Gr[i][j];
#pragma unroll
            for (int k = i - 1; k >= 0; k--) s2 -= Gr[i][k] * Gr[j][k];
            Gr[j][i] = ldiv_r<F>(s2, dg, rdg, fok);
          }
#pragma unroll
          for (int k = i + 1; k < NM; k++) Gr[i][k] = Gr[k][i];
        }
      }
    }
    // fast: the skipping J build below needs a finite factor on every lane (else the IEEE
    // re-solve, whose J build is the literal one) — decided for the whole wave here
    if constexpr (F) {
      bool lfin = true;
#pragma unroll
      for (int i = 0; i < NM; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) lfin = lfin && (fabs(Gr[i][j]) < inf);
      if (wave_any(chol_ok && !lfin)) return false;
    }
    if (chol_ok) {
      double rdiag[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) rdiag[i] = F ? frcp(Gr[i][i]) : 0.0;
      // J = L^{-T}, own rows: row r = 2k+h of J is L^{-1} e_r (forward elimination).  Fast: its
      // first 2k entries are exact zeros for a finite L (skipped at compile time).
      double c2p = 0.0;
#pragma unroll
      for (int k = 0; k < H; k++) {
        const int r = 2 * k + h;
        double y[NM];
#pragma unroll
        for (int i = 0; i < NM; i++) {
          if (F && i < 2 * k) {
            y[i] = 0.0;
            continue;
          }
          double v = (i == r) ? 1.0 : 0.0;
#pragma unroll
          for (int j = 0; j < i; j++)
            if (!(F && j < 2 * k)) v -= Gr[i][j] * y[j];
          y[i] = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
        }
#pragma unroll
        for (int j = 0; j < NM; j++) Jh[k][j] = has_row(k) ? y[j] : 0.0;
        const double yr = (2 * k + 1 < NM && h) ? y[2 * k + 1 < NM ? 2 * k + 1 : 0] : y[2 * k];
        c2p += has_row(k) ? yr : 0.0;
      }
      c2 = psum(c2p);
      // cholesky_solve (@.text+0x31a2): x = -G^{-1} g0 (both lanes, whole x)
      double y[NM], xf[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) {
        double v = g0v[i];
#pragma unroll
        for (int j = 0; j < i; j++) v -= Gr[i][j] * y[j];
        y[i] = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
      }
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        double v = y[i];
#pragma unroll
        for (int j = i + 1; j < NM; j++) v -= Gr[i][j] * xf[j];
        xf[i] = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
      }
#pragma unroll
      for (int i = 0; i < NM; i++) xf[i] = -xf[i];
#pragma unroll
      for (int i = 0; i < NM; i++) fval += g0v[i] * xf[i];
      fval = 0.5 * fval;
#pragma unroll
      for (int k = 0; k < H; k++) {
        const double xo = xf[2 * k + 1 < NM ? 2 * k + 1 : 2 * k];
        xh[k] = (h && has_row(k)) ? xo : (h ? 0.0 : xf[2 * k]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < H; k++)
#pragma unroll
        for (int j = 0; j < NM; j++) Jh[k][j] = 0.0;
    }
  }
  if (!chol_ok) {
    status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
    fval = bad_sum;
  }
  const bool ok_lane = live && chol_ok;
  qp_stamp(a, 1);

  // ---------------------------------------------------------------- state
  double Rv[RI::SIZE];
#pragma unroll
  for (int i = 0; i < RI::SIZE; i++) Rv[i] = 0.0;
  double dv[NM], rv[NM], uv[NM + 1];
  double zh[H], nph[H];  // z and np, own rows
  int Av[NM + 1];
#pragma unroll
  for (int i = 0; i < NM; i++) dv[i] = rv[i] = 0.0;
#pragma unroll
  for (int k = 0; k < H; k++) zh[k] = nph[k] = 0.0;
#pragma unroll
  for (int i = 0; i <= NM; i++) {
    uv[i] = 0.0;
    Av[i] = 0;
  }
  double R_norm = 1.0;
  int iq = 0;

  // d = J^T np: own rows' partial sums, one pair sum per column
  auto compute_d = [&]() {
#pragma unroll
    for (int c = 0; c < NM; c++) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < H; k++) s += Jh[k][c] * nph[k];
      dv[c] = psum(s);
    }
  };
  // LoC: compile-time lower bound on iq
  auto update_z = [&](auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int k = 0; k < H; k++) {
      double z = 0.0;
#pragma unroll
      for (int j = LO; j < NM; j++)
        if (j >= iq) z += Jh[k][j] * dv[j];
      zh[k] = z;
    }
  };
  // (in the loop only the inequality rows i >= p of r feed anything: rows below LO = p skipped)
  auto update_r = [&](auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int i = NM - 1; i >= 0; i--) {
      if (i >= LO && i < iq) {
        double s = 0.0;
#pragma unroll
        for (int j = i + 1; j < NM; j++)
          if (j < LO || j < iq) s += Rv[RI::at(i, j)] * rv[j];
        rv[i] = ldiv<F>(dv[i] - s, Rv[RI::at(i, i)], fok);
      }
    }
  };
  // own-row dot products, summed over the pair
  auto pdot = [&](const double(&u_)[H], const double(&v_)[H]) -> double {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < H; k++) s += u_[k] * v_[k];
    return psum(s);
  };
  // The Givens step (qp_lane.hip's rot_fast): (a, b) -> (+-h, 0), rows (t1, t2) ->
  // (cc t1 + ss t2, ss t1 - cc t2); |h| < eps: the identity.  Coefficients from operands both
  // lanes hold; the rows are each lane's own.
  auto rot = [&](double& a_, double& b_, auto&& apply) {
    const double a0 = a_, b0_ = b_;
    const double hh = ldistance<F>(a0, b0_, fok);
    const bool skip = fabs(hh) < kEps;
    double cc, ss;
    if constexpr (F) {
      const double rh = frcp(hh);
      fok = fok && (skip || rcp_ok(rh));
      cc = fabs(a0) * rh;
      ss = (a0 < 0.0 ? -b0_ : b0_) * rh;
    } else {
      cc = fabs(a0) / hh;
      ss = (a0 < 0.0 ? -b0_ : b0_) / hh;
    }
    a_ = skip ? a0 : (a0 < 0.0 ? -hh : hh);
    b_ = skip ? b0_ : 0.0;
    const double c1_ = skip ? 1.0 : cc, s1_ = skip ? 0.0 : ss;
    const double c2_ = skip ? -1.0 : cc, s2_ = skip ? 0.0 : ss;
    apply([&](double& t1r, double& t2r) {
      const double t1 = t1r, t2 = t2r;
      t1r = c1_ * t1 + s1_ * t2;
      t2r = s2_ * t1 - c2_ * t2;
    });
  };
  auto add_constraint = [&](auto LoC) -> bool {
    constexpr int LO = decltype(LoC)::value;
    if (iq >= n) return false;  // reference UB (p > n); reported as dependent
#pragma unroll
    for (int j = NM - 1; j >= LO + 1; j--) {
      if (j >= iq + 1) {
        rot(dv[j - 1], dv[j], [&](auto&& r_) {
#pragma unroll
          for (int k = 0; k < H; k++) r_(Jh[k][j - 1], Jh[k][j]);
        });
      }
    }
    iq++;
    // R[:iq, iq-1] = d[:iq]
#pragma unroll
    for (int c = LO; c < NM; c++)
#pragma unroll
      for (int i = 0; i <= c; i++) {
        const bool w = (c == iq - 1);
        Rv[RI::at(i, c)] = w ? dv[i] : Rv[RI::at(i, c)];
      }
    const double dd = fabs(lsel_lo<LO < NM ? LO : NM - 1>(dv, iq - 1));
    if (dd <= kEps * R_norm) return false;
    R_norm = (R_norm < dd) ? dd : R_norm;
    return true;
  };
  auto delete_constraint = [&](int l, auto LoC) {
    constexpr int LO = decltype(LoC)::value;  // qq >= LO (the deleted constraint is an inequality)
    int qq = 0;
    bool found = false;
#pragma unroll
    for (int k = 0; k <= NM; k++)
      if (!found && k >= p && k < iq && Av[k] == l) {
        qq = k;
        found = true;
      }
#pragma unroll
    for (int i = LO; i < NM; i++)
      if (i >= qq && i < iq - 1) {
        Av[i] = Av[i + 1];
        uv[i] = uv[i + 1];
      }
#pragma unroll
    for (int c = LO; c < NM - 1; c++) {
      const bool sh = (c >= qq && c < iq - 1);
#pragma unroll
      for (int r = 0; r <= c + 1 && r < NM; r++) Rv[RI::at(r, c)] = sh ? Rv[RI::at(r, c + 1)] : Rv[RI::at(r, c)];
    }
    {
      const int aiq = lsel_lo<LO>(Av, iq);
      const double uiq = lsel_lo<LO>(uv, iq);
      lput_lo<LO>(Av, iq - 1, aiq);
      lput_lo<LO>(uv, iq - 1, uiq);
      lput_lo<LO>(Av, iq, 0);
      lput_lo<LO>(uv, iq, 0.0);
    }
#pragma unroll
    for (int c = LO; c < NM; c++)
#pragma unroll
      for (int r = 0; r <= c + 1 && r < NM; r++) {
        const bool z = (c == iq - 1) && (r < iq);
        Rv[RI::at(r, c)] = z ? 0.0 : Rv[RI::at(r, c)];
      }
    iq--;
    if (iq == 0) return;
#pragma unroll
    for (int j = LO; j < NM - 1; j++) {
      if (j >= qq && j < iq) {
        rot(Rv[RI::at(j, j)], Rv[RI::at(j + 1, j)], [&](auto&& r_) {
#pragma unroll
          for (int k = j + 1; k < NM; k++)
            if (k < iq) r_(Rv[RI::at(j, k)], Rv[RI::at(j + 1, k)]);
#pragma unroll
          for (int k = 0; k < H; k++) r_(Jh[k][j], Jh[k][j + 1]);
        });
      }
    }
  };
  const auto kZero = std::integral_constant<int, 0>{};

  // ---------------------------------------------------------------- equality phase
  // Fully unrolled, iq = i at step i.  Each step issues its CE loads before its part of the CI
  // copy: vector-memory waits count in issue order, so consuming them waits only for copy parts
  // issued kCeAhead steps earlier, not for the pieces streaming in behind them (issued the other
  // way round, every step waited for the previous step's part: 43.6k instead of ~20k cycles per
  // wave, profiles/r04_s12).
  constexpr int kDmaFrom = QPGPU_PAIR_DMA_FROM >= 0 ? (QPGPU_PAIR_DMA_FROM < PX ? QPGPU_PAIR_DMA_FROM : PX - 1)
                                                   : (PX - 1 - kCeAhead > 0 ? PX - 1 - kCeAhead : 0);
  bool done = !ok_lane;
#pragma unroll
  for (int i = 0; i < PX; i++) {
    const double c0 = c0a[i];
#pragma unroll
    for (int k = 0; k < H; k++) nph[k] = cea[i][k];
    if (i + kCeAhead < PX) load_ce(i + kCeAhead < PX ? i + kCeAhead : 0);
    __builtin_amdgcn_sched_barrier(0);
    if (dma && i >= kDmaFrom) dma_ci_part(i - kDmaFrom, PX - kDmaFrom);  // every lane (per-wave copy)
    __builtin_amdgcn_sched_barrier(0);
    if (!done) {
      iq = i;
      compute_d();
      update_z(kZero);
      // (as qp_lane.hip: no update_r and no u[:i] update here: r and the equality constraints' multipliers u[0..p)
      // feed nothing — the active-set loop reads u only for the inequalities (t1, the dual step's
      // drop, the rollback) and x, f never use u — so their back-substitution is skipped; x, f, status and the l1 passes are unchanged)
      double t2 = 0.0;
      const double zz = pdot(zh, zh);
      const double znp = pdot(zh, nph);
      const double npx = pdot(nph, xh);
      if (fabs(zz) > kEps) t2 = ldiv<F>(-npx - c0, znp, fok);
#pragma unroll
      for (int k = 0; k < H; k++) xh[k] += t2 * zh[k];
      uv[i] = t2;
      fval += 0.5 * (t2 * t2) * znp;
      Av[i] = -i - 1;
      if (!add_constraint(kZero)) {
        status = QPGPU_QP_DEPENDENT;
        done = true;
      }
    }
  }
  if constexpr (PX > 0) {  // the warm-up loads retire here, long after they landed
    pf_ce.retire();
    pf_ce0.retire();
    pf_ci.retire();
    pf_ci0.retire();
    if (!dma) pf_cil.retire();
  }
  qp_stamp(a, 2);
  bool ci_ready = false;  // wave-uniform: the LDS copy of CI rows 0..kCiRows-1 is complete
  if (dma) {
    __syncthreads();  // the DMA has landed
    ci_ready = true;
  }
  if constexpr (F) {
    if (wave_any(!fok)) return false;
  }

  // ---------------------------------------------------------------- active-set loop
  // Wave-uniform loop; per-QP work is predicated on `active`, which both lanes of a pair share.
  constexpr int IQLO = PX;
  const auto kLo = std::integral_constant<int, IQLO>{};
  {
    double sv[MH];  // s of the own constraints
#pragma unroll
    for (int i = 0; i < MH; i++) sv[i] = 0.0;
    double xoldh[H], uold[NM];
    int aold[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) {
      uold[i] = 0.0;
      aold[i] = 0;
    }
#pragma unroll
    for (int k = 0; k < H; k++) xoldh[k] = 0.0;
    uint64_t act = 0;   // bit c set <=> iai[c] == -1
    uint64_t excl = 0;  // bit c set <=> iaexcl[c] == false
    int ip = 0, steps = 0;
    double ss = 0.0, ci0ip = 0.0;
    bool need_scan = true, need_select = true;
    bool active = !done;
    const int max_steps = a.max_steps;
    const double* CIall = a.CI + bs * (int64_t)(NM * MM);
    const double* CIown = CIall + h;  // own constraint i of row j at CIown[j * MM + 2 * i]
    const double* ci0all = a.ci0 + bs * MM;
    const double* ci0own = ci0all + h;
    constexpr int NG = NM - kCiRows + 1;  // rows read from global memory by a scan, then ci0

    auto scan_pass = [&]() {
      const bool do_scan = active && need_scan;
      if (wave_any(do_scan)) {
        // the whole x on both lanes of the pair
        double xf[NM];
#pragma unroll
        for (int k = 0; k < H; k++) {
          const double o = psw(xh[k]);
          xf[2 * k] = h ? o : xh[k];
          if (2 * k + 1 < NM) xf[2 * k + 1] = h ? xh[k] : o;
        }
        double psi = 0.0;
        if (do_scan) {
          iter++;
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k >= p && k < iq) act |= 1ull << Av[k];
#pragma unroll
          for (int i = 0; i < MH; i++) sv[i] = 0.0;
          if (ci_ready) {
            // the global rows (and ci0) in flight while the LDS rows are summed (same j order)
            double gbuf[NG][MH];
#pragma unroll
            for (int r = kCiRows; r < NM; r++)
#pragma unroll
              for (int i = 0; i < MH; i++) gbuf[r - kCiRows][i] = CIown[r * MM + 2 * i];
#pragma unroll
            for (int i = 0; i < MH; i++) gbuf[NG - 1][i] = ci0own[2 * i];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < NM; j++) {
              const double xj = xf[j];
              if (j < kCiRows) {
#pragma unroll
                for (int i = 0; i < MH; i++) sv[i] += sbl[ci_own_off(j, i)] * xj;
              } else {
#pragma unroll
                for (int i = 0; i < MH; i++) sv[i] += gbuf[j - kCiRows < NG ? j - kCiRows : 0][i] * xj;
              }
            }
#pragma unroll
            for (int i = 0; i < MH; i++) {
              sv[i] += gbuf[NG - 1][i];
              psi += (sv[i] < 0.0) ? sv[i] : 0.0;
            }
          } else {
            // the first scan without the DMA: rows from global memory two deep, rows
            // 0..kCiRows-1 written to the LDS copy on the way
            double rowbuf[2][MH];
            auto load_row = [&](int r, double* dst) {
              if (r < NM) {
#pragma unroll
                for (int i = 0; i < MH; i++) dst[i] = CIown[r * MM + 2 * i];
              } else if (r == NM) {
#pragma unroll
                for (int i = 0; i < MH; i++) dst[i] = ci0own[2 * i];
              }
            };
            load_row(0, rowbuf[0]);
#pragma unroll
            for (int j = 0; j < NM; j++) {
              load_row(j + 1, rowbuf[(j + 1) % 2]);
              __builtin_amdgcn_sched_barrier(0);
              const double xj = xf[j];
#pragma unroll
              for (int i = 0; i < MH; i++) sv[i] += rowbuf[j % 2][i] * xj;
              if (j < kCiRows) {
#pragma unroll
                for (int i = 0; i < MH; i++) sbl[ci_own_off(j, i)] = rowbuf[j % 2][i];
              }
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < MH; i++) {
              sv[i] += rowbuf[NM % 2][i];
              psi += (sv[i] < 0.0) ? sv[i] : 0.0;
            }
          }
        }
        if (!ci_ready && kCiRows > 0) {
          // the copy's elements are read across the pair from here on: the first scan's LDS
          // writes complete before any later read (one wave: LDS operations stay in order)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          ci_ready = true;
        }
        if (do_scan) {
          psi = psum(psi);
          excl = 0;
          ss = 0.0;
          ip = 0;
          if (fabs(psi) <= (double)m * kEps * c1 * c2 * 100.0) {
            active = false;  // optimal
          } else {
#pragma unroll
            for (int i = 0; i < NM; i++)
              if (i >= IQLO && i < iq) {
                uold[i] = uv[i];
                aold[i] = Av[i];
              }
#pragma unroll
            for (int k = 0; k < H; k++) xoldh[k] = xh[k];
          }
        }
      }
    };
    uint64_t tscan = 0, tsel = 0, nloop = 0;  // diagnostic stamps only
    while (wave_any(active)) {
      const uint64_t tl0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
      scan_pass();
      const uint64_t tl1 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
      tscan += tl1 - tl0;
      nloop++;
      // ---- l2: the most violated constraint (ss deliberately not reset: reference quirk).
      // Each lane takes the first minimum of its own constraints (strict <, ascending), then the
      // pair keeps the smaller value, or at equal values below ss the lower index — the
      // sequential scan's choice.
      if (active && need_select) {
        double sl = ss;
        int il = ip;
        const uint64_t taken = (act | excl) >> h;  // bit 2i: own constraint i is not eligible
#pragma unroll
        for (int i = 0; i < MH; i++) {
          const int c = 2 * i + h;
          const bool elig = !((taken >> (2 * i)) & 1ull);
          const bool take = sv[i] < sl && elig;
          sl = take ? sv[i] : sl;
          il = take ? c : il;
        }
        const double so = psw(sl);
        const int io = pswi(il);
        const double s0 = h ? so : sl, s1 = h ? sl : so;
        const int i0 = h ? io : il, i1 = h ? il : io;
        const bool one = s1 < s0 || (s1 == s0 && s1 < ss && i1 < i0);
        ss = one ? s1 : s0;
        ip = one ? i1 : i0;
        if (ss >= 0.0) {
          active = false;  // optimal
        } else {
#pragma unroll
          for (int k = 0; k < H; k++) {
            const int r = has_row(k) ? 2 * k + h : 0;
            if (2 * k + 1 < kCiRows) {  // both lanes' rows in the LDS copy
              nph[k] = ci_lds_at(r, ip);
            } else if (2 * k >= kCiRows) {  // neither
              const double vg = CIall[r * MM + ip];
              nph[k] = has_row(k) ? vg : 0.0;
            } else {
              const double vl = ci_lds_at(r < kCiRows ? r : 0, ip);
              const double vg = CIall[r * MM + ip];
              nph[k] = r < kCiRows ? vl : vg;
            }
          }
          ci0ip = ci0all[ip];
          lput_lo<IQLO>(uv, iq, 0.0);
          lput_lo<IQLO>(Av, iq, ip);
        }
      }
      if (a.stamps) {
        const double sink = nph[0] + ci0ip;
        asm volatile("" ::"v"(sink));
        tsel += __builtin_amdgcn_s_memtime() - tl1;
      }
      // ---- l2a
      if (active) {
        if (max_steps > 0 && ++steps > max_steps) {
          status = QPGPU_QP_MAX_ITER;
          active = false;
        } else {
          compute_d();
          update_z(kLo);
          update_r(kLo);
          int l = 0;
          double t1 = inf;
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k >= p && k < iq && rv[k] > 0.0) {
              const double q_ = ldiv<F>(uv[k], rv[k], fok);
              const bool take = q_ < t1;
              t1 = take ? q_ : t1;
              l = take ? opq_l(Av[k]) : l;
            }
          const double zz = pdot(zh, zh);
          const double znp = pdot(zh, nph);
          // s[ip] from the lane that owns constraint ip
          const double so = lsel<MH>(sv, ip >> 1);
          const double sp = psw(so);
          const double sip = ((ip & 1) == h) ? so : sp;
          double t2;
          if (fabs(zz) > kEps) {
            t2 = ldiv<F>(-sip, znp, fok);
            if (t2 < 0) t2 = inf;  // Takano Akio patch
          } else {
            t2 = inf;
          }
          const double t = (t2 < t1) ? t2 : t1;
          // the step's outcomes as predicates over one copy of each piece (qp_lane.hip)
          const bool infs = t >= inf;
          const bool dual = !infs && t2 >= inf;
          const bool prim = !infs && !dual;
          const bool fullst = prim && fabs(t - t2) < kEps;
          const bool part = prim && !fullst;
          if (infs) {
            status = QPGPU_QP_INFEASIBLE;
            fval = inf;
            active = false;
          }
          if (prim) {
#pragma unroll
            for (int k = 0; k < H; k++) xh[k] += t * zh[k];
            fval += t * znp * (0.5 * t + lsel_lo<IQLO>(uv, iq));
          }
          if (dual || prim) {
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k >= IQLO && k < iq) uv[k] -= t * rv[k];  // (u[0..p) are never read)
            lput_lo<IQLO>(uv, iq, lsel_lo<IQLO>(uv, iq) + t);
          }
          bool add_fail = false;
          if (fullst) {
            if (!add_constraint(kLo)) {
              add_fail = true;
              excl |= 1ull << ip;
            } else {
              act |= 1ull << ip;
              need_scan = need_select = true;
            }
          }
          if (dual || part) act &= ~(1ull << l);
          if (dual || part || add_fail) delete_constraint((dual || part) ? l : ip, kLo);
          if (add_fail) {  // degenerate: roll back to the l1 state, select again
            act = 0;
#pragma unroll
            for (int i = 0; i < NM; i++)
              if (i >= p && i < iq) {
                Av[i] = aold[i];
                uv[i] = uold[i];
                act |= 1ull << Av[i];
              }
#pragma unroll
            for (int k = 0; k < H; k++) xh[k] = xoldh[k];
            need_scan = false;
            need_select = true;
          }
          if (part) {  // refresh s[ip] = CI[:,ip]^T x + ci0[ip] on the lane that owns ip
            const double s = pdot(nph, xh) + ci0ip;
            const int li = ((ip & 1) == h) ? (ip >> 1) : -1;
#pragma unroll
            for (int i = 0; i < MH; i++) sv[i] = (i == li) ? s : sv[i];
          }
          if (dual || part) need_scan = need_select = false;
        }
      }
    }
    if (a.stamps && lane == 0) {
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 5] = tscan;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 6] = tsel;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 7] = nloop;
    }
  }
  qp_stamp(a, 3);
  if constexpr (F) {
    if (wave_any(!fok)) return false;
  }

  if (live) {
    if (chol_ok) {
      double* xb = a.x + b * (int64_t)NM + h;
#pragma unroll
      for (int k = 0; k < H; k++)
        if (has_row(k)) xb[2 * k] = xh[k];
    }
    if (h == 0) {
      a.f[b] = fval;
      a.status[b] = status;
      if (a.iters) a.iters[b] = iter;
    }
  }
  qp_stamp(a, 4);
  return true;
}

template <int NM, int MM, int PX>
__global__ void __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(2)))
qp_pair_fast_kernel(const QpArgs a) {
  __shared__ double sbuf[kStage];
  if (!pair_body<NM, MM, PX, false>(a, sbuf)) {
    __syncthreads();  // the fast attempt's LDS traffic is over
    pair_body<NM, MM, PX, true>(a, sbuf);
  }
}

struct PairVariant {
  int n, p, m;
  const char* name;
  void (*kernel)(const QpArgs);
};

static const PairVariant kPairVariants[] = {
    {7, 6, 14, "qp_pair_fast<N=7,P=6,M=14>", qp_pair_fast_kernel<7, 14, 6>},
};

const PairVariant* pick_pair(int n, int p, int m) {
  for (const auto& v : kPairVariants)
    if (n == v.n && p == v.p && m == v.m) return &v;
  return nullptr;
}

}  // namespace qpk_pair

// The pair kernel covers exactly its instantiated (n, p, m) in the QP-major layout, without the
// m = 0 snapshot (qpgpu_solve_batched_eq); anything else is left to the other families.
extern "C" hipError_t qpk_launch_pair(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                      const char** name) {
  const qpk_pair::PairVariant* v = qpk_pair::pick_pair(a->n, a->p, a->m);
  if (!v || a->tile != 1 || a->x_eq) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  const int64_t blocks = (a->batch + qpk_pair::kQpw - 1) / qpk_pair::kQpw;
  hipLaunchKernelGGL(v->kernel, dim3((unsigned)blocks), dim3(64), 0, stream, *a);
  return hipGetLastError();
}

extern "C" const char* qpk_pair_name(int n, int p, int m) {
  const qpk_pair::PairVariant* v = qpk_pair::pick_pair(n, p, m);
  return v ? v->name : nullptr;
}
