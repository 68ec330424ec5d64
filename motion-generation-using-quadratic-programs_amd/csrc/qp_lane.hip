// qp_lane.hip — gfx950 batched Goldfarb–Idnani solver, ONE QP PER LANE (n <= 8, m <= 16).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; operation order
// of the prebuilt libquadprog.a fixed in SURVEY.md §3.2) for the 64 QPs of one wavefront.
//
// Why one QP per lane: at these sizes the cost is the serial chain of every QP (Givens
// coefficients = 4 IEEE divisions + 1 sqrt each, back-substitutions, step lengths); running it
// once per QP instead of once per lane of a subgroup cuts issued instructions ~4x versus
// qp_small.hip.  65 536 QPs are exactly one wave per SIMD (1 024 SIMDs), so a launch is as long
// as its slowest wave and every wave's latency is exposed.  State placement (gfx950: 512
// VGPR+AGPR per lane at 1 wave/SIMD, 160 KiB LDS per CU = 40 KiB per wave at 4 waves/CU):
//   * J (= L^{-T}), R (upper triangle + first subdiagonal, the only entries the algorithm makes
//     non-zero), x, z, d, np, u, r, A, s and the loop's rollback copies live in registers for
//     the whole solve, indexed only with compile-time indices (fully unrolled loops with
//     run-time predicates);
//   * G, g0, CE, ce0 are brought in by LDS-DMA (global_load_lds_dwordx4) of the wave's 64
//     contiguous QP blocks into a 40 KiB staging buffer and read per lane from it;
//   * CI / ci0 (QP-major EXACT shapes): the first l1 scan reads them from global memory (their
//     cache lines were touched during the equality phase) and leaves them on chip — rows
//     0..kCiRows-1 in the LDS staging buffer, and (C1-sized shapes with an equality phase) the
//     remaining rows and ci0 in AGPRs — so later scans and the selected-column gathers issue no
//     global loads at all.
// IEEE binary64 throughout, no contraction: results are bitwise identical to the CPU
// restatement (oracle/qp_oracle.c), which tests/ check.
//
// The same source built a second time with QPGPU_LANE_FAST=1 and -ffp-contract=fast
// (qp_lane_fast.hip) is the QPGPU_FLAG_FAST kernel: same algorithm and decisions, but multiply-
// adds fused, every division by a shared divisor a multiplication by one refined reciprocal
// (Cholesky columns, J = L^-T, the solve, the Givens coefficients), and the rotation length as
// sqrt(a^2 + b^2) for operands well inside the exponent range — within north_star's 1e-10
// relative of the reference instead of bit-identical.
#include <type_traits>

#include "qp_common.h"

#ifndef QPGPU_LANE_FAST
#define QPGPU_LANE_FAST 0
#endif
#if QPGPU_LANE_FAST
#define QPK_LANE_NS qpk_fast
#define QP_LANE_KERNEL qp_lane_fast_kernel
#define QPK_LANE_C(name) name##_fast
#else
#define QPK_LANE_NS qpk
#define QP_LANE_KERNEL qp_lane_kernel
#define QPK_LANE_C(name) name
#endif

// Diagnostic s_memtime stamps (tools/stamps.py): compiled in (QPGPU_LANE_STAMPS = 1), each one a
// wave-uniform null test of a.stamps unless a stamp buffer is passed; 0 removes them (measured
// the same C1 time either way, profiles/r05_s8), 2 adds the loop's l2a split.
#ifndef QPGPU_LANE_STAMPS
#define QPGPU_LANE_STAMPS 1
#endif

namespace QPK_LANE_NS {
using namespace qpk;
constexpr bool kFast = QPGPU_LANE_FAST != 0;
constexpr bool kStamps = QPGPU_LANE_STAMPS != 0;
__device__ __forceinline__ void lstamp(const QpArgs& a, int slot) {
  if constexpr (kStamps) qp_stamp(a, slot);
}

// opq_l, lsel_lo, lsel, lput_lo, RIdx, wave_any: qp_common.h (shared with qp_pair.hip)

// A double parked in two AGPRs.  VALU cannot operate on AGPRs, but v_accvgpr_read/write move a
// dword in one issue slot, far cheaper than the L2 / Infinity-Cache round trip the scan would
// otherwise pay; the "a" constraints make the register allocator keep these values in the
// accumulator half of the unified file, which the C1 kernel leaves mostly unused.  The reads
// are volatile so that they stay where the values are consumed (a hoisted read would move the
// value back into a VGPR for the whole loop).
struct AgprD {
  uint32_t lo, hi;
};
__device__ __forceinline__ AgprD to_agpr(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  AgprD a;
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a.lo) : "v"((uint32_t)u));
  asm("v_accvgpr_write_b32 %0, %1" : "=a"(a.hi) : "v"((uint32_t)(u >> 32)));
  return a;
}
__device__ __forceinline__ double from_agpr(const AgprD& a) {
  uint32_t lo, hi;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(lo) : "a"(a.lo));
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(hi) : "a"(a.hi));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

constexpr int kQpw = 64;      // QPs per wave: one per lane
// Two waves per SIMD (QPGPU_LANE_OCC2, an A/B build for VERDICT r05 item 6): 256 registers per
// lane and a 20 KiB stage (eight waves per CU); G and CE no longer stage, each lane loads its own
// from global memory, and the LDS copy of CI shrinks to the rows the smaller stage holds.
#ifndef QPGPU_LANE_OCC2
#define QPGPU_LANE_OCC2 0
#endif
constexpr int kLaneOcc = QPGPU_LANE_OCC2 ? 2 : 1;
constexpr int kStage = QPGPU_LANE_OCC2 ? 2560 : 5120;  // staging buffer, doubles (40 KiB: 4 waves per CU)
// The first l1 scan (which fills the on-chip CI copy) is software-pipelined two rows deep: row
// j+1's loads are issued (and fenced from the scheduler) before row j is consumed, so one memory
// latency covers two rows instead of the scheduler's one-load-at-a-time minimum-pressure order.
constexpr int kScanDepth = 2;
// p = 0 (no equality phase): copy CI rows into LDS by DMA at the end of the setup (1) or let the
// first scan load them (0).  Measured on C2 (profiles/r03_s6): 83.6 us with the DMA, 72.9 without
// — the DMA's per-lane 16-B pieces take ~23k cycles per wave to issue, the first scan's direct
// loads 18.5k, and nothing hides either — so 0; with p > 0 the equality phase hides the DMA.
// 2: a part per Cholesky row (profiles/r06_s15: 75.2 us per launch against 67.6-68.0 with 0,
// pipelined 1.489e9 against 1.449e9 solves/s — an A/B value, not the default).
#ifndef QPGPU_LANE_DMA_P0
#define QPGPU_LANE_DMA_P0 0
#endif
// Where the DMA path touches the CI rows past the LDS copy and ci0 (one dword per 128-B line)
// ahead of the first scan: 0 = nowhere, the first scan loads them (the product since round 5),
// 1 = after the CE -> AGPR move (rounds 3-4), 2 = at the last equality step.  Measured on C1
// (profiles/r05_s3): FETCH 146.4 / 125.0 / 130.1 MB for 1 / 0 / 2 — the touched lines leave L2
// before the first scan reads them, so the touch only adds a second fetch — at 44.6 / 44.8 /
// 45.7 us (two runs each; 0 and 1 within the run-to-run spread).
// Where the setup waits for round B (CE / ce0 into LDS): 1 = after J = L^-T and the solve, which
// need only the factor, 0 = right after the Cholesky (rounds 1-4; A/B only)
#ifndef QPGPU_LANE_CE_LATE
#define QPGPU_LANE_CE_LATE 1
#endif
#ifndef QPGPU_LANE_WARMUP
#define QPGPU_LANE_WARMUP 0
#endif
// The fast build's invalid-fast-form check at the top of every loop pass as well (1, the
// product since round 5) or only after the equality phase and after the loop (0); 2 = compiled
// in but never taken (A/B only).  Round 4 dropped it after a wrong-result run that no committed
// source reproduces (profiles/r05_s2, r05_s3).
#ifndef QPGPU_LANE_LOOPTOP_EXIT
#define QPGPU_LANE_LOOPTOP_EXIT 1
#endif

// ---- arithmetic of the fast build (frcp, rcp_ok, ldiv_r, ldiv, ldistance): qp_common.h,
// shared with the lane-pair kernel (qp_pair.hip).

// PX >= 0: p is the compile-time constant PX as well (C1/C4: 6, C2: 0), which folds every
// [p, iq) loop of the active-set phase (for n = 7, p = 6 that range holds at most one entry).
// The solve of one wave's 64 QPs.  SAFE: the IEEE forms of division and distance (the exact
// build always; the fast build's fallback).  Returns false as soon as a fast form was not
// valid for some lane (checked after the equality phase and after the loop): x, f, status
// and iters are not written then, and the caller re-solves the wave with SAFE, which rewrites
// everything — including the m = 0 snapshot (x_eq, f_eq, st_eq) the fast attempt may already
// have written.  In the fast build (-ffp-contract=fast) the SAFE body's multiply-adds are
// contracted too: a fallback wave keeps the reference's divisions and distance(), not its
// bitwise results (still within 1e-10).
template <int NM, int MM, int T, bool EXACT, int PX, bool SAFE>
__device__ __forceinline__ bool lane_body(const QpArgs& a, double* sbuf) {
  static_assert(MM <= 64, "bitmask bookkeeping holds m <= 64");
  using RI = RIdx<NM>;
  constexpr int STAGE = kStage;
  constexpr bool F = kFast && !SAFE;
  bool fok = true;  // F: every fast form so far was valid on this lane
  // CI / ci0 cache warm-up before the equality phase: only with an equality phase long enough
  // for the loads to land (p > 0 or p unknown).  Measured for p = 0 (no equality phase): the
  // first scan then waits on the same burst either way (profiles/r02_s2, r02_s46).
  constexpr bool kLanePrefetch = PX != 0;

  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kQpw;
  const int64_t b = b0 + lane;
  const int valid = (int)min<int64_t>(kQpw, a.batch - b0);
  const bool live = lane < valid;

  // EXACT: the shape is (NM, *, MM), so every element offset is a compile-time constant
  const int n = EXACT ? NM : a.n;
  const int m = EXACT ? MM : a.m;
  const int p = PX >= 0 ? PX : a.p;
  const double inf = dinf();

  // The wave's 64 QPs occupy [X + b0*E, X + (b0+64)*E) in both layouts (TILED64 arrays hold
  // whole tiles, so its waves are always full).  Staging copies a contiguous span of that
  // range into sbuf with LDS-DMA (global_load_lds_dwordx4: 1 KiB per wave-instruction, no
  // VGPRs, everything in flight at once); a partial last QP-major wave copies per lane.
  const bool full = (T == 64) || (valid == kQpw);
  auto copy_chunk = [&](const double* src, int nd, int off, int k) {  // doubles [k, k+128)
    const int e = k + 2 * lane;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(e < nd ? src + e : src),
                                     (__attribute__((address_space(3))) void*)(sbuf + off + k), 16, 0, 0);
  };
  auto copy_span = [&](const double* src, int nd, int off) {  // nd even, full waves only
#pragma unroll 4
    for (int k = 0; k < nd; k += 128) copy_chunk(src, nd, off, k);
  };
  // whole tile of X (E doubles per QP) -> sbuf[off...]
  auto stage_all = [&](const double* X, int E, int off) {
    if (full) {
      copy_span(X + b0 * (int64_t)E, kQpw * E, off);
    } else if (live) {
      const double* src = X + b * (int64_t)E;
      for (int e = 0; e < E; e++) sbuf[off + lane * E + e] = src[e];
    }
  };
  auto rd_all = [&](int off, int E, int k) -> double {
    if constexpr (T == 64)
      return sbuf[off + k * 64 + lane];
    else
      return sbuf[off + lane * E + k];
  };
  auto view = [&](double* X, int E) -> double* {
    if constexpr (T == 64)
      return X + b0 * (int64_t)E + lane;
    else
      return X + b * (int64_t)E;
  };

  int status = QPGPU_QP_OK;
  double fval = 0.0;
  int iter = 0;
  double xv[NM];
#pragma unroll
  for (int i = 0; i < NM; i++) xv[i] = 0.0;
  double c1 = 0.0, c2 = 0.0;
  // LDS regions: the bottom of the buffer stages G (setup), then CE / ce0 (equality phase),
  // then rows 0..kCiRows-1 of every lane's CI for the active-set loop (16-B pieces, piece k of
  // lane l at doubles (k*64 + l)*2).  RB, at the top, stages g0.
  constexpr int RB = (STAGE - kQpw * NM) / 2 * 2;
  // G and g0 stage through LDS when they fit (the product); else each lane loads its own
  constexpr bool kStageG = RB >= kQpw * NM * NM;
  static_assert(kStageG || QPGPU_LANE_OCC2, "G and g0 staging exceed the stage buffer");
  // CI rows held in LDS through the loop (EXACT QP-major shapes)
  constexpr int kCiRowsFit = (RB / kQpw) / MM;
  constexpr int kCiRows = (EXACT && T == 1 && MM % 2 == 0) ? (kCiRowsFit < NM ? kCiRowsFit : NM) : 0;
  // Rows 0..kCiRows-1 of every lane's CI go straight from HBM into that LDS copy by per-lane
  // LDS-DMA while the setup / equality phase computes (kCiDma: p compile-time, CI 16-B aligned),
  // so the first l1 scan finds them on chip instead of re-reading all of CI from the Infinity
  // Cache after a cache warm-up (that re-read was 11k of a wave's ~88k cycles, profiles/r03_s3).
  // With p > 0 the CE / ce0 staging occupies the LDS then, so once it has landed it moves to
  // AGPRs (ceag, read back once per equality step) and the DMA takes its place.
  constexpr bool kCiDma = kCiRows > 0 && (PX > 0 || (PX == 0 && QPGPU_LANE_DMA_P0));
  constexpr int kCeN = PX > 0 ? NM * PX + PX : 1;  // CE (n x p) then ce0 (p)
  [[maybe_unused]] AgprD ceag[kCiDma ? kCeN : 1];
  const bool dma = kCiDma && (a.flags & kArgAligned16);
  double Jreg[NM][NM];  // J lives in registers for the whole solve
  bool ce_staged = false;
  bool ce_agpr = false;
  // cache warm-up: one dword per 128-B line of this lane's CI / ci0 blocks — with kCiDma only
  // the rows past the LDS copy (which the scans keep reading from L2)
  constexpr int kPfCI = (NM * MM * 8 + 127) / 128 + 1, kPfC0 = (MM * 8 + 127) / 128 + 1;
  [[maybe_unused]] uint32_t pf[kPfCI + kPfC0];
  bool warmed = false;  // the warm-up loads were issued (they retire after the equality phase)
  auto warmup = [&]() {
    warmed = true;
    if (live) {
      const int off = dma ? kCiRows * MM * 8 : 0;  // (repeats the last line when shorter)
      const char* c = reinterpret_cast<const char*>(a.CI + b * (int64_t)(n * m)) + off;
      const char* c0 = reinterpret_cast<const char*>(a.ci0 + b * (int64_t)m);
      const int bc = n * m * 8 - off, b0c = m * 8;
#pragma unroll
      for (int k = 0; k < kPfCI; k++)
        pf[k] = (bc >= 4) ? *reinterpret_cast<const uint32_t*>(c + min(k * 128, bc - 4)) : 0u;
#pragma unroll
      for (int k = 0; k < kPfC0; k++)
        pf[kPfCI + k] = (b0c >= 4) ? *reinterpret_cast<const uint32_t*>(c0 + min(k * 128, b0c - 4)) : 0u;
    }
  };
  // rows 0..kCiRows-1 of this lane's CI block -> LDS piece k at doubles (k*64 + lane)*2 (the
  // scans' layout): one global_load_lds_dwordx4 per 16-B piece, a per-lane source address and
  // the wave-uniform LDS base.  Lanes past the batch copy lane 0's block (never read).  Issued
  // part by part between compute steps (part `part` of `parts`): all 35 pieces at once stall
  // the wave's issue until HBM has delivered most of them (the CU's memory queues fill), which
  // serialised the whole CI transfer with the setup (+25k cycles per wave, profiles/r03_s4).
  constexpr int kCiPieces = kCiRows * MM / 2;
  auto dma_ci_part = [&](int part, int parts) {
    const int per = (kCiPieces + parts - 1) / parts;
    const double* src = a.CI + (live ? b : b0) * (int64_t)(NM * MM);
#pragma unroll
    for (int k = 0; k < kCiPieces; k++)
      if (k >= part * per && k < (part + 1) * per)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 2 * k),
                                         (__attribute__((address_space(3))) void*)(sbuf + k * 2 * kQpw),
                                         16, 0, 0);
  };
  lstamp(a, 0);

  // ---------------------------------------------------------------- setup
  bool chol_ok = live;  // idle lanes (past the batch) never touch LDS slots
  double bad_sum = 0.0;
  {
    double Gr[NM][NM];
    // round A: G and g0
    const int offg0 = RB;
    if constexpr (kStageG) {
      stage_all(a.G, n * n, 0);
      stage_all(a.g0, n, offg0);
    }
    __syncthreads();
    // The LDS reads are unconditional (in range for every lane; an idle lane's slot holds stale
    // data that the select drops): a read under `live` becomes one exec-masked block per element,
    // which the scheduler can neither pair nor overlap.
    double g0v[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) {
#pragma unroll
      for (int j = 0; j < NM; j++) {
        double v;
        if constexpr (kStageG)
          v = (i < n && j < n) ? rd_all(0, n * n, i * n + j) : 0.0;
        else
          v = (live && i < n && j < n) ? view(const_cast<double*>(a.G), n * n)[(i * n + j) * T] : 0.0;
        Gr[i][j] = live ? v : 0.0;
      }
      double v0;
      if constexpr (kStageG)
        v0 = i < n ? rd_all(offg0, n, i) : 0.0;
      else
        v0 = (live && i < n) ? view(const_cast<double*>(a.g0), n)[i * T] : 0.0;
      g0v[i] = live ? v0 : 0.0;
    }
    __syncthreads();
    lstamp(a, 9);  // diagnostic: G / g0 in registers
    // round B: CE and ce0 (equality phase), landing during the Cholesky, the J build and the
    // solve.  A full wave issues its span a part per Cholesky row: issued at once, its LDS-DMA
    // instructions held the wave's issue until most of the data had arrived (the CU's memory
    // queues fill), which serialised the transfer with the Cholesky.
    const int npB = n * p;
    const int offcB = (kQpw * npB + 127) / 128 * 128;
    const bool stageB = p > 0 && offcB + kQpw * p <= STAGE;
    auto round_b = [&](int part, int parts) {
      if (!stageB) return;
      if (!full) {
        if (part == 0) {
          stage_all(a.CE, npB, 0);
          stage_all(a.ce0, p, offcB);
        }
        return;
      }
      const int nce = (kQpw * npB + 127) / 128, tot = nce + (kQpw * p + 127) / 128;
      const int per = (tot + parts - 1) / parts;
      const double* ce = a.CE + b0 * (int64_t)npB;
      const double* c0 = a.ce0 + b0 * (int64_t)p;
      for (int c = part * per; c < min(tot, (part + 1) * per); c++) {
        if (c < nce)
          copy_chunk(ce, kQpw * npB, 0, c * 128);
        else
          copy_chunk(c0, kQpw * p, offcB, (c - nce) * 128);
      }
    };
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) c1 += Gr[i][i];
    // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored
#pragma unroll
    for (int i = 0; i < NM; i++) {
      round_b(i, NM);  // every lane (the copy is per wave)
      // p = 0 (no round B, no equality phase): the CI copy a part per Cholesky row instead
      // (QPGPU_LANE_DMA_P0 = 2; G has left the LDS for registers at the barrier above)
      if constexpr (kCiDma && PX == 0 && QPGPU_LANE_DMA_P0 == 2)
        if (dma) dma_ci_part(i, NM);
      if (i < n && chol_ok) {
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
          for (int j = i + 1; j < NM; j++)
            if (j < n) {
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
    if ((a.flags & QPGPU_FLAG_WRITE_FACTOR) && live) {
      double* Gw = view(a.G, n * n);
#pragma unroll
      for (int i = 0; i < NM; i++)
#pragma unroll
        for (int j = 0; j < NM; j++)
          if (i < n && j < n) Gw[(i * n + j) * T] = Gr[i][j];
    }
    // round B lands: the staged CE / ce0 are read in the equality phase
    auto land_round_b = [&]() {
    if (p > 0) {
      const int np_ = n * p;
      const int offc = (kQpw * np_ + 127) / 128 * 128;
      ce_staged = offc + kQpw * p <= STAGE;
      __syncthreads();
      lstamp(a, 10);  // diagnostic: round B (CE) landed
      if constexpr (kCiDma && PX > 0) {
        if (dma && ce_staged) {
          // CE / ce0 -> AGPRs, then the LDS is the CI copy's (round C)
#pragma unroll
          for (int e = 0; e < NM * PX; e++) {
            const double v = rd_all(0, np_, e);
            ceag[e] = to_agpr(live ? v : 0.0);
          }
#pragma unroll
          for (int e = 0; e < PX; e++) {
            const double v = rd_all(offc, p, e);
            ceag[NM * PX + e] = to_agpr(live ? v : 0.0);
          }
          ce_agpr = true;
          __syncthreads();
          lstamp(a, 11);  // diagnostic: CE in AGPRs
          // the rows past the LDS copy (and ci0) warmed here; the copy itself goes a part per
          // equality step.  Measured (profiles/r03_s10): C1 kernel 47.4 us with the warm-up
          // here, 48.6 without it, 49.9 with it at the first equality step
          if constexpr (QPGPU_LANE_WARMUP == 1) warmup();
        }
      }
    }
    };
    // QPGPU_LANE_CE_LATE: wait for round B after J = L^-T and the solve (which need only the
    // factor), so the CE transfer lands under them instead of stalling the wave after the Cholesky
    if constexpr (!QPGPU_LANE_CE_LATE) land_round_b();
    if (chol_ok) {
      // J = L^{-T}: row r of J = L^{-1} e_r (forward_elimination); c2 = trace(J).
      // With a finite L the first r entries of L^{-1} e_r are exactly +0.0 (0.0 - L*(+0) and
      // 0.0 / L stay +0.0) and contribute exact zeros to later sums, so they are skipped: same
      // bits, ~40% fewer divisions.  A non-finite L (NaN inputs) takes the literal path.
      bool lfin = true;
#pragma unroll
      for (int i = 0; i < NM; i++)
#pragma unroll
        for (int j = 0; j <= i; j++)
          if (i < n) lfin = lfin && (fabs(Gr[i][j]) < inf);
      // fast build: one reciprocal per pivot serves the J build and the solve
      double rdiag[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) rdiag[i] = (F && i < n) ? frcp(Gr[i][i]) : 0.0;
      auto build_j = [&](const bool skip) {
#pragma unroll
        for (int r = 0; r < NM; r++) {
          double y[NM];
#pragma unroll
          for (int i = 0; i < NM; i++) {
            double v = 0.0;
            if (r < n && i < n && !(skip && i < r)) {
              v = (i == r) ? 1.0 : 0.0;
#pragma unroll
              for (int j = 0; j < i; j++)
                if (!(skip && j < r)) v -= Gr[i][j] * y[j];
              v = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
            }
            y[i] = v;
          }
#pragma unroll
          for (int j = 0; j < NM; j++) Jreg[r][j] = y[j];
          if (r < n) c2 += y[r];
        }
      };
      // (fast build: the skipping form unless some lane's factor is non-finite, decided per
      // wave so that the two forms stay separate code)
      if (F ? !wave_any(!lfin) : lfin)
        build_j(true);
      else
        build_j(false);
      // cholesky_solve (@.text+0x31a2): x = -G^{-1} g0
      double y[NM];
#pragma unroll
      for (int i = 0; i < NM; i++) {
        double v = 0.0;
        if (i < n) {
          v = g0v[i];
#pragma unroll
          for (int j = 0; j < i; j++) v -= Gr[i][j] * y[j];
          v = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
        }
        y[i] = v;
      }
#pragma unroll
      for (int i = NM - 1; i >= 0; i--) {
        if (i < n) {
          double v = y[i];
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < n) v -= Gr[i][j] * xv[j];
          xv[i] = ldiv_r<F>(v, Gr[i][i], rdiag[i], fok);
        }
      }
#pragma unroll
      for (int i = 0; i < NM; i++) xv[i] = -xv[i];
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) fval += g0v[i] * xv[i];
      fval = 0.5 * fval;
    }
    if constexpr (QPGPU_LANE_CE_LATE) land_round_b();
  }
  if constexpr (kCiDma && PX == 0) {
    // no equality phase to hide the copy behind: issued after the setup, all at once (the first
    // scan waits for it either way; during the Cholesky its issue stalls the setup's compute)
    if (dma) {
      if constexpr (QPGPU_LANE_DMA_P0 != 2) dma_ci_part(0, 1);
      warmup();
    }
  }
  lstamp(a, 1);
  // Without the DMA: touch every cache line of this lane's CI and ci0 blocks before the
  // equality phase: the loads complete during it (nothing waits on them until its end), so the
  // first l1 scan reads L2 / MALL instead of queueing on one chip-wide HBM burst.  Issued after
  // the setup: vmcnt waits are in issue order, so earlier they would also delay the G / CE
  // waits (measured slower, profiles/r02_s4).
  if constexpr (T == 1 && kLanePrefetch) {
    if (!ce_agpr) warmup();
  }
  if (!chol_ok) {
    status = QPGPU_QP_NOT_POSITIVE_DEFINITE;
    fval = bad_sum;
  }
  const bool ok_lane = live && chol_ok;

  // ---------------------------------------------------------------- state
  double Rv[RI::SIZE];
#pragma unroll
  for (int i = 0; i < RI::SIZE; i++) Rv[i] = 0.0;
  double dv[NM], zv[NM], npv[NM], uv[NM + 1], rv[NM];
  int Av[NM + 1];
#pragma unroll
  for (int i = 0; i < NM; i++) dv[i] = zv[i] = npv[i] = rv[i] = 0.0;
#pragma unroll
  for (int i = 0; i <= NM; i++) {
    uv[i] = 0.0;
    Av[i] = 0;
  }
  double R_norm = 1.0;
  int iq = 0;

  auto compute_d = [&]() {
#pragma unroll
    for (int c = 0; c < NM; c++) {
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NM; j++)
        if (j < n) s += Jreg[j][c] * npv[j];
      dv[c] = s;
    }
  };
  // LoC: compile-time lower bound on iq (see add_constraint below)
  auto update_z = [&](auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int r = 0; r < NM; r++) {
      double z = 0.0;
#pragma unroll
      for (int j = LO; j < NM; j++)
        if (j >= iq && j < n) z += Jreg[r][j] * dv[j];
      zv[r] = z;
    }
  };
  // r = R^{-1} d for the active set's inequality rows only (i >= p; LoC: a compile-time bound on
  // iq, here p).  In the active-set loop only those rows' r feed anything — t1 and the
  // inequalities' multipliers; the equality constraints' multipliers u[0..p) are never read there,
  // nor output — and r[i] for i >= p does not depend on the rows below, so the reference's
  // back-substitution stops at row p (x, f, status and the l1 passes are unchanged).
  auto update_r = [&](auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int i = NM - 1; i >= 0; i--) {
      if (i >= LO && i >= p && i < iq) {
        double s = 0.0;
#pragma unroll
        for (int j = i + 1; j < NM; j++)
          if (j < iq) s += Rv[RI::at(i, j)] * rv[j];
        rv[i] = ldiv<F>(dv[i] - s, Rv[RI::at(i, i)], fok);
      }
    }
  };
  // Fast build: the Givens step of add_constraint / delete_constraint without a branch.  The
  // pair (a, b) -> (+-h, 0) with h = |(a, b)| and the sign of a (the reference's cc < 0 test,
  // h > 0); the rows (t1, t2) -> (cc t1 + ss t2, ss t1 - cc t2), which is the reference's
  // xny (t1 + n1) - t2 with xny = ss / (1 + cc) and ss^2 + cc^2 = 1, without that division.  When
  // |h| < eps the reference skips the rotation: the coefficients become (1, 0 | 0, -1), the
  // identity, and (a, b) stay — so the step is straight-line code the scheduler can overlap with
  // the next rotation's h chain (which needs only +-h, not the coefficients).
  auto rot_fast = [&](double& a_, double& b_, auto&& apply) {
    const double a0 = a_, b0 = b_;
    const double h = ldistance<true>(a0, b0, fok);
    const bool skip = fabs(h) < kEps;
    const double rh = frcp(h);
    fok = fok && (skip || rcp_ok(rh));
    const bool neg = a0 < 0.0;
    const double cc = fabs(a0) * rh;
    const double ss = (neg ? -b0 : b0) * rh;
    a_ = skip ? a0 : (neg ? -h : h);
    b_ = skip ? b0 : 0.0;
    const double c1_ = skip ? 1.0 : cc, s1_ = skip ? 0.0 : ss;
    const double c2_ = skip ? -1.0 : cc, s2_ = skip ? 0.0 : ss;
    apply([&](double& t1r, double& t2r) {
      const double t1 = t1r, t2 = t2r;
      t1r = c1_ * t1 + s1_ * t2;
      t2r = s2_ * t1 - c2_ * t2;
    });
  };
  // LoC: a compile-time lower bound on iq (std::integral_constant).  In the active-set loop
  // iq >= p always (equality constraints are never dropped), so entries below p of R, A, u and
  // d are never the ones written or selected there: with p a compile-time constant (PX) the
  // predicated updates of those entries disappear.
  auto add_constraint = [&](auto LoC) -> bool {
    constexpr int LO = decltype(LoC)::value;
    if (iq >= n) return false;  // reference UB (p > n); reported as dependent
#pragma unroll
    for (int j = NM - 1; j >= LO + 1; j--) {
      if (j <= n - 1 && j >= iq + 1) {
        if constexpr (F) {
          rot_fast(dv[j - 1], dv[j], [&](auto&& rot) {
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < n) rot(Jreg[k][j - 1], Jreg[k][j]);
          });
          continue;
        }
        double cc = dv[j - 1], ss = dv[j];
        const double h = ldistance<F>(cc, ss, fok);
        if (!(fabs(h) < kEps)) {
          dv[j] = 0.0;
          const double rh = F ? frcp(h) : 0.0;
          ss = ldiv_r<F>(ss, h, rh, fok);
          cc = ldiv_r<F>(cc, h, rh, fok);
          if (cc < 0.0) {
            cc = -cc;
            ss = -ss;
            dv[j - 1] = -h;
          } else {
            dv[j - 1] = h;
          }
          const double xny = ldiv<F>(ss, 1.0 + cc, fok);
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k < n) {
              const double t1 = Jreg[k][j - 1], t2 = Jreg[k][j];
              const double n1 = t1 * cc + t2 * ss;
              Jreg[k][j - 1] = n1;
              Jreg[k][j] = xny * (t1 + n1) - t2;
            }
        }
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
    // shift R columns left from qq (only upper + subdiagonal entries exist)
#pragma unroll
    for (int c = LO; c < NM - 1; c++) {
      const bool sh = (c >= qq && c < iq - 1);
#pragma unroll
      for (int r = 0; r <= c + 1 && r < NM; r++) {
        // destination R[r][c] (upper or subdiagonal), source R[r][c+1] (upper)
        Rv[RI::at(r, c)] = sh ? Rv[RI::at(r, c + 1)] : Rv[RI::at(r, c)];
      }
    }
    {
      const int aiq = lsel_lo<LO>(Av, iq);
      const double uiq = lsel_lo<LO>(uv, iq);
      lput_lo<LO>(Av, iq - 1, aiq);
      lput_lo<LO>(uv, iq - 1, uiq);
      lput_lo<LO>(Av, iq, 0);
      lput_lo<LO>(uv, iq, 0.0);
    }
    // R[j][iq-1] = 0 for j < iq
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
        if constexpr (F) {
          rot_fast(Rv[RI::at(j, j)], Rv[RI::at(j + 1, j)], [&](auto&& rot) {
#pragma unroll
            for (int k = j + 1; k < NM; k++)
              if (k < iq) rot(Rv[RI::at(j, k)], Rv[RI::at(j + 1, k)]);
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < n) rot(Jreg[k][j], Jreg[k][j + 1]);
          });
          continue;
        }
        double cc = Rv[RI::at(j, j)], ss = Rv[RI::at(j + 1, j)];
        const double h = ldistance<F>(cc, ss, fok);
        if (!(fabs(h) < kEps)) {
          const double rh = F ? frcp(h) : 0.0;
          cc = ldiv_r<F>(cc, h, rh, fok);
          ss = ldiv_r<F>(ss, h, rh, fok);
          Rv[RI::at(j + 1, j)] = 0.0;
          if (cc < 0.0) {
            Rv[RI::at(j, j)] = -h;
            cc = -cc;
            ss = -ss;
          } else {
            Rv[RI::at(j, j)] = h;
          }
          const double xny = ldiv<F>(ss, 1.0 + cc, fok);
#pragma unroll
          for (int k = j + 1; k < NM; k++)
            if (k < iq) {
              const double t1 = Rv[RI::at(j, k)], t2 = Rv[RI::at(j + 1, k)];
              const double r1 = t1 * cc + t2 * ss;
              Rv[RI::at(j, k)] = r1;
              Rv[RI::at(j + 1, k)] = xny * (t1 + r1) - t2;
            }
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k < n) {
              const double t1 = Jreg[k][j], t2 = Jreg[k][j + 1];
              const double n1 = t1 * cc + t2 * ss;
              Jreg[k][j] = n1;
              Jreg[k][j + 1] = xny * (n1 + t1) - t2;
            }
        }
      }
    }
  };
  auto dot = [&](const double(&u_)[NM], const double(&v_)[NM]) -> double {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) s += u_[i] * v_[i];
    return s;
  };
  const auto kZero = std::integral_constant<int, 0>{};

  // ---------------------------------------------------------------- equality phase
  // Fully unrolled: in step i the active-set size iq equals i (every earlier step added a
  // constraint, or the phase stopped), so pinning iq to the compile-time i folds every
  // iq-predicate of compute_d / update_z / update_r / add_constraint.
  bool done = !ok_lane;
#pragma unroll
  for (int i = 0; i <= NM; i++) {
    if constexpr (kCiDma && PX > 0) {
      if (ce_agpr && i < PX) dma_ci_part(i, PX);  // every lane (the copy is per wave)
      if constexpr (QPGPU_LANE_WARMUP == 2) {
        if (ce_agpr && i == PX - 1) warmup();
      }
    }
    if (i < p && !done) {
      iq = i;
      double c0;
      if (i < NM) {
        const int np_ = n * p;
        const int offc = (kQpw * np_ + 127) / 128 * 128;
#pragma unroll
        for (int j = 0; j < NM; j++) {
          if constexpr (kCiDma && PX > 0) {
            if (ce_agpr) {
              // (idle lanes' ceag already holds zeros)
              npv[j] = j < n ? from_agpr(ceag[(j * PX + i) < kCeN ? j * PX + i : 0]) : 0.0;
              continue;
            }
          }
          if (ce_staged) {  // unconditional LDS read, then the select (see the G reads)
            const double v = j < n ? rd_all(0, np_, j * p + i) : 0.0;
            npv[j] = live ? v : 0.0;
          } else {
            npv[j] = (live && j < n) ? view(const_cast<double*>(a.CE), np_)[(j * p + i) * T] : 0.0;
          }
        }
        bool c0_done = false;
        if constexpr (kCiDma && PX > 0) {
          if (ce_agpr) {
            c0 = from_agpr(ceag[NM * PX + i < kCeN ? NM * PX + i : 0]);
            c0_done = true;
          }
        }
        if (!c0_done) {
          if (ce_staged) {
            const double v = rd_all(offc, p, i);
            c0 = live ? v : 0.0;
          } else {
            c0 = live ? view(const_cast<double*>(a.ce0), p)[i * T] : 0.0;
          }
        }
      } else {  // p > n: the step that reports "dependent" (reference UB, see oracle)
        const double* CEb = view(const_cast<double*>(a.CE), n * p);
#pragma unroll
        for (int j = 0; j < NM; j++) npv[j] = (j < n) ? CEb[(j * p + i) * T] : 0.0;
        c0 = view(const_cast<double*>(a.ce0), p)[i * T];
      }
      compute_d();
      update_z(kZero);
      // (no update_r and no u[:i] update here: r and the equality constraints' multipliers u[0..p)
      // feed nothing — the active-set loop reads u only for the inequalities (t1, the dual step's
      // drop, the rollback) and x, f never use u — so the reference's back-substitution of every
      // equality step is skipped; x, f, status and the l1 passes are unchanged)
      double t2 = 0.0;
      const double zz = dot(zv, zv);
      const double znp = dot(zv, npv);
      if (fabs(zz) > kEps) t2 = ldiv<F>(-dot(npv, xv) - c0, znp, fok);
#pragma unroll
      for (int k = 0; k < NM; k++) xv[k] += t2 * zv[k];
      uv[i < NM + 1 ? i : NM] = t2;
      fval += 0.5 * (t2 * t2) * znp;
      Av[i < NM + 1 ? i : NM] = -i - 1;
      if (!add_constraint(kZero)) {
        status = QPGPU_QP_DEPENDENT;
        done = true;
      }
    }
  }
  // the m = 0 answer (qpgpu_solve_batched_eq): an empty l1 scan returns right here.  Only the
  // generic instantiations carry it; the launcher routes snapshot calls there so the EXACT
  // fast paths keep their register budget.
  if (!EXACT && a.x_eq && live) {
    if (chol_ok) {
      double* xb = view(a.x_eq, n);
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) xb[i * T] = xv[i];
    }
    a.f_eq[b] = fval;
    a.st_eq[b] = status;
  }
  if constexpr (T == 1 && (kLanePrefetch || kCiDma)) {
    if (live && warmed)  // the warm-up loads retire here, long after they landed
#pragma unroll
      for (int k = 0; k < kPfCI + kPfC0; k++) asm volatile("" ::"v"(pf[k]));
  }
  // CI rows 0..kCiRows-1 are kept in LDS for the loop: brought in by the DMA above, or written
  // by the first l1 scan (which every active lane runs, loading those rows into registers
  // anyway).  Later scans then issue only the remaining rows' global loads, and the
  // selected-column gather takes those rows from LDS — no extra global traffic.
  const bool ci_lds = kCiRows > 0 && (a.flags & kArgAligned16);
  bool ci_ready = false;  // wave-uniform: the on-chip copy has been written (or has landed)
  if constexpr (kCiDma) {
    if (dma && (PX == 0 || ce_agpr)) {
      __syncthreads();  // the DMA has landed
      ci_ready = true;
    }
  }
  // element e (= row * MM + column) of this lane's CI from the LDS copy (e < kCiRows * MM)
  auto ci_lds_at = [&](int e) -> double { return sbuf[((e >> 1) * kQpw + lane) * 2 + (e & 1)]; };
  lstamp(a, 2);
  // Fast build: a fast form that went out of range in the setup or the equality phase (or
  // non-finite data) sends the wave to the IEEE re-solve now, instead of after a loop that
  // would run on garbage up to the step cap.  (The CE / CI copies into LDS have landed: the
  // re-solve may restage.)  The loop checks again at the top of every pass
  // (QPGPU_LANE_LOOPTOP_EXIT) and after the last one.
  if constexpr (F) {
    if (wave_any(!fok)) return false;
  }

  // ---------------------------------------------------------------- active-set loop
  // Wave-uniform loop: every lane stays until all 64 are done; per-lane work is predicated on
  // `active`.  Every active lane has iq >= p here (the equality phase completed, only
  // inequalities are ever dropped), so with p known at compile time the loop's iq-indexed
  // updates start at p.
  constexpr int IQLO = PX >= 0 ? (PX <= NM ? PX : NM) : 0;
  const auto kLo = std::integral_constant<int, IQLO>{};
  {
    double sv[MM];
#pragma unroll
    for (int i = 0; i < MM; i++) sv[i] = 0.0;
    // rollback copies (compile-time indices only)
    double xold[NM], uold[NM];
    int aold[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) {
      xold[i] = uold[i] = 0.0;
      aold[i] = 0;
    }
    uint64_t act = 0;   // bit c set <=> iai[c] == -1
    uint64_t excl = 0;  // bit c set <=> iaexcl[c] == false
    int ip = 0, steps = 0;
    double ss = 0.0, ci0ip = 0.0;
    bool need_scan = true, need_select = true;
    bool active = !done;
    const int max_steps = a.max_steps;
    const double* CIg = view(const_cast<double*>(a.CI), n * m);
    const double* ci0g = view(const_cast<double*>(a.ci0), m);
    // element loaders for this lane's CI / ci0 block.  TILED64: raw buffer loads off a
    // wave-uniform descriptor (tile base) + one lane-offset VGPR + element offset in SGPR/imm,
    // so no 64-bit address per element is kept live.
    // descriptor inputs through readfirstlane so the compiler can PROVE them uniform (else
    // it wraps every buffer op in a waterfall loop: guide T20)
    auto uniform_ptr = [](const double* ptr) -> double* {
      const uint64_t v = reinterpret_cast<uint64_t>(ptr);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
      return reinterpret_cast<double*>(((uint64_t)hi << 32) | lo);
    };
    [[maybe_unused]] const auto rsCI = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr(a.CI + b0 * (int64_t)(n * m)), 0,
        __builtin_amdgcn_readfirstlane(64 * n * m * 8), 0x00020000);
    [[maybe_unused]] const auto rsci0 = __builtin_amdgcn_make_buffer_rsrc(
        uniform_ptr(a.ci0 + b0 * (int64_t)m), 0, __builtin_amdgcn_readfirstlane(64 * m * 8),
        0x00020000);
    auto ldCI = [&](int e) -> double {
      if constexpr (T == 64)
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsCI, lane * 8, e * 512, 0));
      else
        return CIg[e];
    };
    auto ldci0 = [&](int e) -> double {
      if constexpr (T == 64)
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsci0, lane * 8, e * 512, 0));
      else
        return ci0g[e];
    };
    // elements i, i+1 of row r (< kCiRows) of the LDS copy
    auto lds_pair = [&](int r, int i) -> double2 {
      return *reinterpret_cast<const double2*>(sbuf + (((r * MM + i) >> 1) * kQpw + lane) * 2);
    };
    // one l1 pass (the first fills the LDS copy when the DMA did not)
    auto scan_pass = [&]() {
        // ---- l1: s = CI^T x + ci0 (each s[i] sums j ascending, then + ci0[i])
        const bool do_scan = active && need_scan;
        if (wave_any(do_scan)) {
          double psi = 0.0;
          if (do_scan) {
            iter++;
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k >= p && k < iq) act |= 1ull << Av[k];
#pragma unroll
            for (int i = 0; i < MM; i++) sv[i] = 0.0;
          }
          if (do_scan) {
            // QP-major rows of an EXACT even-m shape are 16-B aligned when the arrays are
            // (checked on the host: kArgAligned16): load them as dwordx4, half the instructions
            // and half the cache-line lookups per row
            constexpr bool VEC = (T == 1) && EXACT && (MM % 2 == 0);
            const bool vec = VEC && (a.flags & kArgAligned16);
            auto ldrow = [&](double* dst, const double* src) {
              if (VEC && vec) {
#pragma unroll
                for (int i = 0; i < MM; i += 2) {
                  const double2 v = *reinterpret_cast<const double2*>(src + i);
                  dst[i] = v.x;
                  dst[i + 1] = v.y;
                }
              } else {
#pragma unroll
                for (int i = 0; i < MM; i++) dst[i] = (i < m) ? src[i] : 0.0;
              }
            };
            const bool from_chip = ci_lds && ci_ready;
            // "rows" 0..NM-1 are CI's rows (those >= n are never read), row NM is ci0
            auto load_row = [&](int r, double* dst) {
              if (r < NM) {
                if (r < n) {
                  if constexpr (T == 1)
                    ldrow(dst, CIg + r * m);
                  else
#pragma unroll
                    for (int i = 0; i < MM; i++) dst[i] = (i < m) ? ldCI(r * m + i) : 0.0;
                }
              } else if (r == NM) {
                if constexpr (T == 1)
                  ldrow(dst, ci0g);
                else
#pragma unroll
                  for (int i = 0; i < MM; i++) dst[i] = (i < m) ? ldci0(i) : 0.0;
              }
            };
            if (kCiRows > 0 && from_chip) {
              // the LDS rows summed while every global row (the rest of CI, ci0) is in
              // flight (same j order)
              constexpr int NG = NM + 1 - kCiRows;
              double gbuf[NG][MM];
#pragma unroll
              for (int r = kCiRows; r <= NM; r++) load_row(r, gbuf[r - kCiRows]);
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int j = 0; j < NM; j++) {
                if (j < n) {
                  const double xj = xv[j];
                  if (j < kCiRows) {
#pragma unroll
                    for (int i = 0; i < MM; i += 2) {
                      const double2 v = lds_pair(j, i);
                      if (i < m) sv[i] += v.x * xj;
                      if (i + 1 < m) sv[i + 1] += v.y * xj;
                    }
                  } else {
                    const int g = j - kCiRows < NG ? j - kCiRows : 0;
#pragma unroll
                    for (int i = 0; i < MM; i++)
                      if (i < m) sv[i] += gbuf[g][i] * xj;
                  }
                }
              }
#pragma unroll
              for (int i = 0; i < MM; i++)
                if (i < m) {
                  sv[i] += gbuf[NG - 1][i];
                  psi += (sv[i] < 0.0) ? sv[i] : 0.0;
                }
            } else {
              // the first scan without the DMA (and every scan of the shapes without an
              // on-chip copy): software-pipelined two rows deep; row r lands in rowbuf[r % D]
              const bool fill = ci_lds && !ci_ready;
              constexpr int D = kScanDepth;
              double rowbuf[D][MM];
#pragma unroll
              for (int r = 0; r < D - 1; r++) load_row(r, rowbuf[r % D]);
#pragma unroll
              for (int j = 0; j < NM; j++) {
                load_row(j + D - 1, rowbuf[(j + D - 1) % D]);
                __builtin_amdgcn_sched_barrier(0);
                if (j < n) {
                  const double xj = xv[j];
#pragma unroll
                  for (int i = 0; i < MM; i++)
                    if (i < m) sv[i] += rowbuf[j % D][i] * xj;
                  if (j < kCiRows && fill) {
#pragma unroll
                    for (int i = 0; i < MM; i += 2)
                      *reinterpret_cast<double2*>(sbuf + (((j * MM + i) >> 1) * kQpw + lane) * 2) =
                          double2{rowbuf[j % D][i], rowbuf[j % D][i + 1]};
                  }
                }
                __builtin_amdgcn_sched_barrier(0);
              }
#pragma unroll
              for (int i = 0; i < MM; i++)
                if (i < m) {
                  sv[i] += rowbuf[NM % D][i];
                  psi += (sv[i] < 0.0) ? sv[i] : 0.0;
                }
            }
          }
          ci_ready = ci_ready || ci_lds;
          if (do_scan) {
            excl = 0;
            ss = 0.0;
            ip = 0;
            if (fabs(psi) <= (double)m * kEps * c1 * c2 * 100.0) {
              active = false;  // optimal
            } else {
#pragma unroll
              for (int i = 0; i < NM; i++) {
                if (i < IQLO || i < iq) {
                  uold[i] = uv[i];
                  aold[i] = Av[i];
                }
                xold[i] = xv[i];
              }
            }
          }
        }
    };
    uint64_t tscan = 0, tsel = 0, nloop = 0, tfirst = 0;  // diagnostic stamps only
    [[maybe_unused]] uint64_t tdzr = 0, tstep = 0;        // (QPGPU_LANE_STAMPS == 2: l2a split)
    while (wave_any(active)) {
      if constexpr (F && QPGPU_LANE_LOOPTOP_EXIT == 1) {
        if (wave_any(!fok)) return false;
      }
      if constexpr (F && QPGPU_LANE_LOOPTOP_EXIT == 2) {
        if (wave_any(!fok) && a.max_steps < -1) return false;
      }
      const uint64_t tl0 = (kStamps && a.stamps) ? __builtin_amdgcn_s_memtime() : 0;
      scan_pass();
      const uint64_t tl1 = (kStamps && a.stamps) ? __builtin_amdgcn_s_memtime() : 0;
      if (kStamps && a.stamps) {
        tscan += tl1 - tl0;
        if (nloop == 0) tfirst = tl1 - tl0;
      }
      nloop++;
      // ---- l2: pick the most violated constraint (ss deliberately not reset: reference quirk)
      if (active && need_select) {
#pragma unroll
        for (int i = 0; i < MM; i++)
          if (i < m) {
            const bool elig = !((act >> i) & 1ull) && !((excl >> i) & 1ull);
            const bool take = sv[i] < ss && elig;
            ss = take ? sv[i] : ss;
            ip = take ? i : ip;
          }
        if (ss >= 0.0) {
          active = false;  // optimal
        } else {
#pragma unroll
          for (int j = 0; j < NM; j++)
            npv[j] = (j < n) ? ((j < kCiRows && ci_ready) ? ci_lds_at(j * MM + ip) : ldCI(j * m + ip)) : 0.0;
          ci0ip = ldci0(ip);
          lput_lo<IQLO>(uv, iq, 0.0);
          lput_lo<IQLO>(Av, iq, ip);
        }
      }
      if (kStamps && a.stamps) {
        // make the select's loads part of the select span
        const double sink = npv[0] + ci0ip;
        asm volatile("" ::"v"(sink));
        const uint64_t tl2 = __builtin_amdgcn_s_memtime();
        tsel += tl2 - tl1;
      }
      // ---- l2a
      if (active) {
        if (max_steps > 0 && ++steps > max_steps) {
          status = QPGPU_QP_MAX_ITER;
          active = false;
        } else {
          [[maybe_unused]] uint64_t ts0 = 0;
          if constexpr (QPGPU_LANE_STAMPS == 2) ts0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
          compute_d();
          update_z(kLo);
          update_r(kLo);
          if constexpr (QPGPU_LANE_STAMPS == 2) {
            if (a.stamps) {
              const double sink = rv[0] + zv[0] + dv[NM - 1];
              asm volatile("" ::"v"(sink));
              tdzr += __builtin_amdgcn_s_memtime() - ts0;
            }
          }
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
          const double zz = dot(zv, zv);
          const double znp = dot(zv, npv);
          double t2;
          if (fabs(zz) > kEps) {
            t2 = ldiv<F>(-lsel<MM>(sv, ip), znp, fok);
            if (t2 < 0) t2 = inf;  // Takano Akio patch
          } else {
            t2 = inf;
          }
          const double t = (t2 < t1) ? t2 : t1;
          // The step's four outcomes (infeasible, dual step, full step, partial step) as per-lane
          // predicates over ONE copy of each piece: a wave whose lanes take different outcomes
          // executes the union of the pieces, and delete_constraint — which the dual step
          // (drops l), the degenerate full step (drops ip) and the partial step (drops l) all
          // need — is the largest of them.  Each lane runs exactly its outcome's operations in
          // the reference's order (x, f, then u; add_constraint; then the delete; then the
          // rollback or the s[ip] refresh).
          const bool infs = t >= inf;
          const bool dual = !infs && t2 >= inf;
          const bool prim = !infs && !dual;
          const bool full = prim && fabs(t - t2) < kEps;
          const bool part = prim && !full;
          if (infs) {
            status = QPGPU_QP_INFEASIBLE;
            fval = inf;
            active = false;
          }
          if (prim) {
#pragma unroll
            for (int k = 0; k < NM; k++) xv[k] += t * zv[k];
            fval += t * znp * (0.5 * t + lsel_lo<IQLO>(uv, iq));
          }
          if (dual || prim) {
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k >= p && k < iq) uv[k] -= t * rv[k];  // (u[0..p) are never read)
            lput_lo<IQLO>(uv, iq, lsel_lo<IQLO>(uv, iq) + t);
          }
          bool add_fail = false;
          if (full) {
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
            for (int i = 0; i < NM; i++) xv[i] = xold[i];
            need_scan = false;
            need_select = true;
          }
          if (part) {  // refresh s[ip] = CI[:,ip]^T x + ci0[ip]
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < NM; j++)
              if (j < n) s += npv[j] * xv[j];
            lput_lo<0>(sv, ip, s + ci0ip);
          }
          if (dual || part) need_scan = need_select = false;
        }
      }
    }
    if (kStamps && a.stamps && lane == 0) {
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 5] = tscan;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 6] = tsel;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 7] = nloop;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 8] = tfirst;
      if constexpr (QPGPU_LANE_STAMPS == 2) a.stamps[(uint64_t)blockIdx.x * kStampSlots + 12] = tdzr;
    }
  }
  lstamp(a, 3);
  if constexpr (F) {
    if (wave_any(!fok)) return false;
  }

  if (live) {
    if (chol_ok) {
      double* xb = view(a.x, n);
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) xb[i * T] = xv[i];
    }
    a.f[b] = fval;
    if (a.iters) a.iters[b] = iter;
    a.status[b] = status;
  }
  lstamp(a, 4);
  return true;
}

template <int NM, int MM, int T, bool EXACT, int PX>
__global__ void __launch_bounds__(64, kLaneOcc) QP_LANE_KERNEL(const QpArgs a) {
  __shared__ double sbuf[kStage];
  if constexpr (kFast) {
    if (!lane_body<NM, MM, T, EXACT, PX, false>(a, sbuf)) {
      __syncthreads();  // the fast attempt's LDS traffic is over
      lane_body<NM, MM, T, EXACT, PX, true>(a, sbuf);
    }
  } else {
    lane_body<NM, MM, T, EXACT, PX, true>(a, sbuf);
  }
}

// The exact build's p = 0 instantiations (C2, the joint-limit QPs) are compiled in their own
// translation unit (qp_lane_p0.hip, QPGPU_LANE_PART = 2) under LLVM's iterative-minreg scheduler,
// the rest (QPGPU_LANE_PART = 1) under iterative-ilp: measured C2 71.2-71.9 -> 68.6-69.1 us with
// minreg, while C1 is slower with it (43.7-44.7 -> 46.1-47.9 us; profiles/r05_s11).  Part 0 (the
// fast build, A/B builds) keeps every instantiation in one TU.
#ifndef QPGPU_LANE_PART
#define QPGPU_LANE_PART 0
#endif
template <int NM, int MM, int T>
static hipError_t launch_lane_p0(const QpArgs& a, hipStream_t stream);
template <int NM, int MM, int T>
static hipError_t launch_lane_t(const QpArgs& a, hipStream_t stream) {
  const int64_t blocks = (a.batch + kQpw - 1) / kQpw;
  const dim3 g((unsigned)blocks), blk(64);
// A/B builds with one instantiation only refuse every other launch with an error: a launch
// they skipped silently once returned the previous call's f / status / passes through the host
// entry's reused device buffers, with x = 0 (profiles/r05_s26)
#ifdef QPGPU_LANE_AB_C1ONLY
  // A/B experiment builds (tools/ab_build.sh): only the C1 instantiation, for a quick compile
  if constexpr (NM == 7 && MM == 14 && T == 1)
    if (a.n == NM && a.m == MM && !a.x_eq && a.p == 6) {
      hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, true, 6>), g, blk, 0, stream, a);
      return hipSuccess;
    }
  return hipErrorInvalidValue;
#endif
#ifdef QPGPU_LANE_AB_N8P0ONLY
  // A/B / ISA-study builds: only the QP-major (8, 0, 16) instantiation
  if constexpr (NM == 8 && MM == 16 && T == 1)
    if (a.n == NM && a.m == MM && !a.x_eq && a.p == 0) {
      hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, true, 0>), g, blk, 0, stream, a);
      return hipSuccess;
    }
  return hipErrorInvalidValue;
#endif
  if (a.n == NM && a.m == MM && !a.x_eq) {
    if (a.p == 6)
      hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, true, 6>), g, blk, 0, stream, a);
    else if (a.p == 0)
      return launch_lane_p0<NM, MM, T>(a, stream);
    else
      hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, true, -1>), g, blk, 0, stream, a);
  } else {
    hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, false, -1>), g, blk, 0, stream, a);
  }
  return hipSuccess;
}

#if QPGPU_LANE_PART == 1
}  // namespace QPK_LANE_NS
extern "C" hipError_t qpk_launch_lane_p0(const qpk::QpArgs* a, hipStream_t stream);  // qp_lane_p0.hip
namespace QPK_LANE_NS {
template <int NM, int MM, int T>
static hipError_t launch_lane_p0(const QpArgs& a, hipStream_t stream) {
  return qpk_launch_lane_p0(&a, stream);
}
#else
template <int NM, int MM, int T>
static hipError_t launch_lane_p0(const QpArgs& a, hipStream_t stream) {
  const int64_t blocks = (a.batch + kQpw - 1) / kQpw;
  hipLaunchKernelGGL((QP_LANE_KERNEL<NM, MM, T, true, 0>), dim3((unsigned)blocks), dim3(64), 0, stream, a);
  return hipSuccess;
}
#endif

#if QPGPU_LANE_PART != 2
template <int NM, int MM>
static hipError_t launch_lane(const QpArgs& a, hipStream_t stream) {
  const hipError_t e = a.tile == 64 ? launch_lane_t<NM, MM, 64>(a, stream) : launch_lane_t<NM, MM, 1>(a, stream);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

struct LaneVariant {
  int nmax, mmax;
  const char* name;
  hipError_t (*launch)(const QpArgs&, hipStream_t);
};

static const LaneVariant kLaneVariants[] = {
    {7, 14, kFast ? "qp_lane_fast<N=7,M=14>" : "qp_lane<N=7,M=14>", launch_lane<7, 14>},
    {8, 16, kFast ? "qp_lane_fast<N=8,M=16>" : "qp_lane<N=8,M=16>", launch_lane<8, 16>},
};

const LaneVariant* pick_lane(int n, int m) {
  for (const auto& v : kLaneVariants)
    if (n <= v.nmax && m <= v.mmax) return &v;
  return nullptr;
}
#endif  // QPGPU_LANE_PART != 2

}  // namespace QPK_LANE_NS

#if QPGPU_LANE_PART == 2
// part 2: the exact p = 0 kernels only (the caller, part 1's launch_lane_t, has matched the
// shape).  A shape part 1 forwards that this list lacks (a LaneVariant added to kLaneVariants
// without an entry here) is an error, never a silent success with nothing written.
extern "C" hipError_t qpk_launch_lane_p0(const qpk::QpArgs* a, hipStream_t stream) {
  using namespace QPK_LANE_NS;
  if (a->n == 7 && a->m == 14)
    return a->tile == 64 ? launch_lane_p0<7, 14, 64>(*a, stream) : launch_lane_p0<7, 14, 1>(*a, stream);
  if (a->n == 8 && a->m == 16)
    return a->tile == 64 ? launch_lane_p0<8, 16, 64>(*a, stream) : launch_lane_p0<8, 16, 1>(*a, stream);
  return hipErrorInvalidValue;
}
#else
extern "C" hipError_t QPK_LANE_C(qpk_launch_lane)(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                                  const char** name) {
  const QPK_LANE_NS::LaneVariant* v = QPK_LANE_NS::pick_lane(a->n, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  return v->launch(*a, stream);
}

extern "C" const char* QPK_LANE_C(qpk_lane_name)(int n, int /*p*/, int m) {
  const QPK_LANE_NS::LaneVariant* v = QPK_LANE_NS::pick_lane(n, m);
  return v ? v->name : nullptr;
}
#endif  // QPGPU_LANE_PART == 2
