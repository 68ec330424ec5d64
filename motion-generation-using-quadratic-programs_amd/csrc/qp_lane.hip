// qp_lane.hip — gfx950 batched Goldfarb–Idnani solver, ONE QP PER LANE (n <= 8, m <= 16).
//
// Restates solve_quadprog() (reference include/QuadProgpp/QuadProg++.hh:69-72; operation order
// of the prebuilt libquadprog.a fixed in SURVEY.md §3.2) for the 64 QPs of one wavefront.
//
// Why one QP per lane: at these sizes the cost is the serial chain of every QP (Givens
// coefficients = 4 IEEE divisions + 1 sqrt each, back-substitutions, step lengths); running it
// once per QP instead of once per lane of a subgroup cuts issued instructions ~4x versus
// qp_small.hip.  State placement (gfx950: 512 VGPR+AGPR per lane at 1 wave/SIMD, 160 KiB LDS
// per CU = 40 KiB per wave at 4 waves/CU):
//   * J (= L^{-T}), R (upper triangle + first subdiagonal, the only entries the algorithm makes
//     non-zero), x, z, d, np, u, r, A, s live in registers, indexed only with compile-time
//     indices (fully unrolled loops with run-time predicates);
//   * every input block is brought in by COOPERATIVE, coalesced wave loads of the wave's 64
//     contiguous QP blocks into a 40 KiB LDS staging buffer, then read per lane from LDS
//     (QP-major: lane t at [t*(c|1) + k], odd stride = conflict-free ds_read_b64; TILED64:
//     [k*64 + t]).  The l1 scan re-stages CI in row chunks each time any lane of the wave
//     scans, so the main loop is wave-uniform (lanes that are done ride along predicated).
// IEEE binary64 throughout, no contraction: results are bitwise identical to the CPU
// restatement (oracle/qp_oracle.c), which tests/ check.
#include <cstdlib>
#include <type_traits>

#include "qp_common.h"

namespace qpk {

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
template <int N, typename T>
__device__ __forceinline__ void lput(T (&v)[N], int i, T x) {
  lput_lo<0>(v, i, x);
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

constexpr int kStage = 5120;  // staging buffer, doubles (40 KiB: 4 waves per CU)
// rows of the l1 scan in flight per lane (software pipeline depth; CI rows + the ci0 row)
#ifndef QPGPU_SCAN_DEPTH
#define QPGPU_SCAN_DEPTH 2
#endif
constexpr int kScanDepth = QPGPU_SCAN_DEPTH;
#ifndef QPGPU_LANE_JREG_LOOP
#define QPGPU_LANE_JREG_LOOP 2
#endif
// where the active-set loop keeps the rollback copies x_old / u_old / A_old: 0 LDS, 1 registers
// when p > 0 (LDS for p = 0, whose loop already holds J and the Givens state in registers),
// 2 registers always.  Measured: 2 vs 0 on C1 58.4 -> 49.4 us (lane_rollback_regs.log); 1 vs
// 2 on C2 within noise (c2_rollback_lds_*.log, 170 vs 239 AGPRs), so 2 serves both
#ifndef QPGPU_LANE_RB_REGS
#define QPGPU_LANE_RB_REGS 2
#endif
// rows of CI each lane keeps in LDS for the l1 scans (0 disables; see the LDS regions)
#ifndef QPGPU_LANE_CI_LDS
#define QPGPU_LANE_CI_LDS 1
#endif
// warm the caches with this lane's CI / ci0 lines before the equality phase (QP-major layout):
// 0 never, 1 always, 2 when p > 0 (an equality phase long enough for the loads to land).
// Measured on cold inputs (profiles/r02_s2/bench_C{1,2}_{base,pf}.log): C1 (p = 6) kernel
// 55.4 -> 52.6 us and +3 % pipelined; C2 (p = 0, no equality phase) 78.1 -> 80.5 us.  Round 1
// measured it on one warm input set (lane_ci_warmup.log), where it lost ~4 % pipelined.
#ifndef QPGPU_LANE_PREFETCH
#define QPGPU_LANE_PREFETCH 2
#endif
// keep the CI rows that do not fit the LDS (and ci0) in registers from the first l1 scan on, so
// later scans issue no global loads (EXACT QP-major shapes with the LDS rows only): 0 never,
// 1 always, 2 when p > 0 (the p = 0 loop holds J and the Givens state in registers already: with
// the rows too it spills to scratch)
#ifndef QPGPU_LANE_CI_REGS
#define QPGPU_LANE_CI_REGS 0
#endif
// add_constraint's Givens sweep: feed distance() the carried |h| of the previous rotation (or
// the untouched d[j]) instead of the rotated d[j] = +-h, so the chain of h values does not wait
// for the cc = d/h division and sign select (distance() reads magnitudes only: same bits).
// Measured neutral on C1 (equality phase 26.4k cycles/wave either way, profiles/r02_s4): off.
#ifndef QPGPU_LANE_HCHAIN
#define QPGPU_LANE_HCHAIN 0
#endif
// add_constraint's Givens rotations branch-free (both outcomes selected) with the |h| chain
// carried, so consecutive rotations could overlap.  Measured (profiles/r02_s50): C1 kernel
// 51.7 vs 51.9 us, equality phase 24.8k -> 25.8k cycles per wave: off
#ifndef QPGPU_LANE_ADDBF
#define QPGPU_LANE_ADDBF 0
#endif
// p = 0: issue the CI / ci0 cache warm-up as soon as G has landed (before the Cholesky) and
// retire its registers after the active-set loop, whose first scan waits for it anyway.
// Measured on C2 (profiles/r02_s46): kernel 75.1 -> 82.0 us (3-stream steps 54.4 -> 52.9 us):
// off
#ifndef QPGPU_LANE_PF_P0
#define QPGPU_LANE_PF_P0 0
#endif
// issue the CI / ci0 cache warm-up right after the G / CE staging instead of after the setup.
// Measured slower (C1 kernel 54.0 -> 56.5 us, setup 21.7k -> 33.4k cycles/wave: vmcnt waits are
// in issue order, so the G / CE waits then cover the warm-up loads too): off.
#ifndef QPGPU_LANE_PF_EARLY
#define QPGPU_LANE_PF_EARLY 0
#endif
// l1 scans after the first (CI rows 0..kCiRows-1 in LDS): issue every global row (the rest of
// CI and ci0) at the start of the scan, then sum the LDS rows while they are in flight.
// Measured (profiles/r02_s4): C1 kernel 54.0 -> 51.7 us on cold inputs, scan 18.9k -> 16.6k
// cycles/wave, bitwise parity unchanged.
#ifndef QPGPU_LANE_SCANG
#define QPGPU_LANE_SCANG 1
#endif
// cache policy of the once-read LDS-DMA staging (G, g0, CE, ce0): 0 default, 2 non-temporal (so
// the stream does not evict the CI lines the later l1 scans re-read from L2)
#ifndef QPGPU_LANE_STAGE_NT
#define QPGPU_LANE_STAGE_NT 0
#endif
constexpr int kStageAux = QPGPU_LANE_STAGE_NT ? 2 : 0;
static_assert(kScanDepth >= 2, "the pipelined scan needs at least two row buffers");

__device__ __forceinline__ bool wave_any(bool v) { return __builtin_amdgcn_ballot_w64(v) != 0; }

// QPW = QPs per wavefront (64, or 32 to run two waves per SIMD with half the lanes each)
// PX >= 0: p is the compile-time constant PX as well (C1/C4: 6, C2: 0), which folds every
// [p, iq) loop of the active-set phase (for n = 7, p = 6 that range holds at most one entry).
template <int NM, int MM, int T, bool EXACT, int QPW, int PX>
__global__ void __launch_bounds__(64, QPW == 64 ? 1 : 2) qp_lane_kernel(const QpArgs a) {
  constexpr bool kJregLoopCfg = QPGPU_LANE_JREG_LOOP == 2 || (QPGPU_LANE_JREG_LOOP == 1 && PX == 0);
  constexpr bool kRbRegs = QPGPU_LANE_RB_REGS == 2 || (QPGPU_LANE_RB_REGS == 1 && PX != 0);
  constexpr bool kLanePrefetch = QPGPU_LANE_PREFETCH == 1 || (QPGPU_LANE_PREFETCH == 2 && PX > 0);
  // p = 0 (no equality phase): the warm-up right after G lands, retired after the loop
  constexpr bool kPfP0 = QPGPU_LANE_PF_P0 && PX == 0 && !kLanePrefetch;
  static_assert(QPW == 64 || (QPW == 32 && T == 1), "half waves only with the QP-major layout");
  static_assert(MM <= 64, "bitmask bookkeeping holds m <= 64");
  using RI = RIdx<NM>;
  // LDS per wave: J region + rollback region (40 KiB at NM = 7: 4 waves/CU)
  constexpr int STAGE_MIN = (QPW * NM * NM + 127) / 128 * 128 + QPW * (3 * NM + 2);
  constexpr int STAGE_CAP = kStage * QPW / 64;
  constexpr int STAGE = STAGE_MIN > STAGE_CAP ? STAGE_MIN : STAGE_CAP;
  __shared__ double sbuf[STAGE];

  const int lane = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * QPW;
  const int64_t b = b0 + lane;
  const int valid = (int)min<int64_t>(QPW, a.batch - b0);
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
  const bool full = (T == 64) || (valid == QPW);
  auto copy_span = [&](const double* src, int nd, int off) {  // nd even, full waves only
#pragma unroll 4
    for (int k = 0; k < nd; k += 128) {
      const int e = k + 2 * lane;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void*)(e < nd ? src + e : src),
          (__attribute__((address_space(3))) void*)(sbuf + off + k), 16, 0, kStageAux);
    }
  };
  // whole tile of X (E doubles per QP) -> sbuf[off...]
  auto stage_all = [&](const double* X, int E, int off) {
    if (full) {
      copy_span(X + b0 * (int64_t)E, QPW * E, off);
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
  // then — when J stays in registers — rows 0..kCiRows-1 of every lane's CI for the active-set
  // loop (16-B pieces, piece k of lane l at doubles (k*QPW + l)*2); otherwise it holds J's LDS
  // image (element (i,j) of lane l at (i*NM+j)*QPW + l).  RB, at the top, = g0 staging, then
  // (unless they live in registers, kRbRegs) the rollback copies x_old / u_old / A_old.
  constexpr int JA = (QPW * NM * NM + 127) / 128 * 128;
  constexpr int RBSZ = QPW * NM + (kRbRegs ? 0 : 2 * QPW * (NM + 1));
  constexpr int RB = (STAGE - RBSZ) / 2 * 2;
  constexpr int RB_U = RB + QPW * NM, RB_A = RB_U + QPW * (NM + 1);
  static_assert(RB >= JA && RB >= QPW * NM * NM, "LDS regions exceed the stage buffer");
  // CI rows held in LDS through the loop (EXACT QP-major shapes, J in registers)
  constexpr int kCiRowsFit = (RB / QPW) / MM;
  constexpr int kCiRows = (EXACT && T == 1 && kJregLoopCfg && MM % 2 == 0)
                              ? (kCiRowsFit < NM ? kCiRowsFit : NM) : 0;
#define Jr_(i, j) sbuf[((i) * NM + (j)) * QPW + lane]
  // J lives in registers (compile-time indices) through the J build and the equality phase,
  // where every step reads and rotates all of it; the loop then works on its LDS image.  CE
  // and ce0 stay in their LDS staging (read once per equality step) until then.
  double Jreg[NM][NM];
  bool ce_staged = false;
  // keep J in registers through the active-set loop too (QPGPU_LANE_JREG_LOOP: 0 never, 1 when
  // p = 0 — no equality phase, the loop does all the rotations — , 2 always)
  constexpr bool kJregLoop = kJregLoopCfg;
  // one dword per 128-B line of this lane's CI / ci0 blocks (cache warm-up, see below)
  constexpr int kPfCI = (NM * MM * 8 + 127) / 128 + 1, kPfC0 = (MM * 8 + 127) / 128 + 1;
  [[maybe_unused]] uint32_t pf[kPfCI + kPfC0];
  // Touch every cache line of this lane's CI and ci0 blocks before the equality phase: the
  // loads complete during it (nothing waits on them until its end), so the first l1 scan — all
  // lanes of every wave at about the same time — reads L2 / MALL instead of queueing on one
  // chip-wide HBM burst.
  auto warmup = [&]() {
  if constexpr (T == 1 && (kLanePrefetch || kPfP0)) {
    if (live) {
      const char* c = reinterpret_cast<const char*>(a.CI + b * (int64_t)(n * m));
      const char* c0 = reinterpret_cast<const char*>(a.ci0 + b * (int64_t)m);
      const int bc = n * m * 8, b0c = m * 8;
#pragma unroll
      for (int k = 0; k < kPfCI; k++)
        pf[k] = (bc >= 4) ? *reinterpret_cast<const uint32_t*>(c + min(k * 128, bc - 4)) : 0u;
#pragma unroll
      for (int k = 0; k < kPfC0; k++)
        pf[kPfCI + k] = (b0c >= 4) ? *reinterpret_cast<const uint32_t*>(c0 + min(k * 128, b0c - 4)) : 0u;
    }
  }
  };
  qp_stamp(a, 0);

  // ---------------------------------------------------------------- setup
  bool chol_ok = live;  // idle lanes (past the batch, or lanes >= QPW) never touch LDS slots
  double bad_sum = 0.0;
  {
    double Gr[NM][NM];
    // round A: G and g0
    const int offg0 = RB;
    stage_all(a.G, n * n, 0);
    stage_all(a.g0, n, offg0);
    __syncthreads();
    double g0v[NM];
#pragma unroll
    for (int i = 0; i < NM; i++) {
#pragma unroll
      for (int j = 0; j < NM; j++) Gr[i][j] = (live && i < n && j < n) ? rd_all(0, n * n, i * n + j) : 0.0;
      g0v[i] = (live && i < n) ? rd_all(offg0, n, i) : 0.0;
    }
    __syncthreads();
    if constexpr (kPfP0) warmup();
    // round B: CE and ce0 (equality phase), issued now so they land during the Cholesky
    if (p > 0) {
      const int np_ = n * p;
      const int offc = (QPW * np_ + 127) / 128 * 128;
      if (offc + QPW * p <= STAGE) {
        stage_all(a.CE, np_, 0);
        stage_all(a.ce0, p, offc);
      }
    }
    if constexpr (QPGPU_LANE_PF_EARLY) warmup();
#pragma unroll
    for (int i = 0; i < NM; i++)
      if (i < n) c1 += Gr[i][i];
    // cholesky_decomposition (@.text+0x2df0): row-wise, descending-k sums, upper mirrored
#pragma unroll
    for (int i = 0; i < NM; i++) {
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
#pragma unroll
          for (int j = i + 1; j < NM; j++)
            if (j < n) {
              double s2 = Gr[i][j];
#pragma unroll
              for (int k = i - 1; k >= 0; k--) s2 -= Gr[i][k] * Gr[j][k];
              Gr[j][i] = s2 / dg;
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
    // round B lands: CE columns into registers (before J overwrites the JA region)
    if (p > 0) {
      const int np_ = n * p;
      const int offc = (QPW * np_ + 127) / 128 * 128;
      ce_staged = offc + QPW * p <= STAGE;
      __syncthreads();  // the staged CE / ce0 are read in the equality phase
    }
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
              v = v / Gr[i][i];
            }
            y[i] = v;
          }
#pragma unroll
          for (int j = 0; j < NM; j++) Jreg[r][j] = y[j];
          if (r < n) c2 += y[r];
        }
      };
      if (lfin)
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
          v = v / Gr[i][i];
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
          xv[i] = v / Gr[i][i];
        }
      }
#pragma unroll
      for (int i = 0; i < NM; i++) xv[i] = -xv[i];
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) fval += g0v[i] * xv[i];
      fval = 0.5 * fval;
    }
  }
  qp_stamp(a, 1);
  if constexpr (!QPGPU_LANE_PF_EARLY) warmup();
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

  // InReg: std::true_type = J in Jreg (setup / equality phase), false_type = LDS image (loop)
  auto Jat = [&](auto InReg, int i, int j) -> double& {
    if constexpr (decltype(InReg)::value)
      return Jreg[i][j];
    else
      return Jr_(i, j);
  };
  const auto kReg = std::true_type{};
  [[maybe_unused]] const auto kLds = std::false_type{};
  auto compute_d = [&](auto InReg) {
#pragma unroll
    for (int c = 0; c < NM; c++) {
      double s = 0.0;
#pragma unroll
      for (int j = 0; j < NM; j++)
        if (j < n) s += Jat(InReg, j, c) * npv[j];
      dv[c] = s;
    }
  };
  // LoC: compile-time lower bound on iq (see add_constraint below)
  auto update_z = [&](auto InReg, auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int r = 0; r < NM; r++) {
      double z = 0.0;
#pragma unroll
      for (int j = LO; j < NM; j++)
        if (j >= iq && j < n) z += Jat(InReg, r, j) * dv[j];
      zv[r] = z;
    }
  };
  auto update_r = [&](auto LoC) {
    constexpr int LO = decltype(LoC)::value;
#pragma unroll
    for (int i = NM - 1; i >= 0; i--) {
      if (i < LO || i < iq) {
        double s = 0.0;
#pragma unroll
        for (int j = i + 1; j < NM; j++)
          if (j < LO || j < iq) s += Rv[RI::at(i, j)] * rv[j];
        rv[i] = (dv[i] - s) / Rv[RI::at(i, i)];
      }
    }
  };
  // LoC: a compile-time lower bound on iq (std::integral_constant).  In the active-set loop
  // iq >= p always (equality constraints are never dropped), so entries below p of R, A, u and
  // d are never the ones written or selected there: with p a compile-time constant (PX) the
  // predicated updates of those entries disappear.
  auto add_constraint = [&](auto InReg, auto LoC) -> bool {
    constexpr int LO = decltype(LoC)::value;
    if (iq >= n) return false;  // reference UB (p > n); reported as dependent
    // |d[j]| as the rotation at j sees it: the previous rotation's h (applied) or the original
    double carried = 0.0;
    if constexpr (QPGPU_LANE_ADDBF) {
      // branch-free rotations: both outcomes of the |h| < eps test computed and selected, so
      // the compiler can overlap rotation j-1's distance() chain (fed by the carried |h|, no
      // division on it) with rotation j's divisions and J update.  Same operations per branch.
#pragma unroll
      for (int j = NM - 1; j >= LO + 1; j--) {
        if (j <= n - 1 && j >= iq + 1) {
          const double cc0 = dv[j - 1], ss0 = dv[j];
          const double h = qp_distance(cc0, j < n - 1 ? carried : ss0);
          const bool app = !(fabs(h) < kEps);
          carried = app ? h : cc0;
          double ss = ss0 / h, cc = cc0 / h;
          const bool neg = cc < 0.0;
          cc = neg ? -cc : cc;
          ss = neg ? -ss : ss;
          dv[j] = app ? 0.0 : ss0;
          dv[j - 1] = app ? (neg ? -h : h) : cc0;
          const double xny = ss / (1.0 + cc);
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k < n) {
              const double t1 = Jat(InReg, k, j - 1), t2 = Jat(InReg, k, j);
              const double n1 = t1 * cc + t2 * ss;
              const double n2 = xny * (t1 + n1) - t2;
              Jat(InReg, k, j - 1) = app ? n1 : t1;
              Jat(InReg, k, j) = app ? n2 : t2;
            }
        }
      }
    } else
#pragma unroll
    for (int j = NM - 1; j >= LO + 1; j--) {
      if (j <= n - 1 && j >= iq + 1) {
        double cc = dv[j - 1], ss = dv[j];
        const double h = qp_distance(cc, (QPGPU_LANE_HCHAIN && j < n - 1) ? carried : ss);
        carried = (fabs(h) < kEps) ? cc : h;
        if (!(fabs(h) < kEps)) {
          dv[j] = 0.0;
          ss = ss / h;
          cc = cc / h;
          if (cc < 0.0) {
            cc = -cc;
            ss = -ss;
            dv[j - 1] = -h;
          } else {
            dv[j - 1] = h;
          }
          const double xny = ss / (1.0 + cc);
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k < n) {
              const double t1 = Jat(InReg, k, j - 1), t2 = Jat(InReg, k, j);
              const double n1 = t1 * cc + t2 * ss;
              Jat(InReg, k, j - 1) = n1;
              Jat(InReg, k, j) = xny * (t1 + n1) - t2;
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
  auto delete_constraint = [&](int l, auto InReg, auto LoC) {
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
        double cc = Rv[RI::at(j, j)], ss = Rv[RI::at(j + 1, j)];
        const double h = qp_distance(cc, ss);
        if (!(fabs(h) < kEps)) {
          cc = cc / h;
          ss = ss / h;
          Rv[RI::at(j + 1, j)] = 0.0;
          if (cc < 0.0) {
            Rv[RI::at(j, j)] = -h;
            cc = -cc;
            ss = -ss;
          } else {
            Rv[RI::at(j, j)] = h;
          }
          const double xny = ss / (1.0 + cc);
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
              const double t1 = Jat(InReg, k, j), t2 = Jat(InReg, k, j + 1);
              const double n1 = t1 * cc + t2 * ss;
              Jat(InReg, k, j) = n1;
              Jat(InReg, k, j + 1) = xny * (n1 + t1) - t2;
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

    // ---------------------------------------------------------------- equality phase
  // Fully unrolled: in step i the active-set size iq equals i (every earlier step added a
  // constraint, or the phase stopped), so pinning iq to the compile-time i folds every
  // iq-predicate of compute_d / update_z / update_r / add_constraint.
  bool done = !ok_lane;
#pragma unroll
  for (int i = 0; i <= NM; i++) {
    if (i < p && !done) {
      iq = i;
      double c0;
      if (i < NM) {
        const int np_ = n * p;
        const int offc = (QPW * np_ + 127) / 128 * 128;
#pragma unroll
        for (int j = 0; j < NM; j++)
          npv[j] = (live && j < n) ? (ce_staged ? rd_all(0, np_, j * p + i)
                                                : view(const_cast<double*>(a.CE), np_)[(j * p + i) * T])
                                   : 0.0;
        c0 = live ? (ce_staged ? rd_all(offc, p, i) : view(const_cast<double*>(a.ce0), p)[i * T]) : 0.0;
      } else {  // p > n: the step that reports "dependent" (reference UB, see oracle)
        const double* CEb = view(const_cast<double*>(a.CE), n * p);
#pragma unroll
        for (int j = 0; j < NM; j++) npv[j] = (j < n) ? CEb[(j * p + i) * T] : 0.0;
        c0 = view(const_cast<double*>(a.ce0), p)[i * T];
      }
      compute_d(kReg);
      update_z(kReg, std::integral_constant<int, 0>{});
      update_r(std::integral_constant<int, 0>{});
      double t2 = 0.0;
      const double zz = dot(zv, zv);
      const double znp = dot(zv, npv);
      if (fabs(zz) > kEps) t2 = (-dot(npv, xv) - c0) / znp;
#pragma unroll
      for (int k = 0; k < NM; k++) xv[k] += t2 * zv[k];
      uv[i < NM + 1 ? i : NM] = t2;
#pragma unroll
      for (int k = 0; k < NM; k++)
        if (k < i) uv[k] -= t2 * rv[k];
      fval += 0.5 * (t2 * t2) * znp;
      Av[i < NM + 1 ? i : NM] = -i - 1;
      if (!add_constraint(kReg, std::integral_constant<int, 0>{})) {
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
  if constexpr (T == 1 && kLanePrefetch) {
    if (live)  // the warm-up loads retire here, long after they landed
#pragma unroll
      for (int k = 0; k < kPfCI + kPfC0; k++) asm volatile("" ::"v"(pf[k]));
  }
  if (!kJregLoop && ok_lane) {
#pragma unroll
    for (int i = 0; i < NM; i++)
#pragma unroll
      for (int j = 0; j < NM; j++) Jr_(i, j) = Jreg[i][j];
  }
  // CI rows 0..kCiRows-1 are kept in LDS for the loop: the first l1 scan (which every active
  // lane runs, loading those rows into registers anyway) writes them there, so each later scan
  // issues only the remaining rows' global loads and the selected-column gather takes those
  // rows from LDS — no extra global traffic and nothing to wait for.
  const bool ci_lds = QPGPU_LANE_CI_LDS && kCiRows > 0 && (a.flags & kArgAligned16);
  bool ci_ready = false;  // wave-uniform: the LDS copy has been written
  // rows kCiRows..NM-1 of CI and ci0 (index NM - kCiRows) in registers (QPGPU_LANE_CI_REGS)
  constexpr bool kCiRegs = (QPGPU_LANE_CI_REGS == 1 || (QPGPU_LANE_CI_REGS == 2 && PX > 0)) && kCiRows > 0;
  constexpr int kRegRows = kCiRegs ? NM + 1 - kCiRows : 1;
  [[maybe_unused]] double cireg[kRegRows][MM];
  // element e (= row * MM + column) of this lane's CI from the LDS copy (e < kCiRows * MM)
  auto ci_lds_at = [&](int e) -> double { return sbuf[((e >> 1) * QPW + lane) * 2 + (e & 1)]; };
  qp_stamp(a, 2);

  // ---------------------------------------------------------------- active-set loop
  // Wave-uniform loop: every lane stays until all 64 are done, so the cooperative CI staging
  // and its barriers are reached by the whole wave; per-lane work is predicated on `active`.
  // Every active lane has iq >= p here (the equality phase completed, only inequalities are
  // ever dropped), so with p known at compile time the loop's iq-indexed updates start at p.
  constexpr int IQLO = PX >= 0 ? (PX <= NM ? PX : NM) : 0;
  const auto kLo = std::integral_constant<int, IQLO>{};
  // where the loop keeps J: registers (kJregLoop) or the LDS image
  const auto kJL = std::integral_constant<bool, kJregLoop>{};
  {
    double sv[MM];
#pragma unroll
    for (int i = 0; i < MM; i++) sv[i] = 0.0;
    // rollback copies: registers (compile-time indices only) or lane-interleaved LDS
    [[maybe_unused]] double xold_r[NM], uold_r[NM];
    [[maybe_unused]] int aold_r[NM];
#define XOLD(i) (*(kRbRegs ? &xold_r[i] : &sbuf[RB + (i) * QPW + lane]))
#define UOLD(i) (*(kRbRegs ? &uold_r[i] : &sbuf[RB_U + (i) * QPW + lane]))
#define AOLD(i) (*(kRbRegs ? &aold_r[i] : reinterpret_cast<int*>(&sbuf[RB_A + (i) * QPW + lane])))
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
    uint64_t tscan = 0, tsel = 0, nloop = 0;  // diagnostic stamps only
    while (wave_any(active)) {
      nloop++;
      const uint64_t tl0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
      // ---- l1: s = CI^T x + ci0, CI staged in row chunks (each s[i] sums j ascending)
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
        // per-lane loads by the scanning lanes only (a full-tile LDS stage per scan moves ~2x
        // the bytes through the CU's load path and measured slower); TILED64 loads are
        // coalesced 512-B rows through a wave-uniform buffer descriptor
        // Software-pipelined two rows deep: row j+1's loads are issued (and fenced from the
        // scheduler) before row j is consumed, so one memory latency covers two rows instead
        // of the scheduler's one-load-at-a-time minimum-pressure order.
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
          // "rows" 0..NM-1 are CI's rows (those >= n are never read), row NM is ci0; row r lands
          // in rowbuf[r % D], issued D-1 rows ahead of its use
          constexpr int D = kScanDepth;
          double rowbuf[D][MM];
          const bool from_lds = ci_lds && ci_ready;
          const bool fill_lds = ci_lds && !ci_ready;
          auto load_row = [&](int r, double* dst) {
            if (kCiRegs && from_lds && r >= kCiRows && r <= NM) {
#pragma unroll
              for (int i = 0; i < MM; i++) dst[i] = cireg[r - kCiRows < kRegRows ? r - kCiRows : 0][i];
              return;
            }
            if (r < NM) {
              if (r < kCiRows && from_lds) {
#pragma unroll
                for (int i = 0; i < MM; i += 2) {
                  const double2 v =
                      *reinterpret_cast<const double2*>(sbuf + (((r * MM + i) >> 1) * QPW + lane) * 2);
                  dst[i] = v.x;
                  dst[i + 1] = v.y;
                }
              } else if (r < n) {
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
          if (QPGPU_LANE_SCANG && kCiRows > 0 && !kCiRegs && from_lds) {
            // every global row in flight first, the LDS rows summed meanwhile (same j order)
            constexpr int NG = NM + 1 - (kCiRows > 0 ? kCiRows : 0);
            double gbuf[NG][MM];
#pragma unroll
            for (int r = NM + 1 - NG; r <= NM; r++) load_row(r, gbuf[r - (NM + 1 - NG)]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < NM; j++) {
              if (j < n) {
                const double xj = xv[j];
                if (j < NM + 1 - NG) {
#pragma unroll
                  for (int i = 0; i < MM; i += 2) {
                    const double2 v =
                        *reinterpret_cast<const double2*>(sbuf + (((j * MM + i) >> 1) * QPW + lane) * 2);
                    if (i < m) sv[i] += v.x * xj;
                    if (i + 1 < m) sv[i + 1] += v.y * xj;
                  }
                } else {
#pragma unroll
                  for (int i = 0; i < MM; i++)
                    if (i < m) sv[i] += gbuf[j - (NM + 1 - NG) < NG ? j - (NM + 1 - NG) : 0][i] * xj;
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
              if (j < kCiRows && fill_lds) {
#pragma unroll
                for (int i = 0; i < MM; i += 2)
                  *reinterpret_cast<double2*>(sbuf + (((j * MM + i) >> 1) * QPW + lane) * 2) =
                      double2{rowbuf[j % D][i], rowbuf[j % D][i + 1]};
              }
              if (kCiRegs && j >= kCiRows && fill_lds) {
#pragma unroll
                for (int i = 0; i < MM; i++) cireg[j - kCiRows < kRegRows ? j - kCiRows : 0][i] = rowbuf[j % D][i];
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
          if (kCiRegs && fill_lds) {
#pragma unroll
            for (int i = 0; i < MM; i++) cireg[kRegRows - 1][i] = rowbuf[NM % D][i];
          }
#pragma unroll
          for (int i = 0; i < MM; i++)
            if (i < m) {
              sv[i] += rowbuf[NM % D][i];
              psi += (sv[i] < 0.0) ? sv[i] : 0.0;
            }
          }
        }
        ci_ready = ci_lds;
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
                UOLD(i) = uv[i];
                AOLD(i) = Av[i];
              }
              XOLD(i) = xv[i];
            }
          }
        }
      }
      const uint64_t tl1 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
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
      if (a.stamps) {
        // make the select's loads part of the select span
        const double sink = npv[0] + ci0ip;
        asm volatile("" ::"v"(sink));
        const uint64_t tl2 = __builtin_amdgcn_s_memtime();
        tscan += tl1 - tl0;
        tsel += tl2 - tl1;
      }
      // ---- l2a
      if (active) {
        if (max_steps > 0 && ++steps > max_steps) {
          status = QPGPU_QP_MAX_ITER;
          active = false;
        } else {
          compute_d(kJL);
          update_z(kJL, kLo);
          update_r(kLo);
          int l = 0;
          double t1 = inf;
#pragma unroll
          for (int k = 0; k < NM; k++)
            if (k >= p && k < iq && rv[k] > 0.0) {
              const double q_ = uv[k] / rv[k];
              const bool take = q_ < t1;
              t1 = take ? q_ : t1;
              l = take ? opq_l(Av[k]) : l;
            }
          const double zz = dot(zv, zv);
          const double znp = dot(zv, npv);
          double t2;
          if (fabs(zz) > kEps) {
            t2 = -lsel<MM>(sv, ip) / znp;
            if (t2 < 0) t2 = inf;  // Takano Akio patch
          } else {
            t2 = inf;
          }
          const double t = (t2 < t1) ? t2 : t1;
          if (t >= inf) {
            status = QPGPU_QP_INFEASIBLE;
            fval = inf;
            active = false;
          } else if (t2 >= inf) {  // dual step only
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < IQLO || k < iq) uv[k] -= t * rv[k];
            lput_lo<IQLO>(uv, iq, lsel_lo<IQLO>(uv, iq) + t);
            act &= ~(1ull << l);
            delete_constraint(l, kJL, kLo);
            need_scan = need_select = false;
          } else {
#pragma unroll
            for (int k = 0; k < NM; k++) xv[k] += t * zv[k];
            fval += t * znp * (0.5 * t + lsel_lo<IQLO>(uv, iq));
#pragma unroll
            for (int k = 0; k < NM; k++)
              if (k < IQLO || k < iq) uv[k] -= t * rv[k];
            lput_lo<IQLO>(uv, iq, lsel_lo<IQLO>(uv, iq) + t);
            if (fabs(t - t2) < kEps) {  // full step
              if (!add_constraint(kJL, kLo)) {
                excl |= 1ull << ip;
                delete_constraint(ip, kJL, kLo);
                act = 0;
#pragma unroll
                for (int i = 0; i < NM; i++)
                  if (i >= p && i < iq) {
                    Av[i] = (int)AOLD(i);
                    uv[i] = UOLD(i);
                    act |= 1ull << Av[i];
                  }
#pragma unroll
                for (int i = 0; i < NM; i++) xv[i] = XOLD(i);
                need_scan = false;
                need_select = true;
              } else {
                act |= 1ull << ip;
                need_scan = need_select = true;
              }
            } else {  // partial step: drop l, refresh s[ip] = CI[:,ip]^T x + ci0[ip]
              act &= ~(1ull << l);
              delete_constraint(l, kJL, kLo);
              double s = 0.0;
#pragma unroll
              for (int j = 0; j < NM; j++)
                if (j < n) s += npv[j] * xv[j];
              lput<MM>(sv, ip, s + ci0ip);
              need_scan = need_select = false;
            }
          }
        }
      }
    }
    if constexpr (T == 1 && kPfP0) {
      if (live)  // the warm-up loads retire here (the first scan waited for them already)
#pragma unroll
        for (int k = 0; k < kPfCI + kPfC0; k++) asm volatile("" ::"v"(pf[k]));
    }
    if (a.stamps && lane == 0) {
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 5] = tscan;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 6] = tsel;
      a.stamps[(uint64_t)blockIdx.x * kStampSlots + 7] = nloop;
    }
  }
#undef Jr_
#undef XOLD
#undef UOLD
#undef AOLD
  qp_stamp(a, 3);

  if (live) {
    if (chol_ok) {
      double* xb = view(a.x, n);
#pragma unroll
      for (int i = 0; i < NM; i++)
        if (i < n) xb[i * T] = xv[i];
    }
    a.f[b] = fval;
    a.status[b] = status;
    if (a.iters) a.iters[b] = iter;
  }
  qp_stamp(a, 4);
}

template <int NM, int MM, int T, int QPW>
static void launch_lane_t(const QpArgs& a, hipStream_t stream) {
  const int64_t blocks = (a.batch + QPW - 1) / QPW;
  const dim3 g((unsigned)blocks), blk(64);
  if (a.n == NM && a.m == MM && !a.x_eq) {
    if (QPW == 64 && a.p == 6)
      hipLaunchKernelGGL((qp_lane_kernel<NM, MM, T, true, QPW, 6>), g, blk, 0, stream, a);
    else if (QPW == 64 && a.p == 0)
      hipLaunchKernelGGL((qp_lane_kernel<NM, MM, T, true, QPW, 0>), g, blk, 0, stream, a);
    else
      hipLaunchKernelGGL((qp_lane_kernel<NM, MM, T, true, QPW, -1>), g, blk, 0, stream, a);
  } else {
    hipLaunchKernelGGL((qp_lane_kernel<NM, MM, T, false, QPW, -1>), g, blk, 0, stream, a);
  }
}

// QPs per wave for the QP-major layout: QPGPU_LANE_QPW=32 runs half-filled waves at two waves
// per SIMD (tuning knob; default 64).
static int lane_qpw() {
  static int v = 0;
  if (!v) {
    const char* e = getenv("QPGPU_LANE_QPW");
    v = (e && atoi(e) == 32) ? 32 : 64;
  }
  return v;
}

template <int NM, int MM>
static hipError_t launch_lane(const QpArgs& a, hipStream_t stream) {
  if (a.tile == 64)
    launch_lane_t<NM, MM, 64, 64>(a, stream);
  else if (lane_qpw() == 32)
    launch_lane_t<NM, MM, 1, 32>(a, stream);
  else
    launch_lane_t<NM, MM, 1, 64>(a, stream);
  return hipGetLastError();
}

struct LaneVariant {
  int nmax, mmax;
  const char* name;
  hipError_t (*launch)(const QpArgs&, hipStream_t);
};

static const LaneVariant kLaneVariants[] = {
    {7, 14, "qp_lane<N=7,M=14>", launch_lane<7, 14>},
    {8, 16, "qp_lane<N=8,M=16>", launch_lane<8, 16>},
};

const LaneVariant* pick_lane(int n, int m) {
  for (const auto& v : kLaneVariants)
    if (n <= v.nmax && m <= v.mmax) return &v;
  return nullptr;
}

}  // namespace qpk

extern "C" hipError_t qpk_launch_lane(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                      const char** name) {
  const qpk::LaneVariant* v = qpk::pick_lane(a->n, a->m);
  if (!v) {
    *handled = 0;
    return hipSuccess;
  }
  *handled = 1;
  if (name) *name = v->name;
  return v->launch(*a, stream);
}

extern "C" const char* qpk_lane_name(int n, int /*p*/, int m) {
  const qpk::LaneVariant* v = qpk::pick_lane(n, m);
  return v ? v->name : nullptr;
}
