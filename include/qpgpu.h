/*
 * qpgpu.h — C-ABI of the MI355X-native batched Goldfarb–Idnani QP solver.
 *
 * This is the drop-in boundary for the reference's one hot path,
 *   double solve_quadprog(Matrix<double>& G, Vector<double>& g0,
 *                         const Matrix<double>& CE, const Vector<double>& ce0,
 *                         const Matrix<double>& CI, const Vector<double>& ci0,
 *                         Vector<double>& x);
 * declared at reference include/QuadProgpp/QuadProg++.hh:69-72 (body only in the prebuilt
 * lib/QuadProgpp/libquadprog.a, linked at CMakeLists.txt:95) and called from
 * src/mgqp.cpp:708 and src/mgqp.cpp:725.
 *
 * Problem (QuadProg++.hh:8-13, sign convention :35-37):
 *     min 0.5 x^T G x + g0^T x   s.t.  CE^T x + ce0 = 0,  CI^T x + ci0 >= 0
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * The C++ ArrayHH signature above is re-exported by libquadprog_amd.so (see
 * include/quadprog_amd/QuadProg++.hh), which calls qpgpu_solve_batched_host() for one QP.
 *
 * Two batch layouts (qpgpu_problem_desc.layout).  In both, a QP's matrix is row-major exactly
 * as ArrayHH::Matrix stores it (reference Array.hh:910-919: v[0] = new T[n*m],
 * v[i] = v[i-1] + m); e below is that row-major element index.
 *
 * QPGPU_LAYOUT_QP_MAJOR (0, default): QP b occupies a contiguous block in each array:
 *     G  [b][i][j]  at  G  + b*n*n + i*n + j          (n x n)
 *     g0 [b][i]     at  g0 + b*n + i                   (n)
 *     CE [b][i][k]  at  CE + b*n*p + i*p + k           (n x p, i.e. the t(CE) mgqp passes)
 *     ce0[b][k]     at  ce0 + b*p + k                  (p)
 *     CI [b][i][k]  at  CI + b*n*m + i*m + k           (n x m, i.e. the t(CI) mgqp passes)
 *     ci0[b][k]     at  ci0 + b*m + k                  (m)
 *     x  [b][i]     at  x  + b*n + i                   (n, output)
 *     f[b], status[b], iters[b]                        (outputs; iters may be NULL)
 *
 * QPGPU_LAYOUT_TILED64 (1): QPs are grouped in tiles of 64; inside a tile the element index
 * is the slow axis and the QP index the fast one, so lane t of a wavefront reading element e of
 * QP 64k+t touches consecutive addresses (fully coalesced 512-B rows):
 *     element e of a per-QP block of E elements (E = n*n for G, n for g0/x, n*p for CE, ...)
 *     of QP b lives at  X + (b / 64) * 64 * E + e * 64 + (b % 64).
 *     Arrays hold ceil(batch/64) whole tiles; f, status, iters stay one value per QP.
 * qpgpu_relayout() converts one array between the two layouts on the device.
 */
#ifndef QPGPU_H
#define QPGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QPGPU_ABI_VERSION 1

/* ---- per-QP status (what the reference does for that QP) -------------------------------- */
enum qpgpu_qp_status {
  /* solve_quadprog returned normally; f[b] is its return value (may be NaN, as mgqp.cpp:717 expects). */
  QPGPU_QP_OK = 0,
  /* returned std::numeric_limits<double>::infinity() through the "t >= inf" exit
     (QuadProg++.hh:27-29: problem infeasible, x not meaningful); f[b] = +inf. */
  QPGPU_QP_INFEASIBLE = 1,
  /* cholesky_decomposition hit sum <= 0: the reference prints G and throws
     std::logic_error("Error in cholesky decomposition, sum: <sum>").  f[b] holds that sum. */
  QPGPU_QP_NOT_POSITIVE_DEFINITE = 2,
  /* add_constraint failed in the equality phase: std::runtime_error("Constraints are linearly
     dependent").  f[b] holds the objective accumulated so far. */
  QPGPU_QP_DEPENDENT = 3,
  /* The safety cap on active-set steps was reached.  The reference has no cap (it would loop);
     the cap only exists so every GPU wave terminates and never fires on terminating problems. */
  QPGPU_QP_MAX_ITER = 4
};

/* ---- API return codes ------------------------------------------------------------------- */
enum qpgpu_error {
  QPGPU_SUCCESS = 0,
  QPGPU_ERR_INVALID_ARGUMENT = 1,  /* NULL pointer, negative size, n == 0, ...              */
  QPGPU_ERR_UNSUPPORTED_SHAPE = 2, /* (n, p, m) outside what the compiled kernels cover      */
  QPGPU_ERR_HIP = 3,               /* a HIP runtime call failed (message: qpgpu_last_error) */
  QPGPU_ERR_NO_DEVICE = 4          /* no gfx950 device visible                              */
};

/* batch layouts (see the top of this file) */
#define QPGPU_LAYOUT_QP_MAJOR 0u
#define QPGPU_LAYOUT_TILED64 1u

/* flags */
#define QPGPU_FLAG_WRITE_FACTOR 0x1u  /* write the Cholesky factor back into G, as the
                                          reference does (QuadProg++.hh:42-45).  Off by default
                                          in batched use: it is extra HBM traffic. */

#define QPGPU_FLAG_EXACT 0x2u         /* keep the reference's floating-point operation order
                                          everywhere, so x and f are bit-identical to the CPU
                                          restatement of QuadProg++'s order (SURVEY §3.2;
                                          reference-pinned on the demo KAT only).
                                          Shapes with n <= 64 and m <= 256 always do.  The
                                          others (n > 64, or m > 256, which the workspace
                                          variant serves) by default run the O(n^3) setup
                                          (Cholesky, J = L^-T, x0) as blocked f64 MFMA
                                          (qp_panel.hip) and the loop's d, z, r sums as tree
                                          sums, which match within 1e-10 relative (same status
                                          and iteration counts) instead.  Implied by
                                          QPGPU_FLAG_WRITE_FACTOR. */

#define QPGPU_FLAG_FAST 0x4u          /* n <= 64, m <= 256 (the lane kernel's shapes and the wave
                                          kernel's LDS variants: C1, C2, the mgqp levels, C3):
                                          run the fast builds — multiply-adds fused, one refined
                                          reciprocal per divisor, rotation lengths as
                                          sqrt(a^2 + b^2) inside the exponent range — whose x and
                                          f match the reference within 1e-10 relative per QP
                                          (||x - x_ref||_inf / ||x_ref||_inf, |f - f_ref| /
                                          |f_ref|) with the same decisions on well-conditioned
                                          problems, instead of bit for bit.  Other shapes run as
                                          without it (n > 64 already defaults to the 1e-10 MFMA
                                          panel path).  Not combinable with QPGPU_FLAG_EXACT or
                                          QPGPU_FLAG_WRITE_FACTOR (QPGPU_ERR_INVALID_ARGUMENT). */

/* Kernel-family selection (benchmarking / testing knobs; default = fastest for the shape):
 *   LANE      one QP per lane (qp_lane.hip, n <= 8, m <= 16)
 *   SUBGROUP  one QP per S-lane subgroup, register state (qp_small.hip, n <= 16, m <= 64)
 *   WAVE      one QP per 32/64/256 lanes, LDS / workspace state (qp_wave.hip, n <= 256,
 *             m <= 1024; n > 64 uses a cached device workspace of ~1 MiB per QP, allocated by
 *             the first call for that size — call once before capturing into a hipGraph)
 *   GENERIC   one QP per 256-thread workgroup, every array in a device workspace sized from
 *             (n, m) at run time (qp_generic.hip): ANY shape with n*n and n*m below 2^31, as the
 *             reference's solve_quadprog takes any n, p, m (QuadProg++.hh:69-72).  The default
 *             for the shapes no other family covers (n > 256 or m > 1024); bitwise with the
 *             reference's operation order; ~2 n^2 + 12 n + 2 m doubles of workspace per QP.
 * Forcing a family that does not cover the shape returns QPGPU_ERR_UNSUPPORTED_SHAPE.
 * (Bit 0x1000 selected a lane-pair kernel in ABI 4's round-4 builds; it measured slower than
 * LANE and was removed from the library — the bit is now unknown: QPGPU_ERR_INVALID_ARGUMENT.) */
#define QPGPU_FLAG_FORCE_LANE 0x100u
#define QPGPU_FLAG_FORCE_SUBGROUP 0x200u
#define QPGPU_FLAG_FORCE_WAVE 0x400u
#define QPGPU_FLAG_FORCE_GENERIC 0x800u

typedef struct qpgpu_problem_desc {
  int32_t n;         /* variables                      (G.ncols() in the reference)  */
  int32_t p;         /* equality constraints           (CE.ncols())                  */
  int32_t m;         /* inequality constraints         (CI.ncols())                  */
  int32_t max_iter;  /* safety cap on active-set steps per QP; <= 0 selects the default */
  int64_t batch;     /* number of independent QPs                                    */
  uint32_t flags;    /* QPGPU_FLAG_*                                                  */
  uint32_t layout;   /* QPGPU_LAYOUT_* (0 = QP-major)                                  */
} qpgpu_problem_desc;

/* Solve `d->batch` independent QPs.  Every pointer is DEVICE memory (hipMalloc'd or a torch
 * tensor's data_ptr on the current device); `stream` is a hipStream_t (NULL = default stream).
 * The call only enqueues work and does not synchronise, so it can be captured into a hipGraph.
 * Shapes with n > 64 (J and R in global memory) use a device workspace cached per
 * (device, stream): the first call on a stream allocates it (do that before capturing), and
 * launches on different streams never share one.  Host threads may call concurrently, on one
 * stream or several: the workspace cache's lock is held until a call's launches are enqueued, so
 * launches on one stream share its workspace in stream order.  G is read-only unless
 * QPGPU_FLAG_WRITE_FACTOR is set.
 * `iters` (l1 passes per QP, the reference's `iter`) may be NULL.
 * Replaces: the per-QP call at reference src/mgqp.cpp:708, batched. */
int qpgpu_solve_batched(const qpgpu_problem_desc* d,
                        double* G, const double* g0,
                        const double* CE, const double* ce0,
                        const double* CI, const double* ci0,
                        double* x, double* f, int32_t* status, int32_t* iters,
                        void* stream);

/* Same as qpgpu_solve_batched, plus, per QP, the answer of the same problem with the
 * inequality constraints dropped (m = 0): x_eq (n doubles, same layout as x), f_eq, status_eq.
 * That is the state the full solve passes through after its equality phase, so it costs a
 * few stores, and it is bit-identical to a separate qpgpu_solve_batched with m = 0.  This is
 * the retry of reference src/mgqp.cpp:717-736 (solve_quadprog again with CI of 0 columns)
 * folded into the first solve. */
int qpgpu_solve_batched_eq(const qpgpu_problem_desc* d,
                           double* G, const double* g0,
                           const double* CE, const double* ce0,
                           const double* CI, const double* ci0,
                           double* x, double* f, int32_t* status, int32_t* iters,
                           double* x_eq, double* f_eq, int32_t* status_eq,
                           void* stream);

/* Same, with HOST pointers: copies the inputs to the device, solves, copies the outputs back
 * and synchronises.  This is what the ArrayHH drop-in (libquadprog_amd.so) calls for each
 * solve_quadprog(); it always runs the HIP kernel (there is no CPU path in the product).
 * Each host thread has its own device buffers, pinned staging buffer and stream.
 * G receives the Cholesky factor when QPGPU_FLAG_WRITE_FACTOR is set. */
int qpgpu_solve_batched_host(const qpgpu_problem_desc* d,
                             double* G, const double* g0,
                             const double* CE, const double* ce0,
                             const double* CI, const double* ci0,
                             double* x, double* f, int32_t* status, int32_t* iters);

/* Same as qpgpu_solve_batched_host, over several GPUs of one node from one host process: the
 * batch is split into `ndev` contiguous shards (shard k = QPs [k*B/ndev, (k+1)*B/ndev), rounded
 * to whole 64-QP tiles in the TILED64 layout), shard k is solved on device devices[k] by a
 * worker thread of its own (its own device buffers and stream, kept across calls), and each
 * shard's x, f, status, iters (and the factor in G with QPGPU_FLAG_WRITE_FACTOR) land in the
 * caller's buffers at the shard's offset — the gather of SURVEY §8(e) into host memory.  A device
 * may be listed more than once (its shards then run concurrently on separate streams).
 * Returns when every shard is done: the first failing shard's code, or QPGPU_SUCCESS.  Results
 * are identical to one qpgpu_solve_batched_host call on the whole batch.  ndev <= 64.
 * Replaces: the per-QP call at reference src/mgqp.cpp:708, batched over the node's GPUs. */
int qpgpu_solve_batched_multi(const qpgpu_problem_desc* d, int32_t ndev, const int32_t* devices,
                              double* G, const double* g0,
                              const double* CE, const double* ce0,
                              const double* CI, const double* ci0,
                              double* x, double* f, int32_t* status, int32_t* iters);

/* Convert one per-QP array of `elems` doubles per QP between the layouts on the device
 * (to_tiled = 1: QP-major -> TILED64, 0: back).  src and dst must not overlap; the TILED64
 * side holds ceil(batch/64) whole tiles (padding entries are left untouched / not read).
 * Enqueued on `stream`, no synchronisation. */
int qpgpu_relayout(int64_t batch, int32_t elems, const double* src, double* dst, int32_t to_tiled,
                   void* stream);

/* Largest n / m the specialised kernels accept (lane / subgroup / wave families); larger shapes
 * run on the generic kernel (QPGPU_FLAG_FORCE_GENERIC), whose only limits are n*n < 2^31 and
 * n*m < 2^31 and device memory for its workspace. */
int qpgpu_max_n(void);
int qpgpu_max_m(void);

/* Name of the kernel variant qpgpu_solve_batched would launch for this shape ("" if none). */
const char* qpgpu_kernel_name(int32_t n, int32_t p, int32_t m);
/* The same for a launch with these QPGPU_FLAG_* flags (QPGPU_FLAG_FAST selects the lane
 * kernel's fast build where it covers the shape); "" for a flag combination the solve entry
 * points reject (unknown bits, FAST with EXACT or WRITE_FACTOR, two forced families). */
const char* qpgpu_kernel_name_flags(int32_t n, int32_t p, int32_t m, uint32_t flags);

/* Human-readable text for the last QPGPU_ERR_HIP on this thread. */
const char* qpgpu_last_error(void);

/* Number of visible HIP devices (0 if none). */
int qpgpu_device_count(void);

int qpgpu_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* QPGPU_H */
