// qpgpu_api.cpp — host side of the C-ABI declared in include/qpgpu.h.
//
// Validates the descriptor, picks the gfx950 kernel variant for (n, p, m) and enqueues it on the
// caller's stream.  There is deliberately no CPU path: a shape no kernel covers is an error
// (QPGPU_ERR_UNSUPPORTED_SHAPE), and a missing device is an error (QPGPU_ERR_NO_DEVICE).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/qpgpu.h"
#include "qp_common.h"

extern "C" hipError_t qpk_launch_small(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                       const char** name);
extern "C" const char* qpk_small_name(int n, int p, int m);
extern "C" hipError_t qpk_launch_lane(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                      const char** name);
extern "C" const char* qpk_lane_name(int n, int p, int m);
extern "C" hipError_t qpk_launch_lane_fast(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                           const char** name);
extern "C" const char* qpk_lane_name_fast(int n, int p, int m);
extern "C" hipError_t qpk_launch_medium_ws(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                           const char** name, double* ws);
extern "C" int64_t qpk_medium_workspace_bytes(const qpk::QpArgs* a);
extern "C" const char* qpk_medium_name(int n, int p, int m);
extern "C" const char* qpk_medium_name_fast(int n, int p, int m);
extern "C" int qpk_generic_covers(int n, int m);
extern "C" int64_t qpk_generic_workspace_bytes(int n, int m, int64_t batch);
extern "C" const char* qpk_generic_name(int n, int p, int m);
extern "C" hipError_t qpk_launch_generic(const qpk::QpArgs* a, hipStream_t stream, double* ws);
extern "C" hipError_t qpk_launch_medium_fast(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                             const char** name);
extern "C" int qpk_medium_max_n(void);
extern "C" int qpk_medium_max_m(void);
extern "C" hipError_t qpk_relayout(int64_t batch, int E, const double* src, double* dst,
                                   int to_tiled, hipStream_t stream);

namespace {

thread_local std::string g_last_error;
uint64_t* g_stamps = nullptr;  // diagnostic stamp buffer (qpgpu_debug_set_stamps)

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return QPGPU_ERR_HIP;
}

// Default safety cap on active-set steps (l2a entries).  Goldfarb–Idnani terminates in a
// finite number of steps; the cap only guarantees that every wave drains on pathological
// input and is far above any count seen on terminating problems.
int default_max_steps(int n, int p, int m) { return 1000 + 100 * (n + p + m); }

// The flag rules of include/qpgpu.h: known bits only, FAST excludes EXACT and WRITE_FACTOR, at
// most one forced family.  Shared by validate() and qpgpu_kernel_name_flags().
bool flags_valid(uint32_t flags) {
  const uint32_t fam = QPGPU_FLAG_FORCE_LANE | QPGPU_FLAG_FORCE_SUBGROUP | QPGPU_FLAG_FORCE_WAVE |
                       QPGPU_FLAG_FORCE_GENERIC;
  const uint32_t known = QPGPU_FLAG_WRITE_FACTOR | QPGPU_FLAG_EXACT | QPGPU_FLAG_FAST | fam;
  if (flags & ~known) return false;
  if ((flags & QPGPU_FLAG_FAST) && (flags & (QPGPU_FLAG_EXACT | QPGPU_FLAG_WRITE_FACTOR))) return false;
  const uint32_t f = flags & fam;
  return (f & (f - 1)) == 0;
}

int validate(const qpgpu_problem_desc* d) {
  if (!d) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->n <= 0 || d->p < 0 || d->m < 0 || d->batch < 0) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->layout != QPGPU_LAYOUT_QP_MAJOR && d->layout != QPGPU_LAYOUT_TILED64)
    return QPGPU_ERR_INVALID_ARGUMENT;
  if (!flags_valid(d->flags)) return QPGPU_ERR_INVALID_ARGUMENT;
  return QPGPU_SUCCESS;
}

struct HostWorkspace {
  void* buf = nullptr;
  size_t bytes = 0;
  int device = -1;
  hipStream_t stream = nullptr;
  ~HostWorkspace() {
    if (buf) (void)hipFree(buf);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
thread_local HostWorkspace g_ws;

// Device workspace for the kernels that keep J and R in global memory (n > 64).  Grow-only and
// cached per (device, stream), so launches on different streams never share one; growing syncs
// only the stream that used the old buffer.  The caller keeps `hold` (the cache's lock) until its
// launches are enqueued: a host thread that grows the buffer of a stream another thread has just
// been handed — the default stream, say — would otherwise free it before that thread's kernel is
// in the stream (the stream sync before the free only covers work already enqueued).
struct DevWorkspace {
  void* buf = nullptr;
  size_t bytes = 0;
};
std::mutex g_dev_ws_mu;
std::map<std::pair<int, hipStream_t>, DevWorkspace> g_dev_ws;

int device_workspace(int64_t bytes, hipStream_t stream, double** out, std::unique_lock<std::mutex>& hold) {
  *out = nullptr;
  if (bytes <= 0) return QPGPU_SUCCESS;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (!hold.owns_lock()) hold = std::unique_lock<std::mutex>(g_dev_ws_mu);
  DevWorkspace& w = g_dev_ws[{dev, stream}];
  if (w.bytes < (size_t)bytes) {
    if (w.buf) {
      if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
      (void)hipFree(w.buf);
      w.buf = nullptr;
      w.bytes = 0;
    }
    if ((e = hipMalloc(&w.buf, (size_t)bytes)) != hipSuccess) return hip_fail(e, "hipMalloc workspace");
    w.bytes = (size_t)bytes;
  }
  *out = static_cast<double*>(w.buf);
  return QPGPU_SUCCESS;
}

}  // namespace

extern "C" {

int qpgpu_abi_version(void) { return QPGPU_ABI_VERSION; }

const char* qpgpu_last_error(void) { return g_last_error.c_str(); }

int qpgpu_device_count(void) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) return 0;
  return c;
}

int qpgpu_max_n(void) {
  int mn = qpk_medium_max_n();
  return mn > 16 ? mn : 16;
}

int qpgpu_max_m(void) {
  int mm = qpk_medium_max_m();
  return mm > 64 ? mm : 64;
}

// Default family order: lane (n <= 8, m <= 16), then the subgroup kernel only where it is the
// faster one — n <= 8, m <= 32 (its S = 8 variants) — then the wave kernels.  Measured on MI355X
// with 65 536 QPs per launch (profiles/r01_s2/family_crossover.log): the wave family's
// runtime-sized LDS layout beats the S = 16 subgroup kernel from n = 9 up (n = 14, m = 28:
// 2.2 vs 3.5 ms) and at m = 64; the S = 8 subgroup kernel still wins at n <= 8, m <= 32.
static bool default_small(int n, int m) { return n <= 8 && m <= 32; }

// Largest device workspace one generic-kernel launch uses (bytes); larger batches run as
// sub-batches (solve_batched_impl).  4 GiB; qpgpu_debug_set_generic_ws_cap lowers it in tests.
static int64_t g_generic_ws_cap = (int64_t)4 << 30;

const char* qpgpu_kernel_name_flags(int32_t n, int32_t p, int32_t m, uint32_t flags) {
  if (!flags_valid(flags)) return "";  // the launch would be rejected (QPGPU_ERR_INVALID_ARGUMENT)
  // the generic family has no fast build: FAST | FORCE_GENERIC launches the generic kernel
  // (solve_batched_impl), so it is named before the fast builds
  if (flags & QPGPU_FLAG_FORCE_GENERIC) return qpk_generic_name(n, p, m) ? qpk_generic_name(n, p, m) : "";
  if ((flags & QPGPU_FLAG_FAST) && n > 0 && p >= 0 && m >= 0) {
    // the fast builds: the lane kernel's where it covers the shape, else the wave kernel's LDS
    // variants (n <= 64, m <= 256); a forced family keeps to that family
    const bool lane_ok = !(flags & (QPGPU_FLAG_FORCE_SUBGROUP | QPGPU_FLAG_FORCE_WAVE));
    const char* s = lane_ok ? qpk_lane_name_fast(n, p, m) : nullptr;
    if (s) return s;
    const bool wave_ok = (flags & QPGPU_FLAG_FORCE_WAVE) ||
                         (!(flags & (QPGPU_FLAG_FORCE_LANE | QPGPU_FLAG_FORCE_SUBGROUP)) &&
                          !qpk_lane_name(n, p, m) && !(default_small(n, m) && qpk_small_name(n, p, m)));
    s = wave_ok ? qpk_medium_name_fast(n, p, m) : nullptr;
    if (s) return s;
  }
  if (flags & QPGPU_FLAG_FORCE_LANE) return qpk_lane_name(n, p, m) ? qpk_lane_name(n, p, m) : "";
  if (flags & QPGPU_FLAG_FORCE_SUBGROUP) return qpk_small_name(n, p, m) ? qpk_small_name(n, p, m) : "";
  if (flags & QPGPU_FLAG_FORCE_WAVE) return qpk_medium_name(n, p, m) ? qpk_medium_name(n, p, m) : "";
  if (flags & QPGPU_FLAG_FORCE_GENERIC) return qpk_generic_name(n, p, m) ? qpk_generic_name(n, p, m) : "";
  return qpgpu_kernel_name(n, p, m);
}

const char* qpgpu_kernel_name(int32_t n, int32_t p, int32_t m) {
  if (n <= 0 || p < 0 || m < 0) return "";
  const char* s = qpk_lane_name(n, p, m);
  if (s) return s;
  s = default_small(n, m) ? qpk_small_name(n, p, m) : nullptr;
  if (s) return s;
  s = qpk_medium_name(n, p, m);
  if (s) return s;
  s = qpk_generic_name(n, p, m);  // any other shape (n > 256 or m > 1024)
  return s ? s : "";
}

static int solve_batched_impl(const qpgpu_problem_desc* d, double* G, const double* g0,
                              const double* CE, const double* ce0, const double* CI,
                              const double* ci0, double* x, double* f, int32_t* status,
                              int32_t* iters, double* x_eq, double* f_eq, int32_t* st_eq,
                              void* stream, uint32_t internal = 0);

int qpgpu_solve_batched(const qpgpu_problem_desc* d, double* G, const double* g0,
                        const double* CE, const double* ce0, const double* CI,
                        const double* ci0, double* x, double* f, int32_t* status,
                        int32_t* iters, void* stream) {
  return solve_batched_impl(d, G, g0, CE, ce0, CI, ci0, x, f, status, iters, nullptr, nullptr,
                            nullptr, stream);
}

int qpgpu_solve_batched_eq(const qpgpu_problem_desc* d, double* G, const double* g0,
                           const double* CE, const double* ce0, const double* CI,
                           const double* ci0, double* x, double* f, int32_t* status,
                           int32_t* iters, double* x_eq, double* f_eq, int32_t* status_eq,
                           void* stream) {
  if (!x_eq || !f_eq || !status_eq) return QPGPU_ERR_INVALID_ARGUMENT;
  return solve_batched_impl(d, G, g0, CE, ce0, CI, ci0, x, f, status, iters, x_eq, f_eq,
                            status_eq, stream);
}

static int solve_batched_impl(const qpgpu_problem_desc* d, double* G, const double* g0,
                              const double* CE, const double* ce0, const double* CI,
                              const double* ci0, double* x, double* f, int32_t* status,
                              int32_t* iters, double* x_eq, double* f_eq, int32_t* st_eq,
                              void* stream, uint32_t internal) {
  int rc = validate(d);
  if (rc) return rc;
  if (d->batch == 0) return QPGPU_SUCCESS;
  if (!G || !g0 || !x || !f || !status) return QPGPU_ERR_INVALID_ARGUMENT;
  if ((d->p > 0 && (!CE || !ce0)) || (d->m > 0 && (!CI || !ci0)))
    return QPGPU_ERR_INVALID_ARGUMENT;
  qpk::QpArgs a;
  a.n = d->n;
  a.p = d->p;
  a.m = d->m;
  a.max_steps = d->max_iter > 0 ? d->max_iter : default_max_steps(d->n, d->p, d->m);
  a.batch = d->batch;
  a.tile = d->layout == QPGPU_LAYOUT_TILED64 ? 64 : 1;
  a.flags = d->flags;
  a.G = G;
  a.g0 = g0;
  a.CE = CE;
  a.ce0 = ce0;
  a.CI = CI;
  a.ci0 = ci0;
  a.x = x;
  a.f = f;
  a.status = status;
  a.iters = iters;
  a.x_eq = x_eq;
  a.f_eq = f_eq;
  a.st_eq = st_eq;
  a.stamps = g_stamps;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int handled = 0;
  hipError_t e = hipSuccess;
  std::unique_lock<std::mutex> ws_hold;  // the workspace cache's lock, once a workspace is taken
  a.flags = (d->flags & (QPGPU_FLAG_WRITE_FACTOR | QPGPU_FLAG_EXACT)) | internal;
  const bool fast = (d->flags & QPGPU_FLAG_FAST) != 0;
  auto launch_lane = [&]() {
    return fast ? qpk_launch_lane_fast(&a, s, &handled, nullptr) : qpk_launch_lane(&a, s, &handled, nullptr);
  };
  if (((reinterpret_cast<uintptr_t>(CI) | reinterpret_cast<uintptr_t>(ci0)) & 15u) == 0)
    a.flags |= qpk::kArgAligned16;
  auto launch_wave = [&]() -> int {
    if (fast) {
      e = qpk_launch_medium_fast(&a, s, &handled, nullptr);  // LDS variants (n <= 64, m <= 256)
      if (handled) return QPGPU_SUCCESS;
    }
    double* ws = nullptr;
    const int wrc = device_workspace(qpk_medium_workspace_bytes(&a), s, &ws, ws_hold);
    if (wrc) return wrc;
    e = qpk_launch_medium_ws(&a, s, &handled, nullptr, ws);
    return QPGPU_SUCCESS;
  };
  // The generic kernel's workspace is per QP (2n^2 + 12n + 2m doubles): a large shape launches
  // over sub-batches whose workspace stays within g_generic_ws_cap (one allocation reused by every
  // sub-batch in stream order), instead of one allocation for the whole batch — n = 2000 over
  // 1000 QPs would otherwise ask for ~64 GB and keep it cached.  TILED64 sub-batches are whole
  // 64-QP tiles, so each one's arrays start at a tile boundary.
  auto launch_generic = [&]() -> int {
    if (!qpk_generic_covers(a.n, a.m)) return QPGPU_SUCCESS;  // handled stays 0
    const int64_t per = qpk_generic_workspace_bytes(a.n, a.m, 1);
    if (per <= 0) return QPGPU_SUCCESS;  // handled stays 0
    int64_t chunk = a.batch;
    if (a.batch > g_generic_ws_cap / per) {  // per * batch > cap, without the int64 overflow
      chunk = g_generic_ws_cap / per;
      if (a.tile == 64) chunk = chunk / 64 * 64;
      if (chunk < (a.tile == 64 ? 64 : 1)) chunk = a.tile == 64 ? 64 : 1;
    }
    double* ws = nullptr;
    const int wrc = device_workspace(per * (chunk < a.batch ? chunk : a.batch), s, &ws, ws_hold);
    if (wrc) return wrc;
    handled = 1;
    const int64_t n = a.n, p = a.p, m = a.m;
    auto off = [&](int64_t b0, int64_t E) { return a.tile == 64 ? (b0 / 64) * 64 * E : b0 * E; };
    for (int64_t b0 = 0; b0 < a.batch; b0 += chunk) {
      qpk::QpArgs c = a;
      c.batch = (a.batch - b0 < chunk) ? a.batch - b0 : chunk;
      c.G = a.G + off(b0, n * n);
      c.g0 = a.g0 + off(b0, n);
      if (a.CE) c.CE = a.CE + off(b0, n * p);
      if (a.ce0) c.ce0 = a.ce0 + off(b0, p);
      if (a.CI) c.CI = a.CI + off(b0, n * m);
      if (a.ci0) c.ci0 = a.ci0 + off(b0, m);
      c.x = a.x + off(b0, n);
      c.f = a.f + b0;
      c.status = a.status + b0;
      if (a.iters) c.iters = a.iters + b0;
      if (a.x_eq) c.x_eq = a.x_eq + off(b0, n);
      if (a.f_eq) c.f_eq = a.f_eq + b0;
      if (a.st_eq) c.st_eq = a.st_eq + b0;
      c.stamps = nullptr;
      e = qpk_launch_generic(&c, s, ws);
      if (e != hipSuccess) break;
    }
    return QPGPU_SUCCESS;
  };
  int wrc = QPGPU_SUCCESS;
  if (d->flags & QPGPU_FLAG_FORCE_GENERIC) {
    wrc = launch_generic();
  } else if (d->flags & QPGPU_FLAG_FORCE_LANE) {
    e = launch_lane();
  } else if (d->flags & QPGPU_FLAG_FORCE_SUBGROUP) {
    e = qpk_launch_small(&a, s, &handled, nullptr);
  } else if (d->flags & QPGPU_FLAG_FORCE_WAVE) {
    wrc = launch_wave();
  } else {
    e = launch_lane();
    if (!handled && default_small(a.n, a.m)) e = qpk_launch_small(&a, s, &handled, nullptr);
    if (!handled) wrc = launch_wave();
    if (!wrc && !handled) wrc = launch_generic();
  }
  if (wrc) return wrc;
  if (!handled) return QPGPU_ERR_UNSUPPORTED_SHAPE;
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  return QPGPU_SUCCESS;
}

// Does the forced kernel family (if any) cover the shape?  Checked before any copy is queued.
static bool family_covers(uint32_t flags, int n, int p, int m) {
  if (flags & QPGPU_FLAG_FORCE_LANE) return qpk_lane_name(n, p, m) != nullptr;
  if (flags & QPGPU_FLAG_FORCE_SUBGROUP) return qpk_small_name(n, p, m) != nullptr;
  if (flags & QPGPU_FLAG_FORCE_WAVE) return qpk_medium_name(n, p, m) != nullptr;
  if (flags & QPGPU_FLAG_FORCE_GENERIC) return qpk_generic_covers(n, m) != 0;
  return qpgpu_kernel_name(n, p, m)[0] != 0;
}


// Host-pointer entry (the drop-in's path, one QP per solve_quadprog() call, and the batched
// controller's).  Device buffers are one allocation per thread, laid out
//   [G | g0 | CE | ce0 | CI | ci0 | x || f | status | iters]
// (256-B aligned pieces).  Batches up to kStagedBytes go through a pinned host staging buffer of
// the same layout: the inputs are packed on the host, then ONE H2D copy, the launch and ONE D2H
// copy of [x | f | status | iters] (+ G with WRITE_FACTOR) — instead of 7 + 4 pageable copies —
// which is what a 50 ms control cycle's single solves need (latency, tools/dropin_latency.cpp).
// Larger batches copy each array directly (a host-side pack would only add a pass over them).
// Measured for one C1 QP (profiles/r02_s3/latency.log): 41 us p50 staged, 114 us with per-array
// copies.
static constexpr size_t kStagedBytes = 4u << 20;
// Batches up to g_zero_copy_bytes (a few dozen C1 QPs; one drop-in solve_quadprog() call is 2 KB)
// skip both copies: the kernel reads its inputs from, and writes its outputs to, the pinned
// staging buffer itself (mapped host memory), and the call waits for the stream's completion
// once (a hipStreamQuery spin).  Measured per shape, host to host with the factor written
// back as the drop-in asks (profiles/r06_s6/latency_parts.log, copies -> zero-copy): (7, 6, 14)
// 42.6 -> 38.6 us, (14, 10, 28) 85.3 -> 82.0, (30, 6, 60) 214.1 -> 208.2, but (8, 0, 16)
// 61.2 -> 65.1: without an equality phase the first l1 scan waits on the host-memory reads of CI
// at once, so p = 0 calls keep the copies.
static size_t g_zero_copy_bytes = 64u << 10;  // kZeroCopyBytes; qpgpu_debug_set_zero_copy

struct PinnedStage {
  void* buf = nullptr;
  size_t bytes = 0;
  ~PinnedStage() {
    if (buf) (void)hipHostFree(buf);
  }
};
thread_local PinnedStage g_pin;

int qpgpu_solve_batched_host(const qpgpu_problem_desc* d, double* G, const double* g0,
                             const double* CE, const double* ce0, const double* CI,
                             const double* ci0, double* x, double* f, int32_t* status,
                             int32_t* iters) {
  int rc = validate(d);
  if (rc) return rc;
  if (d->batch == 0) return QPGPU_SUCCESS;
  if (!G || !g0 || !x || !f || !status) return QPGPU_ERR_INVALID_ARGUMENT;
  if ((d->p > 0 && (!CE || !ce0)) || (d->m > 0 && (!CI || !ci0)))
    return QPGPU_ERR_INVALID_ARGUMENT;
  if (!family_covers(d->flags, d->n, d->p, d->m)) return QPGPU_ERR_UNSUPPORTED_SHAPE;
  if (qpgpu_device_count() <= 0) {
    g_last_error = "no HIP device visible";
    return QPGPU_ERR_NO_DEVICE;
  }
  const size_t B = (size_t)d->batch, n = d->n, p = d->p, m = d->m;
  // per-QP-block arrays hold whole tiles in the TILED64 layout
  const size_t BB = d->layout == QPGPU_LAYOUT_TILED64 ? (B + 63) / 64 * 64 : B;
  auto al = [](size_t bytes) { return (bytes + 255) & ~(size_t)255; };
  const size_t nG = BB * n * n * 8, ng0 = BB * n * 8, nCE = BB * n * p * 8, nce0 = BB * p * 8,
               nCI = BB * n * m * 8, nci0 = BB * m * 8, nx = BB * n * 8, nf = B * 8, ns = B * 4,
               ni = B * 4;
  // byte offsets of the pieces
  const size_t oG = 0, og0 = oG + al(nG), oCE = og0 + al(ng0), oce0 = oCE + al(nCE),
               oCI = oce0 + al(nce0), oci0 = oCI + al(nCI), ox = oci0 + al(nci0), of = ox + al(nx),
               os = of + al(nf), oi = os + al(ns), total = oi + al(ni);
  hipError_t e;
  int dev = 0;
  if ((e = hipGetDevice(&dev)) != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (g_ws.device != dev || g_ws.bytes < total) {
    if (g_ws.buf) (void)hipFree(g_ws.buf);
    if (g_ws.stream && g_ws.device != dev) {
      (void)hipStreamDestroy(g_ws.stream);
      g_ws.stream = nullptr;
    }
    g_ws.buf = nullptr;
    g_ws.bytes = 0;
    if ((e = hipMalloc(&g_ws.buf, total)) != hipSuccess) return hip_fail(e, "hipMalloc");
    g_ws.bytes = total;
    g_ws.device = dev;
  }
  if (!g_ws.stream) {
    if ((e = hipStreamCreateWithFlags(&g_ws.stream, hipStreamNonBlocking)) != hipSuccess)
      return hip_fail(e, "hipStreamCreate");
  }
  char* base = static_cast<char*>(g_ws.buf);
  auto D = [&](size_t off) { return reinterpret_cast<double*>(base + off); };
  double* dG = D(oG);
  hipStream_t s = g_ws.stream;
  const bool wf = (d->flags & QPGPU_FLAG_WRITE_FACTOR) != 0;
  const bool staged = total <= kStagedBytes;
  // after a failure past the first queued copy, drain the stream before returning so no copy
  // still reads or writes the caller's buffers
  auto fail_drain = [&](hipError_t err, const char* what) {
    (void)hipStreamSynchronize(s);
    return hip_fail(err, what);
  };
  if (staged) {
    if (g_pin.bytes < total) {
      if (g_pin.buf) (void)hipHostFree(g_pin.buf);
      g_pin.buf = nullptr;
      g_pin.bytes = 0;
      if ((e = hipHostMalloc(&g_pin.buf, total, hipHostMallocDefault)) != hipSuccess)
        return hip_fail(e, "hipHostMalloc");
      g_pin.bytes = total;
    }
    char* h = static_cast<char*>(g_pin.buf);
    auto put = [&](size_t off, const void* src, size_t bytes) {
      if (bytes) std::memcpy(h + off, src, bytes);
    };
    put(oG, G, nG);
    put(og0, g0, ng0);
    put(oCE, CE, nCE);
    put(oce0, ce0, nce0);
    put(oCI, CI, nCI);
    put(oci0, ci0, nci0);
    put(ox, x, nx);  // x passes through unchanged on NONPD
    // f | status | iters poisoned (NaN, -1, -1) and sent with the inputs: outputs a kernel did
    // not write never come back as the previous call's values from the reused device buffer
    std::memset(h + of, 0xFF, total - of);
    if (total <= g_zero_copy_bytes && d->p > 0) {
      // zero-copy: the kernel works on the mapped staging buffer directly
      auto Hp = [&](size_t off) { return reinterpret_cast<double*>(h + off); };
      rc = solve_batched_impl(d, Hp(oG), Hp(og0), Hp(oCE), Hp(oce0), Hp(oCI), Hp(oci0), Hp(ox), Hp(of),
                              reinterpret_cast<int32_t*>(h + os), reinterpret_cast<int32_t*>(h + oi),
                              nullptr, nullptr, nullptr, s);
      if (rc) {
        (void)hipStreamSynchronize(s);
        return rc;
      }
      // The outputs are read once the stream has completed (the end-of-kernel release makes every
      // store visible).  Polling the status words instead (the kernel storing x, f, iters, a
      // system-scope fence, then the status; round 6's first form) raced: a status word was seen
      // with x, or the factor's last rows, still the values the host had staged — in the
      // coarse-grained pinned buffer and in a fine-grained one alike (tests/test_gpu_dropin.py::
      // test_eigen_api_matches_oracle, test_single_calls_outputs_fresh; profiles/r06_f6, r06_s26).
      // A hipStreamQuery spin measured slower than the blocking sync (39.2 vs 36.8 us per C1 call,
      // profiles/r06_s27/latency_parts.log).
      if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
      std::memcpy(x, h + ox, nx);
      std::memcpy(f, h + of, nf);
      std::memcpy(status, h + os, ns);
      if (iters) std::memcpy(iters, h + oi, ni);
      if (wf) std::memcpy(G, h + oG, nG);
      return QPGPU_SUCCESS;
    }
    if ((e = hipMemcpyAsync(base, h, total, hipMemcpyHostToDevice, s)) != hipSuccess)
      return fail_drain(e, "hipMemcpyAsync H2D");
    rc = qpgpu_solve_batched(d, dG, D(og0), D(oCE), D(oce0), D(oCI), D(oci0), D(ox), D(of),
                             reinterpret_cast<int32_t*>(base + os),
                             reinterpret_cast<int32_t*>(base + oi), s);
    if (rc) {
      (void)hipStreamSynchronize(s);
      return rc;
    }
    if ((e = hipMemcpyAsync(h + ox, base + ox, total - ox, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return fail_drain(e, "hipMemcpyAsync D2H");
    if (wf && (e = hipMemcpyAsync(h + oG, base + oG, nG, hipMemcpyDeviceToHost, s)) != hipSuccess)
      return fail_drain(e, "hipMemcpyAsync D2H");
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
    std::memcpy(x, h + ox, nx);
    std::memcpy(f, h + of, nf);
    std::memcpy(status, h + os, ns);
    if (iters) std::memcpy(iters, h + oi, ni);
    if (wf) std::memcpy(G, h + oG, nG);
    return QPGPU_SUCCESS;
  }
  auto h2d = [&](size_t off, const void* src, size_t bytes) -> hipError_t {
    if (!bytes) return hipSuccess;
    return hipMemcpyAsync(base + off, src, bytes, hipMemcpyHostToDevice, s);
  };
  if ((e = h2d(oG, G, nG)) != hipSuccess || (e = h2d(og0, g0, ng0)) != hipSuccess ||
      (e = h2d(oCE, CE, nCE)) != hipSuccess || (e = h2d(oce0, ce0, nce0)) != hipSuccess ||
      (e = h2d(oCI, CI, nCI)) != hipSuccess || (e = h2d(oci0, ci0, nci0)) != hipSuccess ||
      (e = h2d(ox, x, nx)) != hipSuccess)  // x passes through unchanged on NONPD
    return fail_drain(e, "hipMemcpyAsync H2D");
  // f | status | iters poisoned (NaN, -1, -1), as in the staged path
  if ((e = hipMemsetAsync(base + of, 0xFF, total - of, s)) != hipSuccess) return fail_drain(e, "hipMemsetAsync");
  rc = qpgpu_solve_batched(d, dG, D(og0), D(oCE), D(oce0), D(oCI), D(oci0), D(ox), D(of),
                           reinterpret_cast<int32_t*>(base + os),
                           reinterpret_cast<int32_t*>(base + oi), s);
  if (rc) {
    (void)hipStreamSynchronize(s);
    return rc;
  }
  auto d2h = [&](void* dst_, size_t off, size_t bytes) -> hipError_t {
    return hipMemcpyAsync(dst_, base + off, bytes, hipMemcpyDeviceToHost, s);
  };
  if (wf && (e = d2h(G, oG, nG)) != hipSuccess) return fail_drain(e, "hipMemcpyAsync D2H");
  if ((e = d2h(x, ox, nx)) != hipSuccess || (e = d2h(f, of, nf)) != hipSuccess ||
      (e = d2h(status, os, ns)) != hipSuccess || (iters && (e = d2h(iters, oi, ni)) != hipSuccess))
    return fail_drain(e, "hipMemcpyAsync D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return QPGPU_SUCCESS;
}

// ---- several GPUs from one process (qpgpu_solve_batched_multi) ---------------------------------
// One persistent worker thread per shard slot: slot k runs shard k's qpgpu_solve_batched_host on
// the device the call names, with that thread's own device buffers, pinned staging and stream
// (the host entry's thread_local state), so a slot's buffers are reused across calls and two
// slots on the same device never share a stream.  Workers are detached and live for the process.
namespace {
struct ShardWorker {
  std::mutex mu;
  std::condition_variable cv;
  std::function<int()> job;
  bool busy = false;
  int rc = 0;
  std::string err;
  ShardWorker() {
    std::thread([this] {
      for (;;) {
        std::function<int()> j;
        {
          std::unique_lock<std::mutex> lk(mu);
          cv.wait(lk, [this] { return job != nullptr; });
          j = std::move(job);
          job = nullptr;
        }
        const int r = j();
        const std::string e = r == QPGPU_ERR_HIP ? g_last_error : std::string();
        {
          std::lock_guard<std::mutex> lk(mu);
          rc = r;
          err = e;
          busy = false;
        }
        cv.notify_all();
      }
    }).detach();
  }
  void submit(std::function<int()> j) {
    std::lock_guard<std::mutex> lk(mu);
    busy = true;
    job = std::move(j);
    cv.notify_all();
  }
  int wait(std::string* e) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !busy; });
    *e = err;
    return rc;
  }
};
std::mutex g_pool_mu;  // one multi-device call at a time owns the pool
// never destroyed: a worker blocks on its condition variable until the process ends
std::vector<ShardWorker*>& g_pool = *new std::vector<ShardWorker*>();
}  // namespace

int qpgpu_solve_batched_multi(const qpgpu_problem_desc* d, int32_t ndev, const int32_t* devices,
                              double* G, const double* g0, const double* CE, const double* ce0,
                              const double* CI, const double* ci0, double* x, double* f,
                              int32_t* status, int32_t* iters) {
  int rc = validate(d);
  if (rc) return rc;
  if (ndev <= 0 || ndev > 64 || !devices) return QPGPU_ERR_INVALID_ARGUMENT;
  const int have = qpgpu_device_count();
  if (have <= 0) {
    g_last_error = "no HIP device visible";
    return QPGPU_ERR_NO_DEVICE;
  }
  for (int k = 0; k < ndev; k++)
    if (devices[k] < 0 || devices[k] >= have) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->batch == 0) return QPGPU_SUCCESS;
  if (!G || !g0 || !x || !f || !status) return QPGPU_ERR_INVALID_ARGUMENT;
  if ((d->p > 0 && (!CE || !ce0)) || (d->m > 0 && (!CI || !ci0))) return QPGPU_ERR_INVALID_ARGUMENT;
  if (!family_covers(d->flags, d->n, d->p, d->m)) return QPGPU_ERR_UNSUPPORTED_SHAPE;
  const bool tiled = d->layout == QPGPU_LAYOUT_TILED64;
  const int64_t B = d->batch, n = d->n, p = d->p, m = d->m;
  // shard bounds: contiguous, whole tiles in TILED64 (a shard may come out empty)
  std::vector<int64_t> lo(ndev + 1);
  for (int k = 0; k <= ndev; k++) {
    int64_t b = B * k / ndev;
    if (tiled) b = (b + 63) / 64 * 64;
    lo[k] = b < B ? b : B;
  }
  auto off = [&](int64_t b0, int64_t E) { return tiled ? (b0 / 64) * 64 * E : b0 * E; };
  std::lock_guard<std::mutex> pool_hold(g_pool_mu);
  while ((int)g_pool.size() < ndev) g_pool.emplace_back(new ShardWorker());
  std::vector<int> used;
  for (int k = 0; k < ndev; k++) {
    const int64_t b0 = lo[k], cnt = lo[k + 1] - lo[k];
    if (cnt <= 0) continue;
    qpgpu_problem_desc dk = *d;
    dk.batch = cnt;
    const int dev = devices[k];
    g_pool[k]->submit([=]() -> int {
      hipError_t e = hipSetDevice(dev);
      if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
      return qpgpu_solve_batched_host(&dk, G + off(b0, n * n), g0 + off(b0, n), CE ? CE + off(b0, n * p) : CE,
                                      ce0 ? ce0 + off(b0, p) : ce0, CI ? CI + off(b0, n * m) : CI,
                                      ci0 ? ci0 + off(b0, m) : ci0, x + off(b0, n), f + b0, status + b0,
                                      iters ? iters + b0 : iters);
    });
    used.push_back(k);
  }
  int first = QPGPU_SUCCESS;
  for (int k : used) {
    std::string e;
    const int r = g_pool[k]->wait(&e);
    if (r && !first) {
      first = r;
      if (r == QPGPU_ERR_HIP) g_last_error = "device " + std::to_string(devices[k]) + ": " + e;
    }
  }
  return first;
}

// Diagnostic hook (not in include/qpgpu.h): device buffer of kStampSlots uint64 per wave that
// the next launches fill with s_memtime phase stamps; NULL turns it off.
void qpgpu_debug_set_stamps(void* dev_buf) { g_stamps = static_cast<uint64_t*>(dev_buf); }

// Test / measurement hook (not in include/qpgpu.h): largest host-entry call (bytes of inputs and
// outputs) that runs zero-copy on the mapped staging buffer; 0 = always copy.
void qpgpu_debug_set_zero_copy(int64_t bytes) { g_zero_copy_bytes = bytes > 0 ? (size_t)bytes : 0; }

// Test hook (not in include/qpgpu.h): 0 skips the n > 64 default path's EXACT re-solve of the
// QPs its tolerance mode did not certify, leaving their marks (0x100 | reasons << 9) in status.
extern "C" void qpk_set_resolve(int on);
void qpgpu_debug_set_resolve(int on) { qpk_set_resolve(on); }

// Test hook (not in include/qpgpu.h): 0 makes the n > 64 default path's l1 scans fp64-only
// (no fp32 copy of CI), the A/B side of the shadow scan's bitwise test.
extern "C" void qpk_set_shadow(int on);
void qpgpu_debug_set_shadow(int on) { qpk_set_shadow(on); }
// Diagnostic (not in include/qpgpu.h): out[0] = l1 scans of the n > 64 default path that tried
// the fp32 copy of CI, out[1] = those its bounds settled, out[2] = the fp64 re-evaluations of
// candidates those made, since the last reset (reset != 0 zeroes them after reading).
// Synchronises the current device.
extern "C" hipError_t qpk_shadow_stats(unsigned long long* out, int reset);
int qpgpu_debug_shadow_stats(uint64_t* out, int reset) {
  unsigned long long v[3] = {0, 0, 0};
  const hipError_t e = qpk_shadow_stats(v, reset);
  if (e != hipSuccess) return hip_fail(e, "shadow stats");
  for (int k = 0; k < 3; k++) out[k] = v[k];
  return QPGPU_SUCCESS;
}

// Test hook (not in include/qpgpu.h): the generic kernel's per-launch workspace cap in bytes
// (<= 0 restores the 4 GiB default), so the sub-batch path runs on small shapes.
void qpgpu_debug_set_generic_ws_cap(int64_t bytes) { g_generic_ws_cap = bytes > 0 ? bytes : ((int64_t)4 << 30); }

int qpgpu_relayout(int64_t batch, int32_t elems, const double* src, double* dst, int32_t to_tiled,
                   void* stream) {
  if (batch < 0 || elems < 0 || (batch > 0 && elems > 0 && (!src || !dst)))
    return QPGPU_ERR_INVALID_ARGUMENT;
  if (batch == 0 || elems == 0) return QPGPU_SUCCESS;
  hipError_t e = qpk_relayout(batch, elems, src, dst, to_tiled ? 1 : 0,
                              reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "relayout launch");
  return QPGPU_SUCCESS;
}

}  // extern "C"
