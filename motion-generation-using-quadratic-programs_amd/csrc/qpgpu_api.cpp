// qpgpu_api.cpp — host side of the C-ABI declared in include/qpgpu.h.
//
// Validates the descriptor, picks the gfx950 kernel variant for (n, p, m) and enqueues it on the
// caller's stream.  There is deliberately no CPU path: a shape no kernel covers is an error
// (QPGPU_ERR_UNSUPPORTED_SHAPE), and a missing device is an error (QPGPU_ERR_NO_DEVICE).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "../../include/qpgpu.h"
#include "qp_common.h"

extern "C" hipError_t qpk_launch_small(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                       const char** name);
extern "C" const char* qpk_small_name(int n, int p, int m);
extern "C" hipError_t qpk_launch_lane(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                      const char** name);
extern "C" const char* qpk_lane_name(int n, int p, int m);
extern "C" hipError_t qpk_launch_medium_ws(const qpk::QpArgs* a, hipStream_t stream, int* handled,
                                           const char** name, double* ws);
extern "C" int64_t qpk_medium_workspace_bytes(int n, int m, int64_t batch);
extern "C" const char* qpk_medium_name(int n, int p, int m);
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

int validate(const qpgpu_problem_desc* d) {
  if (!d) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->n <= 0 || d->p < 0 || d->m < 0 || d->batch < 0) return QPGPU_ERR_INVALID_ARGUMENT;
  if (d->layout != QPGPU_LAYOUT_QP_MAJOR && d->layout != QPGPU_LAYOUT_TILED64)
    return QPGPU_ERR_INVALID_ARGUMENT;
  const uint32_t fam = QPGPU_FLAG_FORCE_LANE | QPGPU_FLAG_FORCE_SUBGROUP | QPGPU_FLAG_FORCE_WAVE;
  const uint32_t known = QPGPU_FLAG_WRITE_FACTOR | QPGPU_FLAG_EXACT | fam;
  if (d->flags & ~known) return QPGPU_ERR_INVALID_ARGUMENT;
  const uint32_t f = d->flags & fam;
  if (f & (f - 1)) return QPGPU_ERR_INVALID_ARGUMENT;  // at most one family
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
// only the stream that used the old buffer.
struct DevWorkspace {
  void* buf = nullptr;
  size_t bytes = 0;
};
std::mutex g_dev_ws_mu;
std::map<std::pair<int, hipStream_t>, DevWorkspace> g_dev_ws;

int device_workspace(int64_t bytes, hipStream_t stream, double** out) {
  *out = nullptr;
  if (bytes <= 0) return QPGPU_SUCCESS;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(g_dev_ws_mu);
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

const char* qpgpu_kernel_name(int32_t n, int32_t p, int32_t m) {
  if (n <= 0 || p < 0 || m < 0) return "";
  const char* s = qpk_lane_name(n, p, m);
  if (s) return s;
  s = default_small(n, m) ? qpk_small_name(n, p, m) : nullptr;
  if (s) return s;
  s = qpk_medium_name(n, p, m);
  return s ? s : "";
}

static int solve_batched_impl(const qpgpu_problem_desc* d, double* G, const double* g0,
                              const double* CE, const double* ce0, const double* CI,
                              const double* ci0, double* x, double* f, int32_t* status,
                              int32_t* iters, double* x_eq, double* f_eq, int32_t* st_eq,
                              void* stream);

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
                              void* stream) {
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
  a.flags = d->flags & (QPGPU_FLAG_WRITE_FACTOR | QPGPU_FLAG_EXACT);
  if (((reinterpret_cast<uintptr_t>(CI) | reinterpret_cast<uintptr_t>(ci0)) & 15u) == 0)
    a.flags |= qpk::kArgAligned16;
  auto launch_wave = [&]() -> int {
    double* ws = nullptr;
    const int wrc = device_workspace(qpk_medium_workspace_bytes(a.n, a.m, a.batch), s, &ws);
    if (wrc) return wrc;
    e = qpk_launch_medium_ws(&a, s, &handled, nullptr, ws);
    return QPGPU_SUCCESS;
  };
  int wrc = QPGPU_SUCCESS;
  if (d->flags & QPGPU_FLAG_FORCE_LANE) {
    e = qpk_launch_lane(&a, s, &handled, nullptr);
  } else if (d->flags & QPGPU_FLAG_FORCE_SUBGROUP) {
    e = qpk_launch_small(&a, s, &handled, nullptr);
  } else if (d->flags & QPGPU_FLAG_FORCE_WAVE) {
    wrc = launch_wave();
  } else {
    e = qpk_launch_lane(&a, s, &handled, nullptr);
    if (!handled && default_small(a.n, a.m)) e = qpk_launch_small(&a, s, &handled, nullptr);
    if (!handled) wrc = launch_wave();
  }
  if (wrc) return wrc;
  if (!handled) return QPGPU_ERR_UNSUPPORTED_SHAPE;
  if (e != hipSuccess) return hip_fail(e, "kernel launch");
  return QPGPU_SUCCESS;
}

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
  if (!qpgpu_kernel_name(d->n, d->p, d->m)[0]) return QPGPU_ERR_UNSUPPORTED_SHAPE;
  if (qpgpu_device_count() <= 0) {
    g_last_error = "no HIP device visible";
    return QPGPU_ERR_NO_DEVICE;
  }
  const size_t B = (size_t)d->batch, n = d->n, p = d->p, m = d->m;
  // per-QP-block arrays hold whole tiles in the TILED64 layout
  const size_t BB = d->layout == QPGPU_LAYOUT_TILED64 ? (B + 63) / 64 * 64 : B;
  auto al = [](size_t bytes) { return (bytes + 255) & ~(size_t)255; };
  const size_t bG = al(BB * n * n * 8), bg0 = al(BB * n * 8), bCE = al(BB * n * p * 8),
               bce0 = al(BB * p * 8), bCI = al(BB * n * m * 8), bci0 = al(BB * m * 8),
               bx = al(BB * n * 8), bf = al(B * 8), bs = al(B * 4), bi = al(B * 4);
  const size_t total = bG + bg0 + bCE + bce0 + bCI + bci0 + bx + bf + bs + bi;
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
  double* dG = reinterpret_cast<double*>(base);
  double* dg0 = reinterpret_cast<double*>(base + bG);
  double* dCE = reinterpret_cast<double*>(base + bG + bg0);
  double* dce0 = reinterpret_cast<double*>(base + bG + bg0 + bCE);
  double* dCI = reinterpret_cast<double*>(base + bG + bg0 + bCE + bce0);
  double* dci0 = reinterpret_cast<double*>(base + bG + bg0 + bCE + bce0 + bCI);
  double* dx = reinterpret_cast<double*>(base + bG + bg0 + bCE + bce0 + bCI + bci0);
  double* df = reinterpret_cast<double*>(base + bG + bg0 + bCE + bce0 + bCI + bci0 + bx);
  int32_t* dst =
      reinterpret_cast<int32_t*>(base + bG + bg0 + bCE + bce0 + bCI + bci0 + bx + bf);
  int32_t* dit =
      reinterpret_cast<int32_t*>(base + bG + bg0 + bCE + bce0 + bCI + bci0 + bx + bf + bs);
  hipStream_t s = g_ws.stream;
  auto h2d = [&](void* dst_, const void* src, size_t bytes) -> hipError_t {
    if (!bytes) return hipSuccess;
    return hipMemcpyAsync(dst_, src, bytes, hipMemcpyHostToDevice, s);
  };
  if ((e = h2d(dG, G, BB * n * n * 8)) != hipSuccess || (e = h2d(dg0, g0, BB * n * 8)) != hipSuccess ||
      (e = h2d(dCE, CE, BB * n * p * 8)) != hipSuccess ||
      (e = h2d(dce0, ce0, BB * p * 8)) != hipSuccess ||
      (e = h2d(dCI, CI, BB * n * m * 8)) != hipSuccess ||
      (e = h2d(dci0, ci0, BB * m * 8)) != hipSuccess ||
      (e = h2d(dx, x, BB * n * 8)) != hipSuccess)  // x passes through unchanged on NONPD
    return hip_fail(e, "hipMemcpyAsync H2D");
  rc = qpgpu_solve_batched(d, dG, dg0, dCE, dce0, dCI, dci0, dx, df, dst, dit, s);
  if (rc) return rc;
  auto d2h = [&](void* dst_, const void* src, size_t bytes) -> hipError_t {
    return hipMemcpyAsync(dst_, src, bytes, hipMemcpyDeviceToHost, s);
  };
  if ((d->flags & QPGPU_FLAG_WRITE_FACTOR) && (e = d2h(G, dG, BB * n * n * 8)) != hipSuccess)
    return hip_fail(e, "hipMemcpyAsync D2H");
  if ((e = d2h(x, dx, BB * n * 8)) != hipSuccess || (e = d2h(f, df, B * 8)) != hipSuccess ||
      (e = d2h(status, dst, B * 4)) != hipSuccess ||
      (iters && (e = d2h(iters, dit, B * 4)) != hipSuccess))
    return hip_fail(e, "hipMemcpyAsync D2H");
  if ((e = hipStreamSynchronize(s)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize");
  return QPGPU_SUCCESS;
}

// Diagnostic hook (not in include/qpgpu.h): device buffer of kStampSlots uint64 per wave that
// the next launches fill with s_memtime phase stamps; NULL turns it off.
void qpgpu_debug_set_stamps(void* dev_buf) { g_stamps = static_cast<uint64_t*>(dev_buf); }

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
