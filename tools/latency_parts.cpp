// latency_parts.cpp — where one single-QP solve's host-to-host time goes (BASELINE config 1,
// VERDICT r05 item 7).  One C1 QP (7, 6, 14), each figure the p50 over `reps` calls, host clock:
//   host_entry     qpgpu_solve_batched_host (what solve_quadprog() calls)
//   solve_dev      qpgpu_solve_batched on device pointers + hipStreamSynchronize
//   h2d / d2h      one hipMemcpyAsync of the staged inputs / outputs (pinned) + sync
//   sync_idle      hipStreamSynchronize on an idle stream
//   kernel_ev      the kernel alone between two HIP events (device clock)
//   usage: latency_parts [reps]          (prints one JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "qpgpu.h"

extern "C" void qpgpu_debug_set_zero_copy(int64_t bytes);

static double p50(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int n = 7, p = 6, m = 14;
  // one general QP (SURVEY §8(d) shape): G = M'M + n I, feasible constraints
  std::vector<double> G(n * n), g0(n), CE(n * p), ce0(p), CI(n * m), ci0(m), x(n);
  uint64_t s = 12345;
  auto u = [&] {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return ((z ^ (z >> 31)) >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  };
  std::vector<double> M(n * n);
  for (auto& v : M) v = u();
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      double a = (i == j) ? n : 0.0;
      for (int k = 0; k < n; ++k) a += M[k * n + i] * M[k * n + j];
      G[i * n + j] = a;
    }
  // feasible by construction: ce0 = -CE' xf, ci0 = -CI' xf + |N|
  std::vector<double> xf(n);
  for (auto& v : g0) v = 10 * u();
  for (auto& v : xf) v = 0.1 * u();
  for (auto& v : CE) v = u();
  for (auto& v : CI) v = u();
  for (int k = 0; k < p; ++k) {
    double a = 0;
    for (int i = 0; i < n; ++i) a += CE[i * p + k] * xf[i];
    ce0[k] = -a;
  }
  for (int k = 0; k < m; ++k) {
    double a = 0;
    for (int i = 0; i < n; ++i) a += CI[i * m + k] * xf[i];
    ci0[k] = -a + std::fabs(u());
  }
  qpgpu_problem_desc d{};
  d.n = n;
  d.p = p;
  d.m = m;
  d.batch = 1;
  double f = 0;
  int32_t st = 0, it = 0;
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  auto timeit = [&](const std::function<void()>& fn) {
    std::vector<double> t;
    for (int r = -50; r < reps; ++r) {
      auto a = clk::now();
      fn();
      auto b = clk::now();
      if (r >= 0) t.push_back(us(a, b));
    }
    return p50(t);
  };
  const double host_entry = timeit([&] {
    std::vector<double> Gc(G);
    if (qpgpu_solve_batched_host(&d, Gc.data(), g0.data(), CE.data(), ce0.data(), CI.data(), ci0.data(),
                                 x.data(), &f, &st, &it) != QPGPU_SUCCESS)
      std::exit(1);
  });
  // device pointers
  hipStream_t stream;
  (void)hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  const size_t inb = 8 * (n * n + n + n * p + p + n * m + m);
  double* dbuf = nullptr;
  (void)hipMalloc(&dbuf, inb + 4096);
  double* dG = dbuf;
  double* dg0 = dG + n * n;
  double* dCE = dg0 + n;
  double* dce0 = dCE + n * p;
  double* dCI = dce0 + p;
  double* dci0 = dCI + n * m;
  double* dx = dci0 + m + 8;
  double* df = dx + 16;
  int32_t* dst = reinterpret_cast<int32_t*>(df + 2);
  void* pin = nullptr;
  (void)hipHostMalloc(&pin, inb + 4096, hipHostMallocDefault);
  char* hp = static_cast<char*>(pin);
  size_t o = 0;
  for (auto* v : {&G, &g0, &CE, &ce0, &CI, &ci0}) {
    std::copy(v->begin(), v->end(), reinterpret_cast<double*>(hp + o));
    o += v->size() * 8;
  }
  (void)hipMemcpy(dbuf, pin, inb, hipMemcpyHostToDevice);
  const double solve_dev = timeit([&] {
    qpgpu_solve_batched(&d, dG, dg0, dCE, dce0, dCI, dci0, dx, df, dst, nullptr, stream);
    (void)hipStreamSynchronize(stream);
  });
  const double h2d = timeit([&] {
    (void)hipMemcpyAsync(dbuf, pin, inb, hipMemcpyHostToDevice, stream);
    (void)hipStreamSynchronize(stream);
  });
  const double d2h = timeit([&] {
    (void)hipMemcpyAsync(hp + inb, dx, 8 * (n + 4), hipMemcpyDeviceToHost, stream);  // (past the inputs)
    (void)hipStreamSynchronize(stream);
  });
  const double sync_idle = timeit([&] { (void)hipStreamSynchronize(stream); });
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  std::vector<double> kev;
  for (int r = -50; r < reps; ++r) {
    (void)hipEventRecord(e0, stream);
    qpgpu_solve_batched(&d, dG, dg0, dCE, dce0, dCI, dci0, dx, df, dst, nullptr, stream);
    (void)hipEventRecord(e1, stream);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (r >= 0) kev.push_back(ms * 1e3);
  }
  // zero-copy variants: the same kernel with its inputs and / or outputs in pinned host memory
  // (the GPU reads / writes it over PCIe), and a host that polls the status word instead of
  // synchronising the stream
  void* zin = nullptr;
  void* zout = nullptr;
  (void)hipHostMalloc(&zin, inb + 4096, hipHostMallocDefault);
  (void)hipHostMalloc(&zout, 4096, hipHostMallocDefault);
  std::memcpy(zin, pin, inb);
  double* zG = static_cast<double*>(zin);
  double* zg0 = zG + n * n;
  double* zCE = zg0 + n;
  double* zce0 = zCE + n * p;
  double* zCI = zce0 + p;
  double* zci0 = zCI + n * m;
  double* zx = static_cast<double*>(zout);
  double* zf = zx + 16;
  volatile int32_t* zst = reinterpret_cast<volatile int32_t*>(zf + 2);
  auto kev_of = [&](double* G_, double* g0_, double* CE_, double* ce0_, double* CI_, double* ci0_, double* x_,
                    double* f_, int32_t* st_) {
    std::vector<double> t;
    for (int r = -50; r < reps; ++r) {
      (void)hipEventRecord(e0, stream);
      qpgpu_solve_batched(&d, G_, g0_, CE_, ce0_, CI_, ci0_, x_, f_, st_, nullptr, stream);
      (void)hipEventRecord(e1, stream);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r >= 0) t.push_back(ms * 1e3);
    }
    return p50(t);
  };
  const double k_zin = kev_of(zG, zg0, zCE, zce0, zCI, zci0, dx, df, dst);
  const double k_zout = kev_of(dG, dg0, dCE, dce0, dCI, dci0, zx, zf, const_cast<int32_t*>(zst));
  const double k_zboth = kev_of(zG, zg0, zCE, zce0, zCI, zci0, zx, zf, const_cast<int32_t*>(zst));
  const int zc_status = *zst;
  const double zc_f = *zf;
  // host to host: pack inputs into the pinned buffer, launch on zero-copy pointers, poll status
  const double poll_both = timeit([&] {
    std::memcpy(zin, pin, inb);
    *zst = -1;
    qpgpu_solve_batched(&d, zG, zg0, zCE, zce0, zCI, zci0, zx, zf, const_cast<int32_t*>(zst), nullptr, stream);
    for (long spin = 0; *zst == -1 && spin < 400000000L; ++spin) {
    }
  });
  (void)hipStreamSynchronize(stream);
  // the same, waiting by a hipStreamQuery spin (the host entry's zero-copy path since the status
  // poll was found racy: a status word can be visible before the kernel's other stores)
  const double query_both = timeit([&] {
    std::memcpy(zin, pin, inb);
    qpgpu_solve_batched(&d, zG, zg0, zCE, zce0, zCI, zci0, zx, zf, const_cast<int32_t*>(zst), nullptr, stream);
    while (hipStreamQuery(stream) == hipErrorNotReady) {
    }
  });
  const double sync_both = timeit([&] {
    std::memcpy(zin, pin, inb);
    qpgpu_solve_batched(&d, zG, zg0, zCE, zce0, zCI, zci0, zx, zf, const_cast<int32_t*>(zst), nullptr, stream);
    (void)hipStreamSynchronize(stream);
  });
  // inputs by one H2D copy, outputs zero-copy + poll
  const double h2d_poll = timeit([&] {
    *zst = -1;
    (void)hipMemcpyAsync(dbuf, pin, inb, hipMemcpyHostToDevice, stream);
    qpgpu_solve_batched(&d, dG, dg0, dCE, dce0, dCI, dci0, zx, zf, const_cast<int32_t*>(zst), nullptr, stream);
    for (long spin = 0; *zst == -1 && spin < 400000000L; ++spin) {
    }
  });
  (void)hipStreamSynchronize(stream);
  // the host entry per shape, zero-copy (the library's default for small calls) and copies
  std::string shapes_json;
  for (int sh = 0; sh < 4; ++sh) {
    const int N = sh == 0 ? 7 : (sh == 1 ? 14 : (sh == 2 ? 30 : 8)), P = sh == 0 ? 6 : (sh == 1 ? 10 : (sh == 2 ? 6 : 0)),
              Mm = sh == 0 ? 14 : (sh == 1 ? 28 : (sh == 2 ? 60 : 16));
    std::vector<double> sG(N * N), sg0(N), sCE(N * P), sce0(P), sCI(N * Mm), sci0(Mm), sx(N), sxf(N), sM(N * N);
    for (auto& v : sM) v = u();
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        double a = (i == j) ? N : 0.0;
        for (int k = 0; k < N; ++k) a += sM[k * N + i] * sM[k * N + j];
        sG[i * N + j] = a;
      }
    for (auto& v : sg0) v = 10 * u();
    for (auto& v : sxf) v = 0.1 * u();
    for (auto& v : sCE) v = u();
    for (auto& v : sCI) v = u();
    for (int k = 0; k < P; ++k) {
      double a = 0;
      for (int i = 0; i < N; ++i) a += sCE[i * P + k] * sxf[i];
      sce0[k] = -a;
    }
    for (int k = 0; k < Mm; ++k) {
      double a = 0;
      for (int i = 0; i < N; ++i) a += sCI[i * Mm + k] * sxf[i];
      sci0[k] = -a + std::fabs(u());
    }
    qpgpu_problem_desc sd{};
    sd.n = N;
    sd.p = P;
    sd.m = Mm;
    sd.batch = 1;
    sd.flags = QPGPU_FLAG_WRITE_FACTOR;  // as the drop-in calls it
    double sf[2];
    int32_t sst[2], sit[2];
    double t_mode[2];
    double fz[2];
    for (int zc = 0; zc < 2; ++zc) {
      qpgpu_debug_set_zero_copy(zc ? (64 << 10) : 0);
      t_mode[zc] = timeit([&] {
        std::vector<double> Gc(sG);
        if (qpgpu_solve_batched_host(&sd, Gc.data(), sg0.data(), sCE.data(), sce0.data(), sCI.data(),
                                     sci0.data(), sx.data(), sf, sst, sit) != QPGPU_SUCCESS)
          std::exit(1);
      });
      fz[zc] = sf[0];
    }
    qpgpu_debug_set_zero_copy(64 << 10);
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s\"(%d,%d,%d)\": {\"copies\": %.2f, \"zero_copy\": %.2f, \"same_f\": %s}",
                  sh ? ", " : "", N, P, Mm, t_mode[0], t_mode[1], fz[0] == fz[1] ? "true" : "false");
    shapes_json += buf;
  }
  std::printf("{\"host_entry_by_shape\": {%s}}\n", shapes_json.c_str());
  std::printf("{\"what\": \"one C1 QP, p50 host-clock us (kernel_*: device clock)\", \"reps\": %d, "
              "\"host_entry\": %.2f, \"solve_dev\": %.2f, \"h2d\": %.2f, \"d2h\": %.2f, \"sync_idle\": %.2f, "
              "\"kernel_ev\": %.2f, \"kernel_zc_in\": %.2f, \"kernel_zc_out\": %.2f, \"kernel_zc_both\": %.2f, "
              "\"zc_both_poll\": %.2f, \"zc_both_query\": %.2f, \"zc_both_sync\": %.2f, \"h2d_zc_out_poll\": %.2f, \"status\": %d, \"f\": %.17g, \"zc_status\": %d, \"zc_f\": %.17g}\n",
              reps, host_entry, solve_dev, h2d, d2h, sync_idle, p50(kev), k_zin, k_zout, k_zboth, poll_both,
              query_both, sync_both, h2d_poll, st, f, zc_status, zc_f);
  return 0;
}
