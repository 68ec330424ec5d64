// multi_dev_test — the C++ host's multi-GPU call (include/qpgpu.h qpgpu_solve_batched_multi),
// the form north_star asks for ("host code stays C++ ... calling HIP through a thin C-ABI"):
// reads a batch file (int32 B n p m, then per QP G g0 CE ce0 CI ci0 as doubles, QP-major), solves
// it over the devices named on the command line and prints one line per QP (status, l1 passes,
// f and x as hex floats) for tests/test_gpu_multi.py to compare with the oracle.
//   usage: multi_dev_test BATCH_FILE DEV [DEV ...]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "qpgpu.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s BATCH_FILE DEV [DEV ...]\n", argv[0]);
    return 2;
  }
  FILE* fh = std::fopen(argv[1], "rb");
  if (!fh) return 2;
  int32_t hdr[4];
  if (std::fread(hdr, sizeof(int32_t), 4, fh) != 4) return 2;
  const int64_t B = hdr[0];
  const int n = hdr[1], p = hdr[2], m = hdr[3];
  std::vector<double> G(B * n * n), g0(B * n), CE(B * n * p), ce0(B * p), CI(B * n * m), ci0(B * m);
  for (int64_t b = 0; b < B; b++) {
    auto rd = [&](std::vector<double>& v, int64_t e) {
      if (e && std::fread(v.data() + b * e, sizeof(double), e, fh) != (size_t)e) std::exit(2);
    };
    rd(G, (int64_t)n * n);
    rd(g0, n);
    rd(CE, (int64_t)n * p);
    rd(ce0, p);
    rd(CI, (int64_t)n * m);
    rd(ci0, m);
  }
  std::fclose(fh);
  std::vector<int32_t> devs;
  for (int k = 2; k < argc; k++) devs.push_back(std::atoi(argv[k]));

  qpgpu_problem_desc d{};
  d.n = n;
  d.p = p;
  d.m = m;
  d.batch = B;
  std::vector<double> x(B * n), f(B);
  std::vector<int32_t> st(B), it(B);
  const int rc = qpgpu_solve_batched_multi(&d, (int32_t)devs.size(), devs.data(), G.data(), g0.data(),
                                           CE.data(), ce0.data(), CI.data(), ci0.data(), x.data(),
                                           f.data(), st.data(), it.data());
  if (rc != QPGPU_SUCCESS) {
    std::printf("error %d %s\n", rc, qpgpu_last_error());
    return 1;
  }
  for (int64_t b = 0; b < B; b++) {
    std::printf("qp %lld %d %d %a x", (long long)b, st[b], it[b], f[b]);
    for (int i = 0; i < n; i++) std::printf(" %a", x[b * n + i]);
    std::printf("\n");
  }
  std::printf("multi_dev_test: OK %lld QPs over %zu device slots\n", (long long)B, devs.size());
  return 0;
}
