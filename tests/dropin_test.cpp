// dropin_test.cpp — exercises libquadprog_amd.so exactly the way the reference calls
// solve_quadprog (src/mgqp.cpp:700-736): ArrayHH containers, t() temporaries bound to const&,
// the infeasible/NaN retry without inequalities (CI.resize(0, n)), and the exceptions.
// Built by __graft_entry__.build(); run by tests/test_gpu_dropin.py on the GPU box.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include <limits>
#include <stdexcept>
#include <string>

#include "QuadProg++.hh"

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::printf("CHECK FAILED line %d: %s\n", __LINE__, #c);      \
      fails++;                                                      \
    }                                                               \
  } while (0)

static bool same_bits(double a, double b) { return std::memcmp(&a, &b, 8) == 0; }

// --qp FILE: solve every QP of a binary batch (int32 count, n, p, m; then per QP G n*n, g0 n,
// CE n*p (the t(CE) layout), ce0 p, CI n*m, ci0 m — doubles) one solve_quadprog() call at a time,
// the way mgqp calls it (constraint ROWS, then ArrayHH::t() temporaries), and print per QP
// "f <hex> x <hex...> G <hex...>" or the exception.  tests/test_gpu_dropin.py compares the lines
// with the oracle, bit for bit.
static int solve_file(const char* path) {
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return 2;
  int32_t hdr[4];
  if (std::fread(hdr, 4, 4, fp) != 4) return 2;
  const int cnt = hdr[0], n = hdr[1], p = hdr[2], m = hdr[3];
  std::vector<double> buf((size_t)n * n + n + n * p + p + n * m + m);
  for (int q = 0; q < cnt; ++q) {
    if (std::fread(buf.data(), 8, buf.size(), fp) != buf.size()) return 2;
    const double* v = buf.data();
    Matrix<double> G(n, n), CEr(p, n), CIr(m, n);
    Vector<double> g0(n), ce0(p), ci0(m), x;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) G[i][j] = *v++;
    for (int i = 0; i < n; ++i) g0[i] = *v++;
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < p; ++k) CEr[k][i] = *v++;
    for (int k = 0; k < p; ++k) ce0[k] = *v++;
    for (int i = 0; i < n; ++i)
      for (int k = 0; k < m; ++k) CIr[k][i] = *v++;
    for (int k = 0; k < m; ++k) ci0[k] = *v++;
    try {
      const double f = solve_quadprog(G, g0, ArrayHH::t(CEr), ce0, ArrayHH::t(CIr), ci0, x);
      std::printf("f %a x", f);
      for (int i = 0; i < n; ++i) std::printf(" %a", x[i]);
      std::printf(" G");
      for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) std::printf(" %a", G[i][j]);
      std::printf("\n");
    } catch (const std::runtime_error& e) {
      std::printf("runtime_error %s\n", e.what());
    } catch (const std::logic_error& e) {
      std::printf("logic_error %s\n", e.what());
    }
  }
  std::fclose(fp);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[1]) == "--qp") return solve_file(argv[2]);
  // 1. QuadProg++ demo (SURVEY §4 archive output: f = 12, x = [1, 2.0000000000000009])
  {
    Matrix<double> G(2, 2), CE(2, 1), CI(2, 3);
    Vector<double> g0(2), ce0(1), ci0(3), x;
    G[0][0] = 4; G[0][1] = -2; G[1][0] = -2; G[1][1] = 4;
    g0[0] = 6; g0[1] = 0;
    CE[0][0] = 1; CE[1][0] = 1; ce0[0] = -3;
    CI[0][0] = 1; CI[0][1] = 0; CI[0][2] = 1; CI[1][0] = 0; CI[1][1] = 1; CI[1][2] = 1;
    ci0[0] = 0; ci0[1] = 0; ci0[2] = -2;
    double f = solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    CHECK(x.size() == 2);
    CHECK(f == 12.0);
    CHECK(same_bits(x[0], 1.0));
    CHECK(same_bits(x[1], 2.0000000000000009));
    CHECK(G[0][0] == 2.0 && G[1][0] == -1.0 && G[0][1] == -1.0 && same_bits(G[1][1], std::sqrt(3.0)));
  }
  // 2. mgqp solveNextStep pattern: G = I, g0 = 0, t(CE) / t(CI) temporaries, retry path
  {
    const int n = 14, p = 3, m = 28;
    Matrix<double> G(n, n), CE(p, n), CI(m, n);  // mgqp builds constraint ROWS, then t()
    Vector<double> g0(n), ce0(p), ci0(m), x;
    for (int i = 0; i < n; i++) {
      g0[i] = 0.0;
      for (int j = 0; j < n; j++) G[i][j] = (i == j) ? 1.0 : 0.0;
    }
    for (int k = 0; k < p; k++) {
      ce0[k] = 0.3 * (k + 1);
      for (int j = 0; j < n; j++) CE[k][j] = std::sin(0.7 * (k + 1) * (j + 1) * (j + 2) + k);
    }
    for (int k = 0; k < m; k++) {  // [-I; +I] box with limits, ordering of mgqp.cpp:1111-1112
      for (int j = 0; j < n; j++) CI[k][j] = 0.0;
      CI[k][k % n] = (k < n) ? -1.0 : 1.0;
      ci0[k] = 5.0;
    }
    double f = solve_quadprog(G, g0, ArrayHH::t(CE), ce0, ArrayHH::t(CI), ci0, x);
    CHECK(std::isfinite(f));
    CHECK(x.size() == (unsigned)n);
    double r = 0;
    for (int k = 0; k < p; k++) {
      double s = ce0[k];
      for (int j = 0; j < n; j++) s += CE[k][j] * x[j];
      r = std::fmax(r, std::fabs(s));
    }
    CHECK(r < 1e-12);
    // retry without inequalities (mgqp.cpp:723-725): G already holds its factor (I)
    CI.resize(0, n);
    ci0.resize(0);
    double f2 = solve_quadprog(G, g0, ArrayHH::t(CE), ce0, ArrayHH::t(CI), ci0, x);
    CHECK(std::isfinite(f2));
  }
  // 3. infeasible -> +inf
  {
    Matrix<double> G(2, 2), CE(2, 0), CI(2, 2);
    Vector<double> g0(2), ce0(0), ci0(2), x;
    G[0][0] = 1; G[0][1] = 0; G[1][0] = 0; G[1][1] = 1;
    g0[0] = g0[1] = 0;
    CI[0][0] = 1; CI[0][1] = -1; CI[1][0] = 0; CI[1][1] = 0;
    ci0[0] = -1; ci0[1] = 0;
    double f = solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    CHECK(f == std::numeric_limits<double>::infinity());
  }
  // 4. exceptions
  {
    Matrix<double> G(3, 3), CE(3, 2), CI(3, 0);
    Vector<double> g0(3), ce0(2), ci0(0), x;
    for (int i = 0; i < 3; i++) {
      g0[i] = 1;
      for (int j = 0; j < 3; j++) G[i][j] = (i == j) ? 2.0 : 0.0;
    }
    CE[0][0] = 1; CE[0][1] = 1; CE[1][0] = 2; CE[1][1] = 2; CE[2][0] = 0; CE[2][1] = 0;
    ce0[0] = 1; ce0[1] = 1;
    std::string what;
    try {
      solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::runtime_error& e) {
      what = e.what();
    }
    CHECK(what == "Constraints are linearly dependent");
  }
  {
    Matrix<double> G(2, 2), CE(2, 0), CI(2, 0);
    Vector<double> g0(2), ce0(0), ci0(0), x;
    G[0][0] = 1; G[0][1] = 2; G[1][0] = 2; G[1][1] = 1;
    g0[0] = g0[1] = 0;
    std::string what;
    try {
      solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::logic_error& e) {
      what = e.what();
    }
    CHECK(what == "Error in cholesky decomposition, sum: -3");
  }
  {
    Matrix<double> G(2, 3), CE(2, 0), CI(2, 0);
    Vector<double> g0(3), ce0(0), ci0(0), x;
    std::string what;
    try {
      solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::logic_error& e) {
      what = e.what();
    }
    CHECK(what == "The matrix G is not a squared matrix (2 x 3)");
  }
  {
    Matrix<double> G(2, 2), CE(3, 1), CI(2, 0);
    Vector<double> g0(2), ce0(1), ci0(0), x;
    std::string what;
    try {
      solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::logic_error& e) {
      what = e.what();
    }
    CHECK(what == "The matrix CE is incompatible (incorrect number of rows 3 , expecting 2)");
  }
  // 5. shapes no kernel covers: the documented exceptions (include/quadprog_amd/QuadProg++.hh)
  {
    Matrix<double> G(0, 0), CE(0, 0), CI(0, 0);
    Vector<double> g0(0), ce0(0), ci0(0), x;
    std::string what;
    try {
      solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::logic_error& e) {
      what = e.what();
    }
    CHECK(what == "qpgpu: n == 0 is not supported (undefined in QuadProg++)");
  }
  {
    // above the specialised kernels (qpgpu_max_n()): solved like any other size, as by the
    // reference (the generic kernel, qp_generic.hip): G = I, g0 = 1 -> x = -1, f = -n/2
    const unsigned n = 300;
    Matrix<double> G(n, n), CE(n, 0), CI(n, 0);
    Vector<double> g0(n), ce0(0), ci0(0), x;
    for (unsigned i = 0; i < n; i++) {
      g0[i] = 1.0;
      for (unsigned j = 0; j < n; j++) G[i][j] = (i == j) ? 1.0 : 0.0;
    }
    std::string what;
    double f = 0.0;
    try {
      f = solve_quadprog(G, g0, CE, ce0, CI, ci0, x);
    } catch (const std::exception& e) {
      what = e.what();
    }
    CHECK(what.empty());
    CHECK(f == -150.0);
    CHECK(x.size() == n);
    bool all = true;
    for (unsigned i = 0; i < n; i++) all = all && x[i] == -1.0;
    CHECK(all);
  }
  std::printf("dropin_test: %s (%d failures)\n", fails ? "FAIL" : "OK", fails);
  return fails ? 1 : 0;
}
