// dropin_latency.cpp — BASELINE config 1 measured as the reference runs it: ONE solve at a time,
// host to host, through the drop-in C++ symbol (src/mgqp.cpp:708 calls solve_quadprog with
// ArrayHH containers and t() temporaries), and one whole updateHook cycle of the controller
// (src/mgqp.cpp:872-1189: two levels, each a solve plus possibly the retry without
// inequalities), against the 50 ms control period of ops/mgqp.ops:184.
//
// usage: dropin_latency [solves] [cycles]      (prints one JSON line)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "QuadProg++.hh"
#include "quadprog_amd/mgqp.hh"

static uint64_t g_s = 12345;
static double nrm() {  // Box-Muller over SplitMix64
  auto u = [] {
    uint64_t z = (g_s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return ((z >> 11) + 1.0) * (1.0 / 9007199254740992.0);
  };
  const double a = u(), b = u();
  return std::sqrt(-2.0 * std::log(a)) * std::cos(6.283185307179586 * b);
}

struct Stats {
  double p50, p99, mean, max;
};
static Stats stats(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  double s = 0;
  for (double x : v) s += x;
  return {v[v.size() / 2], v[(size_t)(v.size() * 0.99)], s / v.size(), v.back()};
}

int main(int argc, char** argv) {
  const int solves = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int cycles = argc > 2 ? std::atoi(argv[2]) : 500;
  const int n = 7, p = 6, m = 14;
  using clk = std::chrono::steady_clock;

  // ---- single (7, 6, 14) solves, a fresh general QP each call (SURVEY §8(d) generator shape)
  std::vector<double> t_solve;
  int ok = 0;
  for (int it = -50; it < solves; ++it) {
    Matrix<double> G(n, n), CE(p, n), CI(m, n);  // constraint ROWS, then t(), as mgqp builds them
    Vector<double> g0(n), ce0(p), ci0(m), x, xf(n);
    std::vector<double> M(n * n);
    for (auto& v : M) v = nrm();
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double s = (i == j) ? n : 0.0;
        for (int k = 0; k < n; ++k) s += M[k * n + i] * M[k * n + j];
        G[i][j] = s;
      }
    for (int i = 0; i < n; ++i) {
      g0[i] = 10.0 * nrm();
      xf[i] = 0.1 * nrm();
    }
    for (int k = 0; k < p; ++k) {
      double s = 0;
      for (int j = 0; j < n; ++j) s += (CE[k][j] = nrm()) * xf[j];
      ce0[k] = -s;
    }
    for (int k = 0; k < m; ++k) {
      double s = 0;
      for (int j = 0; j < n; ++j) s += (CI[k][j] = nrm()) * xf[j];
      ci0[k] = -s + std::fabs(nrm());
    }
    const auto t0 = clk::now();
    const double f = solve_quadprog(G, g0, ArrayHH::t(CE), ce0, ArrayHH::t(CI), ci0, x);
    const auto t1 = clk::now();
    if (it >= 0) {
      t_solve.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      ok += std::isfinite(f) ? 1 : 0;
    }
  }

  // ---- one controller cycle (updateHook), ops/mgqp.ops configuration, DOF 7
  mgqp_amd::MotionGenerationQuadraticProgram c;
  const int dof = 7;
  c.setDOFsize(dof);
  c.setTorqueLimits(std::vector<double>(dof, 100.0), std::vector<double>(dof, -100.0));
  c.setAccelerationLimits(std::vector<double>(dof, 5.0), std::vector<double>(dof, -5.0));
  c.setAngularLimits({0.8, 1.5, 2.5, 1.5, 3.0, 1.5, 3.0}, {-0.8, -1.5, -2.5, -1.5, -3.0, -1.5, -3.0});
  c.setPriorityLevel("in_desiredTaskSpacePosition_7", 0);
  c.setPriorityLevel("in_desiredTaskSpaceVelocity_7", 0);
  c.setPriorityLevel("in_desiredTaskSpaceAcceleration_7", 0);
  c.setPriorityLevel("in_desiredJointSpacePosition_1", 2);
  std::vector<double> t_cycle;
  int written = 0;
  for (int it = -20; it < cycles; ++it) {
    mgqp_amd::CycleInputs in;
    mgqp_amd::JointState js;
    for (int j = 0; j < dof; ++j) {
      js.angles.push_back((float)(0.3 * nrm()));
      js.velocities.push_back((float)(0.2 * nrm()));
    }
    in.robotstatus.set(js);
    mgqp_amd::VecF h(dof);
    for (auto& v : h) v = (float)nrm();
    in.h.set(h);
    mgqp_amd::MatF Mi = mgqp_amd::MatF::identity(dof);
    for (int i = 0; i < dof; ++i) Mi(i, i) += (float)(0.5 + 0.1 * std::fabs(nrm()));
    in.inertia.set(Mi);
    in.joints.resize(dof);
    auto& j7 = in.joints[dof - 1];
    mgqp_amd::MatF J(3, dof), Jd(3, dof);
    for (auto& v : J.a) v = (float)(0.5 * nrm());
    for (auto& v : Jd.a) v = (float)(0.05 * nrm());
    j7.jacobian.set(J);
    j7.jacobianDot.set(Jd);
    auto v3 = [](double sc) { return mgqp_amd::VecF{(float)(sc * nrm()), (float)(sc * nrm()), (float)(sc * nrm())}; };
    j7.currentTaskSpacePosition.set(v3(0.5));
    j7.currentTaskSpaceVelocity.set(v3(0.1));
    j7.currentTaskSpaceAcceleration.set(v3(0.1));
    j7.desiredTaskSpacePosition.set(v3(0.5));
    j7.desiredTaskSpaceVelocity.set(v3(0.1));
    j7.desiredTaskSpaceAcceleration.set(v3(0.1));
    in.joints[0].desiredJointSpacePosition.set((float)(0.3 * nrm()));
    mgqp_amd::CycleOutputs out;
    const auto t0 = clk::now();
    c.updateHook(in, out);
    const auto t1 = clk::now();
    if (it >= 0) {
      t_cycle.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      written += out.code == mgqp_amd::CYCLE_WRITTEN;
    }
  }
  const Stats a = stats(t_solve), b = stats(t_cycle);
  std::printf(
      "{\"what\": \"BASELINE config 1: one solve_quadprog() / one updateHook cycle, host to host\", "
      "\"staging\": \"%s\", \"solve_us\": {\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f, \"max\": %.2f, "
      "\"n\": %d, \"finite\": %d}, \"cycle_us\": {\"p50\": %.2f, \"p99\": %.2f, \"mean\": %.2f, "
      "\"max\": %.2f, \"n\": %d, \"written\": %d}, \"period_us\": 50000}\n",
      "pinned, 1 H2D + 1 D2H", a.p50, a.p99, a.mean,
      a.max, solves, ok, b.p50, b.p99, b.mean, b.max, cycles, written);
  return 0;
}
