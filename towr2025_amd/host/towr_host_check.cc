// towr_host_check — C++ host driver over the C-ABI, used by the tests (tests/test_cpp_host.py).
// It builds a BASELINE configuration through the C++ NlpFormulation mirror, creates the engine and
// walks the IPOPT callback sequence of one iteration:
//   get_nlp_info -> eval_jac_g(structure) -> eval_f(x, new_x = true) -> eval_grad_f(x, false)
//   -> eval_g(x, false) -> eval_jac_g(x, false)
// and dumps everything to a binary file:
//   desc bytes | n m (int32) nnz (int64) | x0[n] | iRow[nnz] jCol[nnz] | (device >= 0) g[m] values[nnz] f grad[n]
// and (device >= 0) the trajectory of x0 sampled at 0.01 s as SaveTrajectoryToCSV writes it, to <out.bin>.csv
// usage: towr_host_check <anymal|anymal_costs|anymal_rotvec|anymal_gait|biped|biped_next|hopper> <out.bin> [device (default -1: layout only)]
//        towr_host_check <cfg> --zerocopy [device] [timed iterations]
//   the zero-copy Jacobian of NlpCallbacks (towr_gpu.hpp) against the engine's own evaluation, bit for bit: IPOPT's
//   values array stable across calls (TNLPAdapter's jac_g_), g before J and J before g, a values array that moves
//   between calls, and the array after finalize_solution; then per-iteration timings (eval_g + eval_jac_g through the
//   callbacks, and eval_jac_g alone) against the cached path (one fused evaluation into the page-locked cache + the
//   nnz-value copy into IPOPT's array). Prints one line "zerocopy ok ..." or fails with a message.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nlp_formulation.hpp"
#include "towr_gpu.hpp"

using namespace towr_gpu;

namespace {

double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0.0 : v[v.size() / 2];
}

int zerocopy_check(const towr_problem_desc_t& d, int device, int iters) {
  Engine e(d, device);
  const int n = e.GetNumberOfOptimizationVariables(), m = e.GetNumberOfConstraints();
  const int nnz = (int)e.GetNumberOfJacobianNonzeros();
  const std::vector<double> x0 = e.GetVariableValues();
  std::vector<std::vector<double>> xs;
  for (int k = 0; k < 3; ++k) {   // x0 and two deterministic perturbations
    std::vector<double> x = x0;
    for (int i = 0; i < n; ++i) x[i] += 0.01 * k * std::sin(0.37 * i + k);
    xs.push_back(x);
  }
  std::vector<std::vector<double>> gr(3, std::vector<double>(m)), vr(3, std::vector<double>(nnz));
  for (int k = 0; k < 3; ++k) e.EvalConstraintsAndJacobian(xs[k].data(), gr[k].data(), vr[k].data());   // the engine's own (staged) evaluation
  auto same = [&](const std::vector<double>& a, const std::vector<double>& b, const char* what, int k) {
    if (std::memcmp(a.data(), b.data(), a.size() * sizeof(double)) != 0) {
      std::fprintf(stderr, "zerocopy: %s differs at x %d\n", what, k);
      return false;
    }
    return true;
  };
  NlpCallbacks nlp(e);
  std::vector<double> g(m), jac_g(nnz);   // IPOPT's TNLPAdapter arrays: allocated once per solve
  for (int rep = 0; rep < 2; ++rep)
    for (int k = 0; k < 3; ++k) {
      std::fill(jac_g.begin(), jac_g.end(), NAN);
      bool ok;
      if (rep == 0) ok = nlp.eval_g(n, xs[k].data(), true, m, g.data()) && nlp.eval_jac_g(n, xs[k].data(), false, m, nnz, nullptr, nullptr, jac_g.data());
      else ok = nlp.eval_jac_g(n, xs[k].data(), true, m, nnz, nullptr, nullptr, jac_g.data()) && nlp.eval_g(n, xs[k].data(), false, m, g.data());
      if (!ok) { std::fprintf(stderr, "zerocopy: callback failed: %s\n", towr_gpu_last_error(e.handle())); return 1; }
      if (!same(g, gr[k], rep ? "g (J first)" : "g", k) || !same(jac_g, vr[k], rep ? "values (J first)" : "values", k)) return 1;
      // (a small Jacobian is copied from the page-locked cache when g came first: no registration then)
      if (!nlp.values_zero_copy() && !(nlp.small_jacobian() && rep == 0)) {
        std::fprintf(stderr, "zerocopy: IPOPT's array was not registered\n");
        return 1;
      }
    }
  if (nlp.values_registrations() != 1) { std::fprintf(stderr, "zerocopy: %d registrations of a stable array\n", nlp.values_registrations()); return 1; }
  for (int k = 0; k < 3; ++k) {   // a values array that moves between calls
    std::vector<double> moved(nnz, NAN);
    if (!nlp.eval_g(n, xs[k].data(), true, m, g.data()) || !nlp.eval_jac_g(n, xs[k].data(), false, m, nnz, nullptr, nullptr, moved.data())) return 1;
    if (!same(moved, vr[k], "values (moved array)", k)) return 1;
    nlp.finalize_solution();   // (the vector is freed next: release its registration first)
  }
  const int want_reg = nlp.small_jacobian() ? 1 : 4;   // (g first: a small Jacobian is copied from the cache)
  if (nlp.values_registrations() != want_reg) {
    std::fprintf(stderr, "zerocopy: %d registrations, expected %d\n", nlp.values_registrations(), want_reg);
    return 1;
  }
  // timings: IPOPT's per-iteration pair through the callbacks, against the cached path of round 4 (one fused
  // evaluation into page-locked g / values caches, then both copied into IPOPT's arrays)
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  std::vector<double> t_pair, t_jac, t_old, t_oldjac;
  std::vector<double> cg(m), cv(nnz);
  const bool pg = e.RegisterHost(cg.data(), cg.size() * sizeof(double)) == TOWR_OK;
  const bool pv = e.RegisterHost(cv.data(), cv.size() * sizeof(double)) == TOWR_OK;
  for (int it = 0; it < iters + 10; ++it) {
    const double* x = xs[it % 3].data();
    auto t0 = clk::now();
    nlp.eval_g(n, x, true, m, g.data());
    auto t1 = clk::now();
    nlp.eval_jac_g(n, x, false, m, nnz, nullptr, nullptr, jac_g.data());
    auto t2 = clk::now();
    e.EvalConstraintsAndJacobian(x, cg.data(), cv.data());
    std::copy(cg.begin(), cg.end(), g.begin());
    auto t3 = clk::now();
    std::copy(cv.begin(), cv.end(), jac_g.begin());
    auto t4 = clk::now();
    if (it >= 10) { t_pair.push_back(us(t0, t2)); t_jac.push_back(us(t1, t2)); t_old.push_back(us(t2, t4)); t_oldjac.push_back(us(t3, t4)); }
  }
  if (pg) e.UnregisterHost(cg.data());
  if (pv) e.UnregisterHost(cv.data());
  std::printf("zerocopy ok n=%d m=%d nnz=%d iters=%d path %s pair_us %.1f jac_us %.1f cached_pair_us %.1f cached_copy_us %.1f\n", n,
              m, nnz, iters, nlp.small_jacobian() ? "cached" : "device-kept", median(t_pair), median(t_jac), median(t_old), median(t_oldjac));
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: %s <anymal|biped|hopper> <out.bin> [device]\n", argv[0]); return 2; }
  const std::string cfg = argv[1];
  const int device = argc > 3 ? std::atoi(argv[3]) : -1;
  const bool zc = std::string(argv[2]) == "--zerocopy";
  NlpFormulation f = (cfg == "anymal" || cfg == "anymal_costs" || cfg == "anymal_rotvec" || cfg == "anymal_gait") ? AnymalTrot()
                     : (cfg == "biped" || cfg == "biped_next") ? BipedWalk() : MonopedHopper();
  if (cfg == "anymal_gait") {   // BASELINE configs[3]: stairs, phase-duration optimisation
    f.terrain_ = HeightMap::MakeTerrain(HeightMap::StairsID);
    f.params_.OptimizePhaseDurations();
  }
  if (cfg == "biped_next") {   // SURVEY §8(f) kinds: Torque, TerrainHard, EELinear (tests/configs.py)
    f.params_.constraints_.push_back(Parameters::Torque);
    f.params_.constraints_.push_back(Parameters::TerrainHard);
    Parameters::EELinearConstraintDef a, b;
    a.terms = {{0, 1, 1.0}, {1, 1, 1.0}};
    a.tolerance = 0.5;
    b.terms = {{0, 2, 0.5}, {1, 0, -1.0}, {0, 2, 0.5}};
    b.target = 1; b.deriv = 1; b.tolerance = 1.0; b.dt = 0.05;
    f.params_.ee_linear_constraints_ = {a, b};
  }
  if (cfg == "anymal_rotvec") f.params_.angular_rep_ = Parameters::RotationVector;
  if (cfg == "anymal_costs") {   // every cost kind (tests/configs.py _with_costs)
    f.params_.costs_ = {{Parameters::ForcesCostID, 1e-3}, {Parameters::EEMotionCostID, 0.5},
                        {Parameters::EnergyCostID, 1e-4}, {Parameters::AngMomCostID, 0.1}};
    f.params_.enable_swing_ee_base_pos_tracking = true;
  }
  try {
    const towr_problem_desc_t d = f.MakeDesc();
    if (zc) return zerocopy_check(d, device < 0 ? 0 : device, argc > 4 ? std::atoi(argv[4]) : 200);
    Engine e(d, device);
    NlpCallbacks nlp(e);
    int n = 0, m = 0, nnz = 0;
    nlp.get_nlp_info(n, m, nnz);
    std::vector<double> x = e.GetVariableValues();
    std::vector<int> iRow(nnz), jCol(nnz);
    if (!nlp.eval_jac_g(n, x.data(), true, m, nnz, iRow.data(), jCol.data(), nullptr)) { std::fprintf(stderr, "structure failed\n"); return 1; }
    FILE* fp = std::fopen(argv[2], "wb");
    if (!fp) return 1;
    std::fwrite(&d, sizeof(d), 1, fp);
    const int32_t nm[2] = {n, m};
    const int64_t nz = nnz;
    std::fwrite(nm, sizeof(nm), 1, fp);
    std::fwrite(&nz, sizeof(nz), 1, fp);
    std::fwrite(x.data(), sizeof(double), x.size(), fp);
    std::fwrite(iRow.data(), sizeof(int), iRow.size(), fp);
    std::fwrite(jCol.data(), sizeof(int), jCol.size(), fp);
    if (device >= 0) {
      std::vector<double> g(m), v(nnz), grad(n);
      double obj = 0.0;
      if (!nlp.eval_f(n, x.data(), true, obj) || !nlp.eval_grad_f(n, x.data(), false, grad.data()) ||
          !nlp.eval_g(n, x.data(), false, m, g.data()) ||
          !nlp.eval_jac_g(n, x.data(), false, m, nnz, nullptr, nullptr, v.data())) {
        std::fprintf(stderr, "evaluation failed: %s\n", towr_gpu_last_error(e.handle()));
        std::fclose(fp);
        return 1;
      }
      std::fwrite(g.data(), sizeof(double), g.size(), fp);
      std::fwrite(v.data(), sizeof(double), v.size(), fp);
      std::fwrite(&obj, sizeof(double), 1, fp);
      std::fwrite(grad.data(), sizeof(double), grad.size(), fp);
      // the trajectory export of x (SaveTrajectoryToCSV), to <out>.csv
      if (!SaveTrajectoryToCSV(e, x.data(), std::string(argv[2]) + ".csv", 0.01)) { std::fprintf(stderr, "csv export failed\n"); return 1; }
    }
    std::fclose(fp);
    std::printf("%s: n=%d m=%d nnz=%d%s\n", cfg.c_str(), n, m, nnz, device >= 0 ? " (evaluated on the GPU)" : " (layout only)");
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "error: %s\n", ex.what());
    return 1;
  }
  return 0;
}
