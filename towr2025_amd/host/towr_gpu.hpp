// towr_gpu.hpp — C++ host side over the C-ABI (include/towr_gpu.h): what a towr/ifopt user calls.
//
// Engine     RAII owner of one towr_gpu handle. The names follow ifopt::Problem, which is what
//            IpoptAdapter reaches for this path (ifopt ≥ 2.0.1, external to the reference):
//              GetNumberOfOptimizationVariables / GetNumberOfConstraints / GetVariableValues,
//              EvalConstraints(x) -> g, EvalNonzerosOfJacobian(x) -> values, the Jacobian
//              structure in RowMajor (iRow, jCol) order.
// NlpCallbacks  the IPOPT TNLP callback subset of ifopt's IpoptAdapter for the hot path
//            (get_nlp_info / eval_f / eval_grad_f / eval_g / eval_jac_g) with Ipopt's argument
//            meaning: eval_jac_g with
//            values == nullptr fills the structure, otherwise the values, written by the device straight
//            into IPOPT's (page-locked) array; eval_g evaluates g alone unless the Jacobian came first at
//            that x (see the class comment).
//
// Error behaviour: construction failures throw std::runtime_error (the reference's
// NlpFormulation throws at setup, nlp_formulation.cc:396, 477-481); the callbacks return false on
// a runtime failure, which makes IPOPT stop with an evaluation error (ifopt's callbacks always
// return true, but it has no failure mode to report). There is no CPU path.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "towr_gpu.h"

namespace towr_gpu {

class Engine {
 public:
  // device < 0: layout-only (sizes, structure, x0; evaluation throws). `data`: side data of
  // towr_gpu_create_ex (LinearEqualityConstraint matrices, SoftConstraint bounds), copied at creation.
  Engine(const towr_problem_desc_t& desc, int device = 0, const std::vector<towr_data_t>& data = {}) {
    const int rc = towr_gpu_create_ex(&desc, (int32_t)data.size(), data.data(), device, &h_);
    if (rc != TOWR_OK) throw std::runtime_error("towr_gpu_create failed (" + std::to_string(rc) + "): " + towr_gpu_last_error(nullptr));
    int32_t n = 0, m = 0;
    int64_t nnz = 0;
    Check(towr_gpu_sizes(h_, &n, &m, &nnz));
    n_ = n; m_ = m; nnz_ = nnz;
  }
  ~Engine() { if (h_) towr_gpu_destroy(h_); }
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  int GetNumberOfOptimizationVariables() const { return n_; }
  int GetNumberOfConstraints() const { return m_; }
  int64_t GetNumberOfJacobianNonzeros() const { return nnz_; }

  std::vector<double> GetVariableValues() const {   // starting point x0
    std::vector<double> x(n_);
    Check(towr_gpu_initial_x(h_, x.data()));
    return x;
  }
  void GetJacobianStructure(int32_t* iRow, int32_t* jCol) const { Check(towr_gpu_jac_structure(h_, iRow, jCol)); }
  void EvalConstraints(const double* x, double* g) const { Check(towr_gpu_eval_g(h_, x, g)); }
  void EvalNonzerosOfJacobian(const double* x, double* values) const { Check(towr_gpu_eval_jac_values(h_, x, values)); }
  void EvalConstraintsAndJacobian(const double* x, double* g, double* values) const { Check(towr_gpu_eval_g_jac(h_, x, g, values)); }
  // g at x, with the Jacobian at x kept on the device; then the values at x from it (or evaluated, for another x)
  void EvalConstraintsKeepJacobian(const double* x, double* g) const { Check(towr_gpu_eval_g_keep_jac(h_, x, g)); }
  void EvalNonzerosOfJacobianKept(const double* x, double* values) const { Check(towr_gpu_eval_jac_values_kept(h_, x, values)); }
  // objective (ifopt Problem::EvaluateCostFunction) and its dense gradient
  double EvalCostFunction(const double* x) const { double f = 0.0; Check(towr_gpu_eval_f(h_, x, &f)); return f; }
  void EvalCostFunctionGradient(const double* x, double* grad) const { Check(towr_gpu_eval_grad_f(h_, x, grad)); }
  // trajectory samples (SaveTrajectoryToCSV's rows, include/towr_gpu.h), n_samples x n_cols
  std::vector<double> SampleTrajectory(const double* x, double T_sample, int* n_samples, int* n_cols) const {
    int32_t ns = 0, nc = 0;
    Check(towr_gpu_trajectory_size(h_, T_sample, &ns, &nc));
    std::vector<double> rows((size_t)ns * nc);
    Check(towr_gpu_sample_trajectory(h_, x, T_sample, rows.data()));
    if (n_samples) *n_samples = ns;
    if (n_cols) *n_cols = nc;
    return rows;
  }
  // B independent problems sharing this layout (host buffers, row-major B x n / m / nnz)
  void SetBatchTerrain(const std::vector<towr_terrain_t>& t) { Check(towr_gpu_set_batch_terrain(h_, (int32_t)t.size(), t.data())); }
  void EvalBatch(int B, const double* X, double* G, double* V) const { Check(towr_gpu_eval_batch(h_, B, X, G, V)); }
  // device-resident batch (HBM pointers), asynchronous on `stream` (hipStream_t, nullptr = default)
  int EvalBatchDevice(int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V, int64_t ldv, void* stream) const {
    return towr_gpu_eval_batch_device(h_, B, X, ldx, G, ldg, V, ldv, 1, 1, stream);
  }
  // page-lock caller memory for in-place host transfers (towr_gpu_register_host); returns the status
  int RegisterHost(void* p, size_t bytes) const { return towr_gpu_register_host(h_, p, (int64_t)bytes); }
  int UnregisterHost(void* p) const { return towr_gpu_unregister_host(h_, p); }
  towr_gpu_handle handle() const { return h_; }

 private:
  void Check(int rc) const {
    if (rc != TOWR_OK) throw std::runtime_error("towr_gpu error " + std::to_string(rc) + ": " + towr_gpu_last_error(h_));
  }
  towr_gpu_handle h_ = nullptr;
  int n_ = 0, m_ = 0;
  int64_t nnz_ = 0;
};

// The eval_f / eval_grad_f / eval_g / eval_jac_g callbacks of an IPOPT TNLP (Index = int,
// Number = double), as ifopt's IpoptAdapter implements them for towr, served by the engine.
//
// One evaluation per x. eval_g at a new x evaluates g AND the Jacobian into the engine's device staging
// (towr_gpu_eval_g_keep_jac) and returns g; eval_jac_g at that x then only moves the kept values into IPOPT's own
// `values` array (towr_gpu_eval_jac_values_kept: one DMA, in place, because the array is page-locked for the engine
// the first time it is seen), so no copy of the nnz values happens on the host (ifopt's IpoptAdapter copies its
// sparse matrix there, ipopt_adapter.cc; at nnz = 241,250 that copy took longer than the evaluation). The values
// are written into IPOPT's array only when IPOPT asks for them, and only for the x it asks about (the engine checks
// x bit for bit), so the array never holds values of an x it did not request (its adapter reuses the array without
// re-asking when the x tag it last evaluated matches). eval_jac_g first at a new x: one launch forms both, straight
// into IPOPT's array, and eval_g serves the cached g.
// IPOPT's TNLPAdapter passes the same array on every call (its jac_g_ member, allocated once per solve), so
// registration happens once per solve; when a different pointer or length arrives, the old one is unregistered and the
// new one registered. If registration fails (the range overlaps one already registered) the values go through the
// page-locked cache and a copy.
// A small Jacobian (below kSmallJacBytes, e.g. ANYmal with fixed phase durations: 225 kB) takes the round-4 path
// instead: eval_g evaluates both in one launch into the page-locked caches, eval_jac_g copies the cached values
// (MI355X, ANYmal, B = 1: 37.6 us per pair against 42.0 through the device staging; ANYmal gait, 1.93 MB of values:
// 92.4 us through the device staging against 148.6 cached and 111.5 for round 5's g-alone + zero-copy Jacobian).
// finalize_solution() is mandatory at the end of a solve (TNLP::finalize_solution; or destroy the callbacks): it
// unregisters IPOPT's array before IPOPT frees it. A solve whose integration does not forward finalize_solution
// would leave a registration of freed memory behind.
class NlpCallbacks {
 public:
  // Lifetime: the Engine must outlive these callbacks (declare the Engine first): the destructor
  // unregisters through the Engine's handle.
  static constexpr size_t kSmallJacBytes = 1u << 20;
  explicit NlpCallbacks(Engine& e)
      : e_(e), g_(e.GetNumberOfConstraints()), small_(e.GetNumberOfJacobianNonzeros() * sizeof(double) < kSmallJacBytes) {
    pin_g_ = !g_.empty() && e_.RegisterHost(g_.data(), g_.size() * sizeof(double)) == TOWR_OK;
  }
  ~NlpCallbacks() {
    ReleaseValues();
    if (pin_g_) e_.UnregisterHost(g_.data());
    if (pin_v_) e_.UnregisterHost(v_.data());
  }
  NlpCallbacks(const NlpCallbacks&) = delete;
  NlpCallbacks& operator=(const NlpCallbacks&) = delete;

  bool eval_f(int n, const double* x, bool new_x, double& obj_value) {
    if (n != e_.GetNumberOfOptimizationVariables()) return false;
    NewX(new_x);
    try { obj_value = e_.EvalCostFunction(x); } catch (const std::exception&) { return false; }
    return true;
  }
  bool eval_grad_f(int n, const double* x, bool new_x, double* grad_f) {
    if (n != e_.GetNumberOfOptimizationVariables()) return false;
    NewX(new_x);
    try { e_.EvalCostFunctionGradient(x, grad_f); } catch (const std::exception&) { return false; }
    return true;
  }

  bool get_nlp_info(int& n, int& m, int& nnz_jac_g) const {
    n = e_.GetNumberOfOptimizationVariables();
    m = e_.GetNumberOfConstraints();
    nnz_jac_g = (int)e_.GetNumberOfJacobianNonzeros();
    return true;
  }
  bool eval_g(int n, const double* x, bool new_x, int m, double* g) {
    if (n != e_.GetNumberOfOptimizationVariables() || m != e_.GetNumberOfConstraints()) return false;
    NewX(new_x);
    if (!g_valid_) {   // g, with the Jacobian kept for eval_jac_g at this x (on the device, or in the cache)
      try {
        if (small_) {
          CacheValues();
          e_.EvalConstraintsAndJacobian(x, g_.data(), v_.data());
          v_valid_ = true;
        } else {
          e_.EvalConstraintsKeepJacobian(x, g_.data());
        }
      } catch (const std::exception&) { return false; }
      g_valid_ = true;
    }
    for (int i = 0; i < m; ++i) g[i] = g_[i];
    return true;
  }
  bool eval_jac_g(int n, const double* x, bool new_x, int m, int nele_jac, int* iRow, int* jCol, double* values) {
    if (n != e_.GetNumberOfOptimizationVariables() || m != e_.GetNumberOfConstraints() ||
        nele_jac != (int)e_.GetNumberOfJacobianNonzeros())
      return false;
    if (values == nullptr) {   // structure (IPOPT asks once)
      try { e_.GetJacobianStructure(iRow, jCol); } catch (const std::exception&) { return false; }
      return true;
    }
    NewX(new_x);
    if (small_ && g_valid_ && v_valid_) {   // the cached values of this x
      for (int k = 0; k < nele_jac; ++k) values[k] = v_[k];
      return true;
    }
    double* dst = Values(values, nele_jac);   // IPOPT's array when registered, else the page-locked cache
    try {
      if (g_valid_) e_.EvalNonzerosOfJacobianKept(x, dst);   // the values eval_g kept (or evaluated, another x)
      else e_.EvalConstraintsAndJacobian(x, g_.data(), dst);   // first callback at this x: g comes along
    } catch (const std::exception&) { g_valid_ = false; return false; }
    g_valid_ = true;
    if (dst != values)
      for (int k = 0; k < nele_jac; ++k) values[k] = dst[k];
    return true;
  }
  // TNLP::finalize_solution: the solve is over, IPOPT's array is released
  void finalize_solution() { ReleaseValues(); }

  // introspection for tests: whether the last eval_jac_g wrote IPOPT's array directly, registrations so far
  bool values_zero_copy() const { return reg_ != nullptr; }
  bool small_jacobian() const { return small_; }   // the cached path (kSmallJacBytes)
  int values_registrations() const { return n_reg_; }

 private:
  // IPOPT's new_x == true on the first callback at a new x (whichever it is) invalidates the cached g (and values)
  void NewX(bool new_x) { if (new_x) g_valid_ = v_valid_ = false; }
  void CacheValues() {   // the page-locked values cache (small Jacobians, and the fallback of Values)
    const size_t nele = (size_t)e_.GetNumberOfJacobianNonzeros();
    if (v_.size() == nele) return;
    if (pin_v_) e_.UnregisterHost(v_.data());
    v_.assign(nele, 0.0);
    pin_v_ = nele > 0 && e_.RegisterHost(v_.data(), v_.size() * sizeof(double)) == TOWR_OK;
  }
  double* Values(double* values, int nele) {
    if (values == reg_ && nele == reg_n_) return values;
    ReleaseValues();
    if (nele > 0 && e_.RegisterHost(values, (size_t)nele * sizeof(double)) == TOWR_OK) {
      reg_ = values;
      reg_n_ = nele;
      ++n_reg_;
      return values;
    }
    if (v_.size() != (size_t)nele) {   // fallback: the page-locked cache and a copy
      if (pin_v_) e_.UnregisterHost(v_.data());
      v_.assign((size_t)nele, 0.0);
      pin_v_ = nele > 0 && e_.RegisterHost(v_.data(), v_.size() * sizeof(double)) == TOWR_OK;
    }
    return v_.data();
  }
  void ReleaseValues() {
    if (reg_) e_.UnregisterHost(reg_);
    reg_ = nullptr;
    reg_n_ = 0;
  }
  Engine& e_;
  std::vector<double> g_, v_;
  bool pin_g_ = false, pin_v_ = false;
  bool g_valid_ = false, v_valid_ = false;
  const bool small_;
  double* reg_ = nullptr;   // IPOPT's values array, registered (reg_n_ values)
  int reg_n_ = 0;
  int n_reg_ = 0;
};

// The CSV text of SaveTrajectoryToCSV (towr/src/utils/save_data.cpp:9-130): the reference's header,
// fixed notation with 6 decimals, is_contact_phase as 0/1.
inline bool WriteTrajectoryCSV(std::FILE* fp, const double* rows, int n_samples, int n_ee) {
  static const char* base[] = {"time", "base_pos_x", "base_pos_y", "base_pos_z", "base_vel_x", "base_vel_y", "base_vel_z",
                               "base_acc_x", "base_acc_y", "base_acc_z", "base_euler_roll", "base_euler_pitch",
                               "base_euler_yaw", "base_omega_x", "base_omega_y", "base_omega_z", "base_omegadot_x",
                               "base_omegadot_y", "base_omegadot_z"};
  static const char* ee[] = {"ee_pos_x_", "ee_pos_y_", "ee_pos_z_", "ee_vel_x_", "ee_vel_y_", "ee_vel_z_", "ee_acc_x_",
                             "ee_acc_y_", "ee_acc_z_", "ee_euler_roll_", "ee_euler_pitch_", "ee_euler_yaw_", "ee_omega_x_",
                             "ee_omega_y_", "ee_omega_z_", "ee_omegadot_x_", "ee_omegadot_y_", "ee_omegadot_z_",
                             "contact_force_x_", "contact_force_y_", "contact_force_z_", "contact_torque_x_",
                             "contact_torque_y_", "contact_torque_z_", "is_contact_phase_"};
  for (int c = 0; c < 19; ++c) std::fprintf(fp, c ? ",%s" : "%s", base[c]);
  for (int i = 0; i < n_ee; ++i)
    for (int c = 0; c < 25; ++c) std::fprintf(fp, ",%s%d", ee[c], i);
  std::fprintf(fp, "\n");
  const int cols = 19 + 25 * n_ee;
  for (int k = 0; k < n_samples; ++k) {
    const double* r = rows + (size_t)k * cols;
    for (int c = 0; c < cols; ++c) {
      const bool contact = c >= 19 && (c - 19) % 25 == 24;
      if (contact) std::fprintf(fp, ",%d", r[c] != 0.0 ? 1 : 0);
      else std::fprintf(fp, c ? ",%.6f" : "%.6f", r[c]);
    }
    std::fprintf(fp, "\n");
  }
  return std::ferror(fp) == 0;
}

// SaveTrajectoryToCSV(solution, filename, T_sample) for a solution vector x of the engine's problem
inline bool SaveTrajectoryToCSV(const Engine& e, const double* x, const std::string& filename, double T_sample = 0.001) {
  int ns = 0, nc = 0;
  const std::vector<double> rows = e.SampleTrajectory(x, T_sample, &ns, &nc);
  std::FILE* fp = std::fopen(filename.c_str(), "w");
  if (!fp) return false;
  const bool ok = WriteTrajectoryCSV(fp, rows.data(), ns, (nc - 19) / 25);
  return std::fclose(fp) == 0 && ok;
}

}  // namespace towr_gpu
