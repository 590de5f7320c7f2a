// towr_host_check — C++ host driver over the C-ABI, used by the tests (tests/test_cpp_host.py).
// It builds a BASELINE configuration through the C++ NlpFormulation mirror, creates the engine and
// walks the IPOPT callback sequence of one iteration:
//   get_nlp_info -> eval_jac_g(structure) -> eval_f(x, new_x = true) -> eval_grad_f(x, false)
//   -> eval_g(x, false) -> eval_jac_g(x, false)
// and dumps everything to a binary file:
//   desc bytes | n m (int32) nnz (int64) | x0[n] | iRow[nnz] jCol[nnz] | (device >= 0) g[m] values[nnz] f grad[n]
// and (device >= 0) the trajectory of x0 sampled at 0.01 s as SaveTrajectoryToCSV writes it, to <out.bin>.csv
// usage: towr_host_check <anymal|anymal_costs|anymal_rotvec|biped|biped_next|hopper> <out.bin> [device (default -1: layout only)]
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "nlp_formulation.hpp"
#include "towr_gpu.hpp"

using namespace towr_gpu;

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: %s <anymal|biped|hopper> <out.bin> [device]\n", argv[0]); return 2; }
  const std::string cfg = argv[1];
  const int device = argc > 3 ? std::atoi(argv[3]) : -1;
  NlpFormulation f = (cfg == "anymal" || cfg == "anymal_costs" || cfg == "anymal_rotvec") ? AnymalTrot() : (cfg == "biped" || cfg == "biped_next") ? BipedWalk() : MonopedHopper();
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
