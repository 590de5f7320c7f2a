// TEST INFRASTRUCTURE ONLY — AddressSanitizer / UndefinedBehaviorSanitizer driver of the engine's host
// code (tests/test_sanitizers.py): the layout builder (towr2025_amd/csrc/layout.hip: variable maps, time
// grids, structure pass, CSR, tiles, slot tables, streaming tables, cost items) and the host instantiation
// of engine_math.h through the emulation (emu.hip), built host-only with the sanitizers. Input: the
// problem file format of oracle/sancheck.c. Built by `make sanitize`.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../towr2025_amd/csrc/layout.h"

extern "C" int emu_eval_ex(const towr_problem_desc_t* d, int n_data, const towr_data_t* data, const double* x, double* g,
                           double* v, char* err, int errlen);
extern "C" int emu_cost(const towr_problem_desc_t* d, const double* x, double* f, double* grad, char* err, int errlen);
extern "C" int emu_traj(const towr_problem_desc_t* d, const double* x, double dt, double* out, int max_rows);

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: %s problem.bin\n", argv[0]); return 2; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  towr_problem_desc_t d;
  int32_t nd = 0;
  if (std::fread(&d, sizeof d, 1, f) != 1 || std::fread(&nd, 4, 1, f) != 1 || nd < 0 || nd > 64) return 3;
  std::vector<towr_data_t> data((size_t)nd);
  std::vector<std::vector<double>> keep((size_t)nd);
  for (int i = 0; i < nd; ++i) {
    if (std::fread(&data[i].kind, 4, 1, f) != 1 || std::fread(&data[i].index, 4, 1, f) != 1 || std::fread(&data[i].count, 8, 1, f) != 1) return 3;
    keep[i].resize((size_t)data[i].count);
    if (data[i].count && std::fread(keep[i].data(), sizeof(double), (size_t)data[i].count, f) != (size_t)data[i].count) return 3;
    data[i].data = keep[i].data();
  }
  std::fclose(f);
  tg::Layout L;
  std::string err;
  if (int rc = tg::build_layout_ex(d, nd, data.data(), L, err)) { std::fprintf(stderr, "layout: %s\n", err.c_str()); return 4; }
  std::vector<double> x = L.x0, g((size_t)L.m + 1), v((size_t)L.nnz + 1), grad((size_t)L.n);
  char e[256];
  if (emu_eval_ex(&d, nd, data.data(), x.data(), g.data(), v.data(), e, sizeof e)) { std::fprintf(stderr, "emu: %s\n", e); return 5; }
  double fv = 0.0;
  if (d.n_costs && nd == 0 && emu_cost(&d, x.data(), &fv, grad.data(), e, sizeof e)) { std::fprintf(stderr, "cost: %s\n", e); return 6; }
  const int rows = emu_traj(&d, x.data(), 0.05, nullptr, 0);
  std::vector<double> tr((size_t)(rows > 0 ? rows : 1) * (19 + 25 * d.robot.n_ee));
  emu_traj(&d, x.data(), 0.05, tr.data(), rows);
  std::printf("ok n=%d m=%d nnz=%lld\n", L.n, L.m, (long long)L.nnz);
  return 0;
}
