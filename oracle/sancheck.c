/* TEST INFRASTRUCTURE ONLY — AddressSanitizer / UndefinedBehaviorSanitizer driver of the CPU oracle
 * (tests/test_sanitizers.py). Reads a problem file written by the test:
 *   towr_problem_desc_t bytes | int32 n_data | n_data x (int32 kind, int32 index, int64 count, double[count])
 * and runs every oracle entry point at x0 and at a perturbed x. Built by `make sanitize`. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "towr_oracle.h"

static int rd(void* p, size_t n, FILE* f) { return fread(p, 1, n, f) == n; }

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s problem.bin\n", argv[0]); return 2; }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  towr_problem_desc_t d;
  int32_t nd = 0;
  if (!rd(&d, sizeof d, f) || !rd(&nd, sizeof nd, f) || nd < 0 || nd > 64) return 3;
  towr_data_t data[64];
  for (int i = 0; i < nd; ++i) {
    if (!rd(&data[i].kind, 4, f) || !rd(&data[i].index, 4, f) || !rd(&data[i].count, 8, f) || data[i].count < 0) return 3;
    double* v = (double*)malloc(sizeof(double) * (size_t)(data[i].count + 1));
    if (!rd(v, sizeof(double) * (size_t)data[i].count, f)) return 3;
    data[i].data = v;
  }
  fclose(f);
  char err[256];
  oracle_t* o = oracle_create_ex(&d, nd, data, err, sizeof err);
  if (!o) { fprintf(stderr, "create: %s\n", err); return 4; }
  int n = 0, m = 0;
  oracle_sizes(o, &n, &m);
  double* x = (double*)malloc(sizeof(double) * (size_t)n);
  double* g = (double*)malloc(sizeof(double) * (size_t)(m + 1));
  double* grad = (double*)malloc(sizeof(double) * (size_t)n);
  oracle_initial_x(o, x);
  unsigned s = 20261015u;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass) for (int j = 0; j < n; ++j) { s = s * 1664525u + 1013904223u; x[j] += 0.01 * ((double)(s >> 8) / (1 << 24) - 0.5); }
    oracle_eval_g(o, x, g);
    long nnz = oracle_eval_jac(o, x, 0, NULL, NULL, NULL);
    int* r = (int*)malloc(sizeof(int) * (size_t)(nnz + 1));
    int* c = (int*)malloc(sizeof(int) * (size_t)(nnz + 1));
    double* v = (double*)malloc(sizeof(double) * (size_t)(nnz + 1));
    oracle_eval_jac(o, x, nnz, r, c, v);
    oracle_eval_jac_values(o, x, v);
    double fv = 0.0;
    oracle_eval_f(o, x, &fv);
    oracle_eval_grad_f(o, x, grad);
    int ns = oracle_sample_trajectory(o, x, 0.05, NULL);
    double* tr = (double*)malloc(sizeof(double) * (size_t)(ns > 0 ? ns : 1) * (19 + 25 * d.robot.n_ee));
    oracle_sample_trajectory(o, x, 0.05, tr);
    free(tr); free(r); free(c); free(v);
  }
  oracle_destroy(o);
  free(x); free(g); free(grad);
  for (int i = 0; i < nd; ++i) free((void*)data[i].data);
  printf("ok n=%d m=%d\n", n, m);
  return 0;
}
