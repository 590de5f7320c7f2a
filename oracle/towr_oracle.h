/*
 * TEST INFRASTRUCTURE ONLY — the CPU oracle for the eval_g / eval_jac_g path of hexb66/towr2025.
 *
 * A plain-C restatement of the reference algorithm (every function cites the reference file:line
 * it follows). It keeps the reference's algorithmic structure — per (constraint set x variable set
 * x instant) loops, O(n_set) column scans in NodeSpline::FillJacobianWrtNodes, linear
 * GetOptIndex searches, triplet-sorted Jacobian assembly — so that it is also an honest CPU
 * baseline ("port") for bench.py.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * (towr2025_amd/, libtowr_gpu.so) never links or calls it.
 *
 * Parity status: the reference cannot be built here (Eigen3, ifopt and Ipopt are absent) and its
 * own tests hold no golden vectors (towr/test/dynamic_constraint_test.cc:40-43 is an empty stub),
 * so this oracle is "parity unpinned" by the reference; it is pinned by sympy known-answer tests
 * and central finite differences (tests/test_oracle_*.py).
 */
#ifndef TOWR_ORACLE_H_
#define TOWR_ORACLE_H_

#include "../include/towr_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_s oracle_t;

oracle_t* oracle_create(const towr_problem_desc_t* desc, char* err, int errlen);
/* with side data (LinearEqualityConstraint M, SoftConstraint bounds), as towr_gpu_create_ex      */
oracle_t* oracle_create_ex(const towr_problem_desc_t* desc, int n_data, const towr_data_t* data, char* err, int errlen);
void      oracle_destroy(oracle_t* o);
int       oracle_sizes(oracle_t* o, int* n, int* m);
int       oracle_initial_x(oracle_t* o, double* x0);
/* ifopt Problem::EvalConstraints */
int       oracle_eval_g(oracle_t* o, const double* x, double* g);
/* ifopt Problem::GetJacobianOfConstraints at x: pattern AND values at x (row-major, sorted).
 * Returns nnz; fills at most cap triplets.                                                    */
long      oracle_eval_jac(oracle_t* o, const double* x, long cap, int* rows, int* cols, double* vals);
/* ifopt Problem::EvalNonzerosOfJacobian: values in the pattern order at x (nnz returned).      */
long      oracle_eval_jac_values(oracle_t* o, const double* x, double* values);
/* objective (sum of the cost terms) and its dense gradient */
int       oracle_eval_f(oracle_t* o, const double* x, double* f);
int       oracle_eval_grad_f(oracle_t* o, const double* x, double* grad);
int       oracle_sample_trajectory(oracle_t* o, const double* x, double dt, double* out);  /* rows, or -1 */
/* constraint-set row ranges: row0 / n_rows of constraint i                                      */
int       oracle_constraint_rows(oracle_t* o, int i, int* row0, int* n_rows);
int       oracle_varset_cols(oracle_t* o, int i, int* col0, int* n_cols);
/* Times `calls_per_thread` full calls (eval_g + eval_jac_g) per thread, one independent problem
 * instance per thread, cycling over nx pre-generated x vectors. Returns wall seconds.           */
double    oracle_bench(const towr_problem_desc_t* desc, int threads, int calls_per_thread,
                       int nx, const double* X, long* calls_done);

#ifdef __cplusplus
}
#endif

#endif
