/*
 * TEST INFRASTRUCTURE — part of the CPU oracle, never linked into the product.
 *
 * A minimal row-major sparse matrix that reproduces the STRUCTURAL semantics of
 * Eigen::SparseMatrix<double, Eigen::RowMajor> as the reference uses it
 * (towr/include/towr/variables/angular_converter.h:26-28, models/dynamic_model.h:74):
 *   - coeffRef() inserts an explicit entry even when the stored value is 0.0;
 *   - sparse +/- sparse keeps the union of both structures (no pruning of cancellations);
 *   - sparse * sparse is Eigen's "conservative" product: every structurally reachable entry is
 *     kept even if its value is 0.0;
 *   - dense.sparseView() drops exact zeros; dense.sparseView(1.0, -1.0) keeps every entry;
 *   - middleRows(r, k) = X replaces those rows by X's rows (structure included);
 *   - setFromTriplets sorts and sums duplicates (done in towr_oracle.c's assembly).
 * Entries of each row are kept sorted by column, as in compressed RowMajor storage.
 */
#ifndef TOWR_ORACLE_SPARSE_H_
#define TOWR_ORACLE_SPARSE_H_

typedef struct { int col; double val; } sp_ent;
typedef struct { int n, cap; sp_ent* e; } sp_row;
typedef struct { int rows, cols; sp_row* r; } spmat;

spmat   sp_zero(int rows, int cols);                 /* Jacobian(rows, cols): empty            */
void    sp_free(spmat* a);
spmat   sp_copy(const spmat* a);
double* sp_coeffref(spmat* a, int r, int c);         /* insert-if-absent, returns &value        */
spmat   sp_scale(const spmat* a, double s);          /* s * A (keeps structure)                 */
spmat   sp_lincomb(const spmat* a, double sa, const spmat* b, double sb); /* sa*A + sb*B, union  */
void    sp_add_inplace(spmat* dst, const spmat* src, double s);           /* dst += s*src        */
spmat   sp_mul(const spmat* a, const spmat* b);      /* conservative sparse*sparse product      */
spmat   sp_transpose(const spmat* a);
spmat   sp_from_dense(int rows, int cols, const double* rowmajor, int keep_zeros);
spmat   sp_row_of(const spmat* a, int r);            /* A.row(r) as 1 x cols                    */
void    sp_set_rows(spmat* dst, int row0, const spmat* src);  /* dst.middleRows(row0,k) = src  */
void    sp_set_row_from(spmat* dst, int row, const spmat* src1xn); /* dst.row(row) = src       */
void    sp_mul_vec(const spmat* a, const double* v, double* out);  /* dense result            */
long    sp_nnz(const spmat* a);

#endif
