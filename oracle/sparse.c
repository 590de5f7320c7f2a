/* TEST INFRASTRUCTURE — see sparse.h. Eigen structural semantics, plain C. */
#include "sparse.h"

#include <stdlib.h>
#include <string.h>

static void row_reserve(sp_row* r, int cap) {
  if (cap <= r->cap) return;
  int nc = r->cap ? r->cap : 4;
  while (nc < cap) nc *= 2;
  r->e = (sp_ent*)realloc(r->e, sizeof(sp_ent) * (size_t)nc);
  r->cap = nc;
}

spmat sp_zero(int rows, int cols) {
  spmat a;
  a.rows = rows; a.cols = cols;
  a.r = (sp_row*)calloc((size_t)(rows > 0 ? rows : 1), sizeof(sp_row));
  return a;
}

void sp_free(spmat* a) {
  if (!a->r) return;
  for (int i = 0; i < a->rows; ++i) free(a->r[i].e);
  free(a->r);
  a->r = NULL;
}

spmat sp_copy(const spmat* a) {
  spmat b = sp_zero(a->rows, a->cols);
  for (int i = 0; i < a->rows; ++i) {
    row_reserve(&b.r[i], a->r[i].n);
    if (a->r[i].n) memcpy(b.r[i].e, a->r[i].e, sizeof(sp_ent) * (size_t)a->r[i].n);
    b.r[i].n = a->r[i].n;
  }
  return b;
}

double* sp_coeffref(spmat* a, int r, int c) {
  sp_row* row = &a->r[r];
  int lo = 0, hi = row->n;
  while (lo < hi) { int mid = (lo + hi) / 2; if (row->e[mid].col < c) lo = mid + 1; else hi = mid; }
  if (lo < row->n && row->e[lo].col == c) return &row->e[lo].val;
  row_reserve(row, row->n + 1);
  memmove(&row->e[lo + 1], &row->e[lo], sizeof(sp_ent) * (size_t)(row->n - lo));
  row->e[lo].col = c; row->e[lo].val = 0.0;
  row->n++;
  return &row->e[lo].val;
}

spmat sp_scale(const spmat* a, double s) {
  spmat b = sp_copy(a);
  for (int i = 0; i < b.rows; ++i)
    for (int k = 0; k < b.r[i].n; ++k) b.r[i].e[k].val *= s;
  return b;
}

static void row_lincomb(const sp_row* x, double sx, const sp_row* y, double sy, sp_row* out) {
  out->n = 0;
  row_reserve(out, x->n + y->n);
  int i = 0, j = 0;
  while (i < x->n || j < y->n) {
    sp_ent e;
    if (j >= y->n || (i < x->n && x->e[i].col < y->e[j].col)) {
      e.col = x->e[i].col; e.val = sx * x->e[i].val; ++i;
    } else if (i >= x->n || y->e[j].col < x->e[i].col) {
      e.col = y->e[j].col; e.val = sy * y->e[j].val; ++j;
    } else {
      e.col = x->e[i].col; e.val = sx * x->e[i].val + sy * y->e[j].val; ++i; ++j;
    }
    out->e[out->n++] = e;
  }
}

spmat sp_lincomb(const spmat* a, double sa, const spmat* b, double sb) {
  spmat c = sp_zero(a->rows, a->cols);
  for (int i = 0; i < a->rows; ++i) row_lincomb(&a->r[i], sa, &b->r[i], sb, &c.r[i]);
  return c;
}

void sp_add_inplace(spmat* dst, const spmat* src, double s) {
  for (int i = 0; i < dst->rows; ++i) {
    sp_row out = {0, 0, NULL};
    row_lincomb(&dst->r[i], 1.0, &src->r[i], s, &out);
    free(dst->r[i].e);
    dst->r[i] = out;
  }
}

spmat sp_mul(const spmat* a, const spmat* b) {
  spmat c = sp_zero(a->rows, b->cols);
  double* acc = (double*)calloc((size_t)(b->cols > 0 ? b->cols : 1), sizeof(double));
  char* mask = (char*)calloc((size_t)(b->cols > 0 ? b->cols : 1), 1);
  int* idx = (int*)malloc(sizeof(int) * (size_t)(b->cols > 0 ? b->cols : 1));
  for (int i = 0; i < a->rows; ++i) {
    int nz = 0;
    for (int k = 0; k < a->r[i].n; ++k) {
      int kk = a->r[i].e[k].col; double av = a->r[i].e[k].val;
      const sp_row* br = &b->r[kk];
      for (int t = 0; t < br->n; ++t) {
        int j = br->e[t].col;
        if (!mask[j]) { mask[j] = 1; acc[j] = av * br->e[t].val; idx[nz++] = j; }
        else acc[j] += av * br->e[t].val;
      }
    }
    /* sorted insertion order (compressed row-major storage) */
    for (int p = 1; p < nz; ++p) { int v = idx[p], q = p - 1; while (q >= 0 && idx[q] > v) { idx[q + 1] = idx[q]; --q; } idx[q + 1] = v; }
    row_reserve(&c.r[i], nz);
    for (int p = 0; p < nz; ++p) { c.r[i].e[p].col = idx[p]; c.r[i].e[p].val = acc[idx[p]]; mask[idx[p]] = 0; }
    c.r[i].n = nz;
  }
  free(acc); free(mask); free(idx);
  return c;
}

spmat sp_transpose(const spmat* a) {
  spmat t = sp_zero(a->cols, a->rows);
  for (int i = 0; i < a->rows; ++i)
    for (int k = 0; k < a->r[i].n; ++k) {
      sp_row* row = &t.r[a->r[i].e[k].col];
      row_reserve(row, row->n + 1);
      row->e[row->n].col = i; row->e[row->n].val = a->r[i].e[k].val; row->n++;
    }
  return t;
}

spmat sp_from_dense(int rows, int cols, const double* d, int keep_zeros) {
  spmat a = sp_zero(rows, cols);
  for (int i = 0; i < rows; ++i) {
    row_reserve(&a.r[i], cols);
    for (int j = 0; j < cols; ++j) {
      double v = d[i * cols + j];
      /* sparseView(): !isMuchSmallerThan(v, 0, eps) <=> |v| > 0; sparseView(1,-1): always kept */
      if (keep_zeros || v != 0.0) { a.r[i].e[a.r[i].n].col = j; a.r[i].e[a.r[i].n].val = v; a.r[i].n++; }
    }
  }
  return a;
}

spmat sp_row_of(const spmat* a, int r) {
  spmat b = sp_zero(1, a->cols);
  row_reserve(&b.r[0], a->r[r].n);
  if (a->r[r].n) memcpy(b.r[0].e, a->r[r].e, sizeof(sp_ent) * (size_t)a->r[r].n);
  b.r[0].n = a->r[r].n;
  return b;
}

void sp_set_rows(spmat* dst, int row0, const spmat* src) {
  for (int i = 0; i < src->rows; ++i) {
    sp_row* d = &dst->r[row0 + i];
    d->n = 0;
    row_reserve(d, src->r[i].n);
    if (src->r[i].n) memcpy(d->e, src->r[i].e, sizeof(sp_ent) * (size_t)src->r[i].n);
    d->n = src->r[i].n;
  }
}

void sp_set_row_from(spmat* dst, int row, const spmat* src) { sp_set_rows(dst, row, src); }

void sp_mul_vec(const spmat* a, const double* v, double* out) {
  for (int i = 0; i < a->rows; ++i) {
    double s = 0.0;
    for (int k = 0; k < a->r[i].n; ++k) s += a->r[i].e[k].val * v[a->r[i].e[k].col];
    out[i] = s;
  }
}

long sp_nnz(const spmat* a) {
  long n = 0;
  for (int i = 0; i < a->rows; ++i) n += a->r[i].n;
  return n;
}
