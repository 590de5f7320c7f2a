/*
 * TEST INFRASTRUCTURE ONLY — CPU oracle / "port" baseline for the eval_g + eval_jac_g path of
 * hexb66/towr2025. See towr_oracle.h for the contract. Every function names the reference
 * function and file:line (relative to /root/reference/towr/) it restates. The product never links
 * this file.
 */
#include "towr_oracle.h"
#include "sparse.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { kPos = 0, kVel = 1, kAcc = 2 };           /* state.h:41 Dx                        */
enum { X = 0, Y = 1, Z = 2 };                    /* cartesian_dimensions.h:49             */
enum { AX = 0, AY, AZ, LX, LY, LZ };             /* cartesian_dimensions.h:59             */
enum { START = 0, END = 1 };                     /* nodes_variables.h:159 Side            */
#define MAXE TOWR_MAX_EE

/* =============================================================================================
 * CubicHermitePolynomial (src/helpers/polynomial.cc)
 * ===========================================================================================*/
typedef struct { double T; double n0[2][3], n1[2][3]; double c[4][3]; } Poly;

/* Polynomial::GetDerivativeWrtCoeff, polynomial.cc:61-72 */
static double poly_dwc(double t, int deriv, int c) {
  switch (deriv) {
    case kPos: return pow(t, c);
    case kVel: return c >= 1 ? c * pow(t, c - 1) : 0.0;
    case kAcc: return c >= 2 ? c * (c - 1) * pow(t, c - 2) : 0.0;
  }
  return 0.0;
}

/* Polynomial::GetPoint, polynomial.cc:47-58 -> out[deriv][dim] */
static void poly_get_point(const Poly* p, double t, double out[3][3]) {
  for (int d = 0; d < 3; ++d)
    for (int k = 0; k < 3; ++k) out[d][k] = 0.0;
  for (int d = 0; d < 3; ++d)
    for (int c = 0; c < 4; ++c) {
      double w = poly_dwc(t, d, c);
      for (int k = 0; k < 3; ++k) out[d][k] += w * p->c[c][k];
    }
}

/* CubicHermitePolynomial::UpdateCoeff, polynomial.cc:97-104 */
static void poly_update_coeff(Poly* p) {
  for (int k = 0; k < 3; ++k) {
    double p0 = p->n0[kPos][k], v0 = p->n0[kVel][k], p1 = p->n1[kPos][k], v1 = p->n1[kVel][k];
    p->c[0][k] = p0;
    p->c[1][k] = v0;
    p->c[2][k] = -(3 * (p0 - p1) + p->T * (2 * v0 + v1)) / pow(p->T, 2);
    p->c[3][k] = (2 * (p0 - p1) + p->T * (v0 + v1)) / pow(p->T, 3);
  }
}

/* polynomial.cc:135-214 : Get{Pos,Vel,Acc}WrtStartNode / EndNode */
static double poly_d_start(const Poly* p, int dfdt, int nd, double t) {
  double T = p->T, T2 = pow(T, 2), T3 = pow(T, 3), t2 = pow(t, 2), t3 = pow(t, 3);
  switch (dfdt) {
    case kPos: return nd == kPos ? (2 * t3) / T3 - (3 * t2) / T2 + 1 : t - (2 * t2) / T + t3 / T2;
    case kVel: return nd == kPos ? (6 * t2) / T3 - (6 * t) / T2 : (3 * t2) / T2 - (4 * t) / T + 1;
    case kAcc: return nd == kPos ? (12 * t) / T3 - 6 / T2 : (6 * t) / T2 - 4 / T;
  }
  return 0.0;
}
static double poly_d_end(const Poly* p, int dfdt, int nd, double t) {
  double T = p->T, T2 = pow(T, 2), T3 = pow(T, 3), t2 = pow(t, 2), t3 = pow(t, 3);
  switch (dfdt) {
    case kPos: return nd == kPos ? (3 * t2) / T2 - (2 * t3) / T3 : t3 / T2 - t2 / T;
    case kVel: return nd == kPos ? (6 * t) / T2 - (6 * t2) / T3 : (3 * t2) / T2 - (2 * t) / T;
    case kAcc: return nd == kPos ? 6 / T2 - (12 * t) / T3 : (6 * t) / T2 - 2 / T;
  }
  return 0.0;
}

/* CubicHermitePolynomial::GetDerivativeOfPosWrtDuration, polynomial.cc:236-257 */
static void poly_d_pos_wrt_duration(const Poly* p, double t, double out[3]) {
  double t2 = pow(t, 2), t3 = pow(t, 3), T = p->T, T2 = pow(T, 2), T3 = pow(T, 3), T4 = pow(T, 4);
  for (int k = 0; k < 3; ++k) {
    double x0 = p->n0[kPos][k], x1 = p->n1[kPos][k], v0 = p->n0[kVel][k], v1 = p->n1[kVel][k];
    out[k] = (t3 * (v0 + v1)) / T3 - (t2 * (2 * v0 + v1)) / T2
           - (3 * t3 * (2 * x0 - 2 * x1 + T * v0 + T * v1)) / T4
           + (2 * t2 * (3 * x0 - 3 * x1 + 2 * T * v0 + T * v1)) / T3;
  }
}

/* =============================================================================================
 * NodesVariables (src/variables/nodes_variables*.cc)
 * ===========================================================================================*/
typedef struct { int id, deriv, dim; } Nvi;
typedef struct { int phase, poly_in_phase, n_polys_in_phase, is_constant; } PolyInfo;
struct Spline;

typedef struct NodesVar {
  int kind, ee;
  int n_nodes;
  double (*nodes)[2][3];         /* nodes_[id].at(deriv)(dim)                                 */
  int n_rows;
  int all;                       /* NodesVariablesAll (computed GetNodeValuesInfo)           */
  int* nvi_n; Nvi (*nvi)[2];     /* index_to_node_value_info_ (phase-based)                  */
  int n_polys; PolyInfo* pinfo;  /* polynomial_info_                                          */
  struct Spline* obs[4]; int n_obs;
} NodesVar;

/* NodesVariablesAll::GetNodeValuesInfo, nodes_variables_all.cc:45-61 /
 * NodesVariablesPhaseBased::GetNodeValuesInfo, nodes_variables_phase_based.h:170-172 */
static int nv_info(const NodesVar* v, int idx, Nvi out[2]) {
  if (v->all) {
    int per = 2 * 3, internal = idx % per;
    out[0].deriv = internal < 3 ? kPos : kVel;
    out[0].dim = internal % 3;
    out[0].id = idx / per;
    return 1;
  }
  out[0] = v->nvi[idx][0];
  if (v->nvi_n[idx] > 1) out[1] = v->nvi[idx][1];
  return v->nvi_n[idx];
}

/* NodesVariables::GetOptIndex, nodes_variables.cc:44-54 (linear search, as the reference) */
static int nv_opt_index(const NodesVar* v, int id, int deriv, int dim) {
  Nvi l[2];
  for (int idx = 0; idx < v->n_rows; ++idx) {
    int n = nv_info(v, idx, l);
    for (int k = 0; k < n; ++k)
      if (l[k].id == id && l[k].deriv == deriv && l[k].dim == dim) return idx;
  }
  return -1;  /* NodeValueNotOptimized */
}

/* NodesVariables::GetValues, nodes_variables.cc:56-66 */
static void nv_get_values(const NodesVar* v, double* x) {
  Nvi l[2];
  for (int idx = 0; idx < v->n_rows; ++idx) {
    int n = nv_info(v, idx, l);
    for (int k = 0; k < n; ++k) x[idx] = v->nodes[l[k].id][l[k].deriv][l[k].dim];
  }
}

static void spline_update_nodes(struct Spline* s);

/* NodesVariables::SetVariables + UpdateObservers, nodes_variables.cc:68-83 */
static void nv_set_variables(NodesVar* v, const double* x) {
  Nvi l[2];
  for (int idx = 0; idx < v->n_rows; ++idx) {
    int n = nv_info(v, idx, l);
    for (int k = 0; k < n; ++k) v->nodes[l[k].id][l[k].deriv][l[k].dim] = x[idx];
  }
  for (int i = 0; i < v->n_obs; ++i) spline_update_nodes(v->obs[i]);
}

/* NodesVariables::SetByLinearInterpolation, nodes_variables.cc:131-154 */
static void nv_set_linear(NodesVar* v, const double ini[3], const double fin[3], double t_total) {
  double dp[3], avg[3];
  for (int k = 0; k < 3; ++k) { dp[k] = fin[k] - ini[k]; avg[k] = dp[k] / t_total; }
  Nvi l[2];
  for (int idx = 0; idx < v->n_rows; ++idx) {
    int n = nv_info(v, idx, l);
    for (int q = 0; q < n; ++q) {
      if (l[q].deriv == kPos) {
        double s = l[q].id / (double)(v->n_nodes - 1);
        v->nodes[l[q].id][kPos][l[q].dim] = ini[l[q].dim] + s * dp[l[q].dim];
      }
      if (l[q].deriv == kVel) v->nodes[l[q].id][kVel][l[q].dim] = avg[l[q].dim];
    }
  }
}

/* EulerConverter::GetRotationMatrixBaseToWorld(xyz), euler_converter.cc:207-221 (dense values) */
static void euler_R(const double xyz[3], double R[3][3]) {
  double x = xyz[X], y = xyz[Y], z = xyz[Z];
  R[0][0] = cos(y) * cos(z); R[0][1] = cos(z) * sin(x) * sin(y) - cos(x) * sin(z); R[0][2] = sin(x) * sin(z) + cos(x) * cos(z) * sin(y);
  R[1][0] = cos(y) * sin(z); R[1][1] = cos(x) * cos(z) + sin(x) * sin(y) * sin(z); R[1][2] = cos(x) * sin(y) * sin(z) - cos(z) * sin(x);
  R[2][0] = -sin(y);         R[2][1] = cos(y) * sin(x);                           R[2][2] = cos(x) * cos(y);
}

/* NodesVariables::SetByLinearInterpolationRelativeToBase, nodes_variables.cc:157-217 */
static void nv_set_linear_rel_base(NodesVar* v, const double ee0[3], const double ee1[3],
                                   const double b0[3], const double b1[3],
                                   const double rpy0[3], const double rpy1[3], double t_total) {
  int N = v->n_nodes;
  if (N < 2) return;
  double R0[3][3], RT[3][3], r0B[3], rTB[3], dpB[3], avgB[3], bavg[3], d0[3], dT[3];
  euler_R(rpy0, R0); euler_R(rpy1, RT);
  for (int k = 0; k < 3; ++k) { d0[k] = ee0[k] - b0[k]; dT[k] = ee1[k] - b1[k]; }
  for (int i = 0; i < 3; ++i) {
    r0B[i] = R0[0][i] * d0[0] + R0[1][i] * d0[1] + R0[2][i] * d0[2];
    rTB[i] = RT[0][i] * dT[0] + RT[1][i] * dT[1] + RT[2][i] * dT[2];
  }
  for (int k = 0; k < 3; ++k) { dpB[k] = rTB[k] - r0B[k]; avgB[k] = dpB[k] / t_total; bavg[k] = (b1[k] - b0[k]) / t_total; }
  Nvi l[2];
  for (int idx = 0; idx < v->n_rows; ++idx) {
    int n = nv_info(v, idx, l);
    for (int q = 0; q < n; ++q) {
      double a = l[q].id / (double)(N - 1), bp[3], rpy[3], R[3][3], rB[3];
      for (int k = 0; k < 3; ++k) {
        bp[k] = (1.0 - a) * b0[k] + a * b1[k];
        rpy[k] = (1.0 - a) * rpy0[k] + a * rpy1[k];
        rB[k] = r0B[k] + a * dpB[k];
      }
      euler_R(rpy, R);
      int d = l[q].dim;
      if (l[q].deriv == kPos)
        v->nodes[l[q].id][kPos][d] = bp[d] + (R[d][0] * rB[0] + R[d][1] * rB[1] + R[d][2] * rB[2]);
      if (l[q].deriv == kVel)
        v->nodes[l[q].id][kVel][d] = bavg[d] + (R[d][0] * avgB[0] + R[d][1] * avgB[1] + R[d][2] * avgB[2]);
    }
  }
  /* SetVariables(GetValues()) : harmonise shared (stance) node values */
  double* x = (double*)malloc(sizeof(double) * (size_t)v->n_rows);
  nv_get_values(v, x);
  nv_set_variables(v, x);
  free(x);
}

/* BuildPolyInfos, nodes_variables_phase_based.cc:39-59 */
static int build_poly_infos(int phase_count, int first_constant, int n_changing, PolyInfo* out) {
  int n = 0, c = first_constant;
  for (int i = 0; i < phase_count; ++i) {
    if (c) { out[n].phase = i; out[n].poly_in_phase = 0; out[n].n_polys_in_phase = 1; out[n].is_constant = 1; ++n; }
    else for (int j = 0; j < n_changing; ++j) {
      out[n].phase = i; out[n].poly_in_phase = j; out[n].n_polys_in_phase = n_changing; out[n].is_constant = 0; ++n;
    }
    c = !c;
  }
  return n;
}

/* GetAdjacentPolyIds / IsInConstantPhase / IsConstantNode, nodes_variables_phase_based.cc:101-183 */
static int nv_is_constant_node(const NodesVar* v, int node) {
  int last = v->n_nodes - 1;
  if (node == 0) return v->pinfo[0].is_constant;
  if (node == last) return v->pinfo[last - 1].is_constant;
  return v->pinfo[node - 1].is_constant || v->pinfo[node].is_constant;
}
/* GetPhase, :133-140 */
static int nv_get_phase(const NodesVar* v, int node) {
  int poly = (node == 0) ? 0 : (node == v->n_nodes - 1 ? v->n_nodes - 2 : node - 1);
  return v->pinfo[poly].phase;
}
/* GetPolyIDAtStartOfPhase / GetNodeIDAtStartOfPhase, :142-165 */
static int nv_node_at_start_of_phase(const NodesVar* v, int phase) {
  for (int i = 0; i < v->n_polys; ++i)
    if (v->pinfo[i].phase == phase) return i;  /* GetNodeId(poly, Start) = poly */
  return -1;
}

static void nv_alloc_map(NodesVar* v, int cap) {
  v->nvi_n = (int*)calloc((size_t)cap, sizeof(int));
  v->nvi = (Nvi(*)[2])calloc((size_t)cap, sizeof(Nvi[2]));
}
static void map_push(NodesVar* v, int idx, int id, int deriv, int dim) {
  Nvi e = {id, deriv, dim};
  v->nvi[idx][v->nvi_n[idx]++] = e;
}

/* NodesVariablesPhaseBased ctor (:61-73) + the four GetPhaseBasedEEParameterization (:201-396) */
static NodesVar* nv_phase_based(int kind, int ee, int phase_count, int contact_at_start, int n_changing) {
  NodesVar* v = (NodesVar*)calloc(1, sizeof(NodesVar));
  v->kind = kind; v->ee = ee;
  /* motion, ang: contact phase constant; force, torque: contact phase non-constant */
  int first_constant = (kind == TOWR_VAR_EE_MOTION || kind == TOWR_VAR_EE_ANG) ? contact_at_start : !contact_at_start;
  v->pinfo = (PolyInfo*)calloc((size_t)(phase_count * (n_changing + 1) + 1), sizeof(PolyInfo));
  v->n_polys = build_poly_infos(phase_count, first_constant, n_changing, v->pinfo);
  v->n_nodes = v->n_polys + 1;
  v->nodes = (double(*)[2][3])calloc((size_t)v->n_nodes, sizeof(double[2][3]));
  nv_alloc_map(v, v->n_nodes * 6 + 6);
  int idx = 0;
  for (int id = 0; id < v->n_nodes; ++id) {
    if (!nv_is_constant_node(v, id)) {
      for (int dim = 0; dim < 3; ++dim) {
        if (kind == TOWR_VAR_EE_MOTION) {          /* :223-237 */
          map_push(v, idx++, id, kPos, dim);
          if (dim == Z) v->nodes[id][kVel][Z] = 0.0;
          else map_push(v, idx++, id, kVel, dim);
        } else {                                   /* force :283-288, torque :329-333, ang :374-378 */
          map_push(v, idx++, id, kPos, dim);
          map_push(v, idx++, id, kVel, dim);
        }
      }
    } else {
      if (kind == TOWR_VAR_EE_MOTION || kind == TOWR_VAR_EE_ANG) {  /* :240-254, :381-392 */
        for (int k = 0; k < 3; ++k) { v->nodes[id][kVel][k] = 0.0; if (id + 1 < v->n_nodes) v->nodes[id + 1][kVel][k] = 0.0; }
        for (int dim = 0; dim < 3; ++dim) {
          map_push(v, idx, id, kPos, dim);
          map_push(v, idx, id + 1, kPos, dim);
          idx++;
        }
      } else {                                                     /* :290-300, :335-346 */
        for (int q = 0; q < 2; ++q) for (int k = 0; k < 3; ++k) if (id + 1 < v->n_nodes) { v->nodes[id][q][k] = 0.0; v->nodes[id + 1][q][k] = 0.0; }
      }
      id += 1;  /* already added next constant node, so skip */
    }
  }
  v->n_rows = idx;
  return v;
}

/* NodesVariablesAll ctor, nodes_variables_all.cc:34-43 */
static NodesVar* nv_all(int kind, int n_nodes) {
  NodesVar* v = (NodesVar*)calloc(1, sizeof(NodesVar));
  v->kind = kind; v->ee = 0; v->all = 1;
  v->n_nodes = n_nodes;
  v->nodes = (double(*)[2][3])calloc((size_t)n_nodes, sizeof(double[2][3]));
  v->n_rows = n_nodes * 2 * 3;
  return v;
}

/* ConvertPhaseToPolyDurations, nodes_variables_phase_based.cc:75-86 */
static void nv_phase_to_poly_durations(const NodesVar* v, const double* phase_d, double* out) {
  for (int i = 0; i < v->n_polys; ++i) out[i] = phase_d[v->pinfo[i].phase] / v->pinfo[i].n_polys_in_phase;
}

/* =============================================================================================
 * PhaseDurations (src/variables/phase_durations.cc)
 * ===========================================================================================*/
typedef struct PhaseDur {
  int ee, n;                 /* durations_.size()                                             */
  double d[TOWR_MAX_PHASES];
  double t_total;
  int initial_contact;
  struct Spline* obs[4]; int n_obs;
} PhaseDur;

static void spline_update_poly_durations(struct Spline* s);

/* PhaseDurations::SetVariables, phase_durations.cc:79-100 */
static void pd_set_variables(PhaseDur* p, const double* x) {
  double sum = 0.0;
  for (int i = 0; i < p->n - 1; ++i) { p->d[i] = x[i]; }
  for (int i = 0; i < p->n - 1; ++i) sum += x[i];  /* x.sum() */
  p->d[p->n - 1] = p->t_total - sum;
  for (int i = 0; i < p->n_obs; ++i) spline_update_poly_durations(p->obs[i]);
}

/* =============================================================================================
 * Spline / NodeSpline / PhaseSpline (src/helpers/spline.cc, node_spline.cc, phase_spline.cc)
 * ===========================================================================================*/
typedef struct Spline {
  NodesVar* nv;
  int n_polys;
  Poly* polys;
  PhaseDur* pd;      /* non-NULL: PhaseSpline                                                 */
  spmat jac_struct;  /* jac_wrt_nodes_structure_                                              */
} Spline;

static int g_segment_overflow = 0;

/* Spline::GetSegmentID, spline.cc:48-66 */
static int get_segment_id(double t_global, const double* d, int n) {
  double eps = 1e-10, t = 0;
  for (int i = 0; i < n; ++i) {
    t += d[i];
    if (t >= t_global - eps) return i;  /* at junctions, returns previous spline (=) */
  }
  g_segment_overflow++;
  return n - 1;  /* reference: assert(false), undefined in Release */
}

/* Spline::GetPolyDurations, spline.cc:108-116 */
static void spline_durations(const Spline* s, double* out) {
  for (int i = 0; i < s->n_polys; ++i) out[i] = s->polys[i].T;
}

/* Spline::GetLocalTime, spline.cc:68-78 */
static int spline_local_time(const Spline* s, double t_global, double* t_local) {
  double d[512];
  spline_durations(s, d);
  int id = get_segment_id(t_global, d, s->n_polys);
  double tl = t_global;
  for (int i = 0; i < id; i++) tl -= d[i];
  *t_local = tl;
  return id;
}

/* Spline::GetPoint, spline.cc:80-93 */
static void spline_point(const Spline* s, double t, double out[3][3]) {
  double tl; int id = spline_local_time(s, t, &tl);
  poly_get_point(&s->polys[id], tl, out);
}

/* NodeSpline::UpdateNodes, node_spline.cc:45-54 */
static void spline_update_nodes(Spline* s) {
  for (int i = 0; i < s->n_polys; ++i) {
    memcpy(s->polys[i].n0, s->nv->nodes[i], sizeof(double[2][3]));
    memcpy(s->polys[i].n1, s->nv->nodes[i + 1], sizeof(double[2][3]));
  }
  for (int i = 0; i < s->n_polys; ++i) poly_update_coeff(&s->polys[i]);
}

/* NodeSpline::FillJacobianWrtNodes, node_spline.cc:84-112 (O(n_set) scan, as the reference) */
static void spline_fill_jac(const Spline* s, int poly_id, double tl, int dxdt, spmat* jac, int zeros) {
  Nvi l[2];
  for (int idx = 0; idx < jac->cols; ++idx) {
    int n = nv_info(s->nv, idx, l);
    for (int q = 0; q < n; ++q)
      for (int side = START; side <= END; ++side) {
        int node = poly_id + side;
        if (node == l[q].id) {
          double val = side == START ? poly_d_start(&s->polys[poly_id], dxdt, l[q].deriv, tl)
                                     : poly_d_end(&s->polys[poly_id], dxdt, l[q].deriv, tl);
          if (zeros) val = 0.0;
          *sp_coeffref(jac, l[q].dim, idx) += val;
        }
      }
  }
}

/* NodeSpline::GetJacobianWrtNodes(id, t_local, dxdt), node_spline.cc:71-82 */
static spmat spline_jac_id(const Spline* s, int id, double tl, int dxdt) {
  spmat jac = sp_copy(&s->jac_struct);
  spline_fill_jac(s, id, tl, dxdt, &jac, 0);
  return jac;
}
/* NodeSpline::GetJacobianWrtNodes(t_global, dxdt), node_spline.cc:62-69 */
static spmat spline_jac(const Spline* s, double t, int dxdt) {
  double tl; int id = spline_local_time(s, t, &tl);
  return spline_jac_id(s, id, tl, dxdt);
}

/* PhaseSpline::UpdatePolynomialDurations, phase_spline.cc:54-65 */
static void spline_update_poly_durations(Spline* s) {
  double pdur[512];
  nv_phase_to_poly_durations(s->nv, s->pd->d, pdur);
  for (int i = 0; i < s->n_polys; ++i) s->polys[i].T = pdur[i];
  for (int i = 0; i < s->n_polys; ++i) poly_update_coeff(&s->polys[i]);
}

/* Spline ctor (spline.cc:36-46) + NodeSpline ctor (node_spline.cc:36-43) [+ PhaseSpline ctor,
 * phase_spline.cc:35-52, when pd != NULL] */
static Spline* spline_new(NodesVar* nv, const double* durations, PhaseDur* pd) {
  Spline* s = (Spline*)calloc(1, sizeof(Spline));
  s->nv = nv;
  s->n_polys = nv->n_nodes - 1;
  s->polys = (Poly*)calloc((size_t)s->n_polys, sizeof(Poly));
  for (int i = 0; i < s->n_polys; ++i) s->polys[i].T = durations[i];
  for (int i = 0; i < s->n_polys; ++i) poly_update_coeff(&s->polys[i]);
  nv->obs[nv->n_obs++] = s;     /* NodesObserver ctor registers (nodes_observer.cc:35-41) */
  spline_update_nodes(s);
  s->jac_struct = sp_zero(3, nv->n_rows);
  if (pd) {
    s->pd = pd;
    pd->obs[pd->n_obs++] = s;   /* PhaseDurationsObserver ctor (phase_durations_observer.cc:37-43) */
    spline_update_poly_durations(s);
    for (int i = 0; i < nv->n_polys; ++i) spline_fill_jac(s, i, 0.0, kPos, &s->jac_struct, 1);
  }
  return s;
}

/* PhaseSpline::GetDerivativeOfPosWrtPhaseDuration, phase_spline.cc:77-93 */
static void spline_d_pos_wrt_phase_duration(const Spline* s, double t, double out[3]) {
  double tl; int poly = spline_local_time(s, t, &tl);
  double st[3][3]; spline_point(s, t, st);
  double dxdT[3]; poly_d_pos_wrt_duration(&s->polys[poly], tl, dxdT);
  double inner = 1. / s->nv->pinfo[poly].n_polys_in_phase;
  double prev = s->nv->pinfo[poly].poly_in_phase;
  for (int k = 0; k < 3; ++k) out[k] = inner * (dxdT[k] - prev * st[kVel][k]);
}

/* PhaseDurations::GetJacobianOfPos, phase_durations.cc:126-154 */
static spmat pd_jac_of_pos(const PhaseDur* p, int current_phase, const double dxdT[3], const double xd[3]) {
  int cols = p->n - 1;
  double* J = (double*)calloc((size_t)(3 * (cols > 0 ? cols : 1)), sizeof(double));
  int last = (current_phase == p->n - 1);
  if (!last) for (int k = 0; k < 3; ++k) J[k * cols + current_phase] = dxdT[k];
  for (int ph = 0; ph < current_phase; ++ph) {
    for (int k = 0; k < 3; ++k) J[k * cols + ph] = -1 * xd[k];
    if (last) for (int k = 0; k < 3; ++k) J[k * cols + ph] -= dxdT[k];
  }
  spmat r = sp_from_dense(3, cols, J, 1);  /* sparseView(1.0, -1.0) */
  free(J);
  return r;
}

/* PhaseSpline::GetJacobianOfPosWrtDurations, phase_spline.cc:67-75 */
static spmat spline_jac_pos_wrt_durations(const Spline* s, double t) {
  double dxdT[3]; spline_d_pos_wrt_phase_duration(s, t, dxdT);
  double st[3][3]; spline_point(s, t, st);
  int phase = get_segment_id(t, s->pd->d, s->pd->n);
  return pd_jac_of_pos(s->pd, phase, dxdT, st[kVel]);
}

/* =============================================================================================
 * HeightMap (src/terrain/height_map.cc, height_map_examples.cc, height_map_examples.h)
 * ===========================================================================================*/
typedef towr_terrain_t Terrain;
static double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static double ter_h(const Terrain* T, double x, double y) {
  const double* p = T->p;
  switch (T->id) {
    case TOWR_TERRAIN_FLAT: return p[0];
    case TOWR_TERRAIN_BLOCK: {           /* Block::GetHeight, height_map_examples.cc:41-53 */
      double bs = p[0], len = p[1], hh = p[2], eps = p[3], slope = hh / eps, h = 0.0;
      if (bs <= x && x <= bs + eps) h = slope * (x - bs);
      if (bs + eps <= x && x <= bs + len) h = hh;
      return h;
    }
    case TOWR_TERRAIN_STAIRS: {          /* Stairs::GetHeight, :70-84 */
      double h = 0.0;
      if (x >= p[0]) h = p[2];
      if (x >= p[0] + p[1]) h = p[3];
      if (x >= p[0] + p[1] + p[4]) h = 0.0;
      return h;
    }
    case TOWR_TERRAIN_GAP: {             /* Gap::GetHeight, :89-98 ; constants height_map_examples.h:96-111 */
      double gs = p[0], w = p[1], hh = p[2], dx = w / 2.0, xc = gs + dx, ge = gs + w;
      double a = (4 * hh) / (w * w), b = -(8 * hh * xc) / (w * w), c = -(hh * (w - 2 * xc) * (w + 2 * xc)) / (w * w);
      double h = 0.0;
      if (gs <= x && x <= ge) h = a * x * x + b * x + c;
      return h;
    }
    case TOWR_TERRAIN_SLOPE: {           /* Slope::GetHeight, :125-141 */
      double ss = p[0], xd = ss + p[1], xf = xd + p[2], hc = p[3], slope = hc / p[1], z = 0.0;
      if (x >= ss) z = slope * (x - ss);
      if (x >= xd) z = hc - slope * (x - xd);
      if (x >= xf) z = 0.0;
      return z;
    }
    case TOWR_TERRAIN_CHIMNEY: {         /* Chimney::GetHeight, :162-170 */
      double z = 0.0;
      if (p[0] <= x && x <= p[0] + p[1]) z = p[3] * (y - p[2]);
      return z;
    }
    case TOWR_TERRAIN_CHIMNEY_LR: {      /* ChimneyLR::GetHeight, :186-197 */
      double z = 0.0, e1 = p[0] + p[1], e2 = p[0] + 2 * p[1];
      if (p[0] <= x && x <= e1) z = p[3] * (y - p[2]);
      if (e1 <= x && x <= e2) z = -p[3] * (y + p[2]);
      return z;
    }
    case TOWR_TERRAIN_STEPS: {           /* FiveStepStairs::GetHeight, test/hopper_example.cc:62-79 */
      if (x < p[0]) return 0.0;
      double rel = x - p[0];
      int step = (int)(rel / p[1]);
      if (step >= (int)p[3]) return p[3] * p[2];
      return (step + 1) * p[2];
    }
  }
  return 0.0;
}

static double ter_dx(const Terrain* T, double x, double y) {
  const double* p = T->p;
  (void)y;
  switch (T->id) {
    case TOWR_TERRAIN_BLOCK: { double bs = p[0], eps = p[3]; return (bs <= x && x <= bs + eps) ? p[2] / eps : 0.0; }
    case TOWR_TERRAIN_GAP: {
      double gs = p[0], w = p[1], hh = p[2], xc = gs + w / 2.0, ge = gs + w;
      double a = (4 * hh) / (w * w), b = -(8 * hh * xc) / (w * w);
      return (gs <= x && x <= ge) ? 2 * a * x + b : 0.0;
    }
    case TOWR_TERRAIN_SLOPE: {
      double ss = p[0], xd = ss + p[1], xf = xd + p[2], slope = p[3] / p[1], d = 0.0;
      if (x >= ss) d = slope;
      if (x >= xd) d = -slope;
      if (x >= xf) d = 0.0;
      return d;
    }
  }
  return 0.0;
}
static double ter_dy(const Terrain* T, double x, double y) {
  const double* p = T->p;
  (void)y;
  switch (T->id) {
    case TOWR_TERRAIN_CHIMNEY: return (p[0] <= x && x <= p[0] + p[1]) ? p[3] : 0.0;
    case TOWR_TERRAIN_CHIMNEY_LR: {
      double e1 = p[0] + p[1], e2 = p[0] + 2 * p[1], d = 0.0;
      if (p[0] <= x && x <= e1) d = p[3];
      if (e1 <= x && x <= e2) d = -p[3];
      return d;
    }
  }
  return 0.0;
}
static double ter_dxx(const Terrain* T, double x, double y) {
  (void)y;
  if (T->id == TOWR_TERRAIN_GAP) {
    double gs = T->p[0], w = T->p[1], hh = T->p[2], ge = gs + w, a = (4 * hh) / (w * w);
    return (gs <= x && x <= ge) ? 2 * a : 0.0;
  }
  return 0.0;
}
/* HeightMap::GetDerivativeOfHeightWrt, height_map.cc:52-60 */
static double ter_dh(const Terrain* T, int dim, double x, double y) { return dim == X ? ter_dx(T, x, y) : ter_dy(T, x, y); }
/* HeightMap::GetSecondDerivativeOfHeightWrt, height_map.cc:150-163 (XY/YX/YY default 0) */
static double ter_d2h(const Terrain* T, int d1, int d2, double x, double y) {
  if (d1 == X && d2 == X) return ter_dxx(T, x, y);
  return 0.0;
}

enum { NORMAL = 0, TANGENT1 = 1, TANGENT2 = 2 };

/* HeightMap::GetBasis / GetNormal / GetTangent1 / GetTangent2, height_map.cc:68-139.
 * deriv < 0: basis requested; else derivative w.r.t. dim `deriv`.                              */
static void ter_basis(const Terrain* T, int basis, double x, double y, int deriv, double v[3]) {
  int req = deriv < 0;
  switch (basis) {
    case NORMAL:
      for (int d = X; d <= Y; ++d) v[d] = req ? -ter_dh(T, d, x, y) : -ter_d2h(T, d, deriv, x, y);
      v[Z] = req ? 1.0 : 0.0;
      break;
    case TANGENT1:
      v[X] = req ? 1.0 : 0.0; v[Y] = 0.0;
      v[Z] = req ? ter_dh(T, X, x, y) : ter_d2h(T, X, deriv, x, y);
      break;
    case TANGENT2:
      v[X] = 0.0; v[Y] = req ? 1.0 : 0.0;
      v[Z] = req ? ter_dh(T, Y, x, y) : ter_d2h(T, Y, deriv, x, y);
      break;
  }
}

/* Eigen normalized(): v / sqrt(|v|^2) if |v|^2 > 0 */
static void normalized(const double v[3], double o[3]) {
  double z = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  if (z > 0) { double s = sqrt(z); for (int k = 0; k < 3; ++k) o[k] = v[k] / s; }
  else for (int k = 0; k < 3; ++k) o[k] = v[k];
}

/* HeightMap::GetNormalizedBasis, height_map.cc:62-66 */
static void ter_nbasis(const Terrain* T, int basis, double x, double y, double o[3]) {
  double v[3]; ter_basis(T, basis, x, y, -1, v); normalized(v, o);
}

/* HeightMap::GetDerivativeOfNormalizedBasisWrt, height_map.cc:80-91, 141-148 */
static void ter_d_nbasis(const Terrain* T, int basis, int dim, double x, double y, double o[3]) {
  double dv[3], v[3], vn[3];
  ter_basis(T, basis, x, y, dim, dv);
  ter_basis(T, basis, x, y, -1, v);
  double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2], nrm = sqrt(sq);
  normalized(v, vn);
  for (int k = 0; k < 3; ++k) {
    double u = (k == dim) ? 1.0 : 0.0;
    double dn = 1 / sq * (nrm * u - v[dim] * vn[k]);
    o[k] = dn * dv[k];
  }
}

/* =============================================================================================
 * EulerConverter (src/helpers/euler_converter.cc)
 * ===========================================================================================*/
typedef struct { const Spline* euler; spmat jac_struct; int rotvec; } Euler;   /* rotvec: RotVecConverter */

/* ---------------------------------------------------------------------------------------------
 * RotVecConverter (src/helpers/rotvec_converter.cc; Parameters::RotationVector, parameters.h:334):
 * the base angular spline holds a rotation vector theta; R = exp([theta]x) (Rodrigues),
 * omega = J_L(theta) theta_dot, omega_dot = J_L_dot theta_dot + J_L theta_ddot. The Jacobians keep
 * the reference's structure: DenseTimesSparse (every row for each active column) followed by
 * EnsureFullPattern (all 3 rows of every column active in d pos / d vel).
 * -------------------------------------------------------------------------------------------*/
#define RV_EPS 1e-10   /* kEps, :10 */
typedef struct { double alpha, beta, gamma, dalpha, dbeta, dgamma; } RvCoeffs;

static double rv_norm(const double v[3]) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

/* ComputeCoeffs, :30-59 */
static RvCoeffs rv_coeffs(double theta) {
  RvCoeffs c;
  double t2 = theta * theta;
  if (theta < RV_EPS) {
    c.alpha = 1.0 - t2 / 6.0; c.beta = 1.0 / 6.0 - t2 / 120.0; c.gamma = 0.5 - t2 / 24.0;
    c.dalpha = -theta / 3.0; c.dbeta = -theta / 60.0; c.dgamma = -theta / 12.0;
  } else {
    double st = sin(theta), ct = cos(theta), t3 = t2 * theta, t4 = t3 * theta;
    c.alpha = st / theta; c.beta = (theta - st) / t3; c.gamma = (1.0 - ct) / t2;
    c.dalpha = (theta * ct - st) / t2;
    c.dbeta = (-2.0 * theta - theta * ct + 3.0 * st) / t4;
    c.dgamma = (theta * st - 2.0 + 2.0 * ct) / t3;
  }
  return c;
}
/* Skew, :20-28 */
static void rv_skew(const double v[3], double S[3][3]) {
  S[0][0] = 0;     S[0][1] = -v[2]; S[0][2] = v[1];
  S[1][0] = v[2];  S[1][1] = 0;     S[1][2] = -v[0];
  S[2][0] = -v[1]; S[2][1] = v[0];  S[2][2] = 0;
}
static void m3_mul(const double A[3][3], const double B[3][3], double C[3][3]) {
  double T[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
  memcpy(C, T, sizeof T);
}
static void m3_vec(const double A[3][3], const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = A[i][0] * v[0] + A[i][1] * v[1] + A[i][2] * v[2];
}
/* Rodrigues, :61-72 */
static void rv_rodrigues(const double rv[3], double R[3][3]) {
  double theta = rv_norm(rv), K[3][3];
  rv_skew(rv, K);
  if (theta < RV_EPS) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) R[i][j] = (i == j ? 1.0 : 0.0) + K[i][j];
    return;
  }
  double s = sin(theta) / theta, h = (1.0 - cos(theta)) / (theta * theta), KK[3][3];
  m3_mul(K, K, KK);
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + s * K[i][j]) + h * KK[i][j];
}
/* LeftJacobian, :74-85 */
static void rv_left_jac(const double rv[3], double J[3][3]) {
  double theta = rv_norm(rv), S[3][3];
  rv_skew(rv, S);
  if (theta < RV_EPS) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) J[i][j] = (i == j ? 1.0 : 0.0) + 0.5 * S[i][j];
    return;
  }
  RvCoeffs c = rv_coeffs(theta);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) J[i][j] = (c.alpha * (i == j ? 1.0 : 0.0) + c.beta * (rv[i] * rv[j])) + c.gamma * S[i][j];
}
/* LeftJacobianDot, :87-107 */
static void rv_left_jac_dot(const double rv[3], const double rvd[3], double J[3][3]) {
  double theta = rv_norm(rv), S[3][3], Sd[3][3];
  rv_skew(rv, S); rv_skew(rvd, Sd);
  if (theta < RV_EPS) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) J[i][j] = 0.5 * Sd[i][j];
    return;
  }
  RvCoeffs c = rv_coeffs(theta);
  double theta_dot = (rv[0] * rvd[0] + rv[1] * rvd[1] + rv[2] * rvd[2]) / theta;
  double ad = c.dalpha * theta_dot, bd = c.dbeta * theta_dot, gd = c.dgamma * theta_dot;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      J[i][j] = (((ad * (i == j ? 1.0 : 0.0) + bd * (rv[i] * rv[j])) + c.beta * (rvd[i] * rv[j] + rv[i] * rvd[j])) + gd * S[i][j]) + c.gamma * Sd[i][j];
}
static void rv_R_t(const Euler* e, double t, double R[3][3]) {   /* GetRotationMatrixBaseToWorld, :118-123 */
  double st[3][3]; spline_point(e->euler, t, st);
  rv_rodrigues(st[kPos], R);
}
static void rv_omega(const Euler* e, double t, double w[3]) {   /* GetAngularVelocityInWorld, :125-130 */
  double st[3][3], J[3][3]; spline_point(e->euler, t, st);
  rv_left_jac(st[kPos], J); m3_vec(J, st[kVel], w);
}
static void rv_omega_dot(const Euler* e, double t, double wd[3]) {   /* GetAngularAccelerationInWorld, :132-138 */
  double st[3][3], J[3][3], Jd[3][3], a[3], b[3]; spline_point(e->euler, t, st);
  rv_left_jac_dot(st[kPos], st[kVel], Jd); rv_left_jac(st[kPos], J);
  m3_vec(Jd, st[kVel], a); m3_vec(J, st[kAcc], b);
  for (int k = 0; k < 3; ++k) wd[k] = a[k] + b[k];
}
/* DenseTimesSparse, :148-174: all 3 rows for every column active in B */
static spmat rv_dense_times_sparse(const double A[3][3], const spmat* B) {
  int n = B->cols;
  char* act = (char*)calloc((size_t)n + 1, 1);
  for (int r = 0; r < B->rows; ++r) for (int q = 0; q < B->r[r].n; ++q) act[B->r[r].e[q].col] = 1;
  spmat out = sp_zero(3, n);
  for (int col = 0; col < n; ++col) {
    if (!act[col]) continue;
    double bc[3] = {0, 0, 0};
    for (int r = 0; r < 3; ++r)
      for (int q = 0; q < B->r[r].n; ++q) if (B->r[r].e[q].col == col) bc[r] = B->r[r].e[q].val;
    double rc[3]; m3_vec(A, bc, rc);
    for (int r = 0; r < 3; ++r) *sp_coeffref(&out, r, col) = rc[r];
  }
  free(act);
  return out;
}
/* EnsureFullPattern, :176-208 */
static void rv_full_pattern(const Euler* e, double t, spmat* J) {
  spmat jp = spline_jac(e->euler, t, kPos), jv = spline_jac(e->euler, t, kVel);
  int n = J->cols;
  char* act = (char*)calloc((size_t)n + 1, 1);
  for (int r = 0; r < 3; ++r) {
    for (int q = 0; q < jp.r[r].n; ++q) act[jp.r[r].e[q].col] = 1;
    for (int q = 0; q < jv.r[r].n; ++q) act[jv.r[r].e[q].col] = 1;
  }
  for (int r = 0; r < J->rows; ++r) for (int q = 0; q < J->r[r].n; ++q) act[J->r[r].e[q].col] = 1;
  for (int c = 0; c < n; ++c)
    if (act[c]) for (int r = 0; r < 3; ++r) (void)sp_coeffref(J, r, c);   /* existing value or 0 */
  free(act); sp_free(&jp); sp_free(&jv);
}
/* DerivOfRotVecMult, :210-233: d(R v)/dtheta = -[R v]x J_L, d(R^T v)/dtheta = R^T [v]x J_L */
static spmat rv_d_rotvec(const Euler* e, double t, const double v[3], int inverse) {
  double st[3][3], R[3][3], JL[3][3], A[3][3], S[3][3];
  spline_point(e->euler, t, st);
  rv_rodrigues(st[kPos], R); rv_left_jac(st[kPos], JL);
  spmat jac_pos = spline_jac(e->euler, t, kPos);
  if (inverse) {
    double Rt[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Rt[i][j] = R[j][i];
    rv_skew(v, S); m3_mul(Rt, S, A); m3_mul(A, JL, A);
  } else {
    double Rv[3]; m3_vec(R, v, Rv);
    rv_skew(Rv, S);
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) S[i][j] = -S[i][j];
    m3_mul(S, JL, A);
  }
  spmat res = rv_dense_times_sparse(A, &jac_pos);
  rv_full_pattern(e, t, &res);
  sp_free(&jac_pos);
  return res;
}
static void rv_row_add(spmat* res, int j, const spmat* row1xn, double s) {   /* result.row(j) += s * row */
  spmat cur = sp_row_of(res, j);
  sp_add_inplace(&cur, row1xn, s);
  sp_set_row_from(res, j, &cur);
  sp_free(&cur);
}
/* Levi-Civita sign of the skew entry (dim, j): [theta]x_{dim,j} = sign * theta_k, k = 3 - dim - j */
static double rv_sign(int dim, int j) { return ((j - dim + 3) % 3 == 1) ? -1.0 : 1.0; }

/* GetDerivJLwrtNodes, :235-325: result.row(j) = d(J_L[dim][j]) / d nodes */
static spmat rv_dJL(const Euler* e, double t, int dim) {
  double st[3][3]; spline_point(e->euler, t, st);
  const double* rv = st[kPos];
  double theta = rv_norm(rv);
  RvCoeffs c = rv_coeffs(theta);
  spmat jac_pos = spline_jac(e->euler, t, kPos);
  int n = jac_pos.cols;
  spmat result = sp_copy(&e->jac_struct);
  spmat pr[3];
  for (int l = 0; l < 3; ++l) pr[l] = sp_row_of(&jac_pos, l);
  spmat da = sp_zero(1, n), db = sp_zero(1, n), dg = sp_zero(1, n);
  if (theta >= RV_EPS) {
    double inv = 1.0 / theta;
    spmat tj = sp_zero(1, n);
    for (int l = 0; l < 3; ++l) if (fabs(rv[l]) > 1e-15) sp_add_inplace(&tj, &pr[l], rv[l] * inv);
    sp_free(&da); sp_free(&db); sp_free(&dg);
    da = sp_scale(&tj, c.dalpha); db = sp_scale(&tj, c.dbeta); dg = sp_scale(&tj, c.dgamma);
    sp_free(&tj);
  }
  double Sk[3][3]; rv_skew(rv, Sk);
  for (int j = 0; j < 3; ++j) {
    if (dim == j) rv_row_add(&result, j, &da, 1.0);
    double rvdj = rv[dim] * rv[j];
    if (fabs(rvdj) > 1e-15) rv_row_add(&result, j, &db, rvdj);
    if (fabs(c.beta) > 1e-15) {
      if (fabs(rv[j]) > 1e-15) rv_row_add(&result, j, &pr[dim], c.beta * rv[j]);
      if (fabs(rv[dim]) > 1e-15) rv_row_add(&result, j, &pr[j], c.beta * rv[dim]);
    }
    double sk = Sk[dim][j];
    if (fabs(sk) > 1e-15) rv_row_add(&result, j, &dg, sk);
    if (fabs(c.gamma) > 1e-15 && dim != j) rv_row_add(&result, j, &pr[3 - dim - j], c.gamma * rv_sign(dim, j));
  }
  for (int l = 0; l < 3; ++l) sp_free(&pr[l]);
  sp_free(&da); sp_free(&db); sp_free(&dg); sp_free(&jac_pos);
  return result;
}

/* GetDerivJLdotwrtNodes, :327-506: result.row(j) = d(J_L_dot[dim][j]) / d nodes */
static spmat rv_dJLdot(const Euler* e, double t, int dim) {
  double st[3][3]; spline_point(e->euler, t, st);
  const double *rv = st[kPos], *rvd = st[kVel];
  double theta = rv_norm(rv);
  RvCoeffs c = rv_coeffs(theta);
  spmat jac_pos = spline_jac(e->euler, t, kPos), jac_vel = spline_jac(e->euler, t, kVel);
  int n = jac_pos.cols;
  spmat result = sp_copy(&e->jac_struct);
  spmat pr[3], vr[3];
  for (int l = 0; l < 3; ++l) { pr[l] = sp_row_of(&jac_pos, l); vr[l] = sp_row_of(&jac_vel, l); }
  double theta_dot = 0.0;
  if (theta > RV_EPS) theta_dot = (rv[0] * rvd[0] + rv[1] * rvd[1] + rv[2] * rvd[2]) / theta;
  double beta_dot = c.dbeta * theta_dot, gamma_dot = c.dgamma * theta_dot;
  spmat dad = sp_zero(1, n), dbd = sp_zero(1, n), dgd = sp_zero(1, n);
  spmat nhat = sp_zero(1, n);   /* n_hat^T jac_pos (theta > eps only) */
  if (theta > RV_EPS) {
    double inv = 1.0 / theta, t2 = theta * theta;
    spmat dtd = sp_zero(1, n);
    for (int l = 0; l < 3; ++l) { sp_add_inplace(&dtd, &pr[l], rvd[l] * inv); sp_add_inplace(&dtd, &vr[l], rv[l] * inv); }
    for (int l = 0; l < 3; ++l) sp_add_inplace(&nhat, &pr[l], rv[l] * inv);
    sp_add_inplace(&dtd, &nhat, -(theta_dot * inv));
    double st_ = sin(theta), ct = cos(theta);
    double alpha_pp = (-theta * st_ - 2.0 * (theta * ct - st_) / theta) / t2;
    double beta_pp, gamma_pp;
    { double num = -2.0 * theta - theta * ct + 3.0 * st_, dnum = -2.0 - ct + theta * st_ + 3.0 * ct, t4 = t2 * t2;
      beta_pp = (dnum - 4.0 * num / theta) / t4; }
    { double num = theta * st_ - 2.0 + 2.0 * ct, dnum = st_ + theta * ct - 2.0 * st_, t3 = t2 * theta;
      gamma_pp = (dnum - 3.0 * num / theta) / t3; }
    sp_free(&dad); sp_free(&dbd); sp_free(&dgd);
    dad = sp_lincomb(&nhat, alpha_pp * theta_dot, &dtd, c.dalpha);
    dbd = sp_lincomb(&nhat, beta_pp * theta_dot, &dtd, c.dbeta);
    dgd = sp_lincomb(&nhat, gamma_pp * theta_dot, &dtd, c.dgamma);
    sp_free(&dtd);
  }
  double Sk[3][3], Skd[3][3]; rv_skew(rv, Sk); rv_skew(rvd, Skd);
  for (int j = 0; j < 3; ++j) {
    if (dim == j) rv_row_add(&result, j, &dad, 1.0);
    double rv_dj = rv[dim] * rv[j];
    if (fabs(rv_dj) > 1e-15) rv_row_add(&result, j, &dbd, rv_dj);
    if (fabs(beta_dot) > 1e-15) {
      if (fabs(rv[j]) > 1e-15) rv_row_add(&result, j, &pr[dim], beta_dot * rv[j]);
      if (fabs(rv[dim]) > 1e-15) rv_row_add(&result, j, &pr[j], beta_dot * rv[dim]);
    }
    double td_dj = rvd[dim] * rv[j] + rv[dim] * rvd[j];
    if (fabs(td_dj) > 1e-15 && fabs(c.beta) > 1e-15 && theta > RV_EPS) rv_row_add(&result, j, &nhat, c.dbeta * td_dj);
    if (fabs(c.beta) > 1e-15) {
      if (fabs(rv[j]) > 1e-15) rv_row_add(&result, j, &vr[dim], c.beta * rv[j]);
      if (fabs(rvd[dim]) > 1e-15) rv_row_add(&result, j, &pr[j], c.beta * rvd[dim]);
      if (fabs(rvd[j]) > 1e-15) rv_row_add(&result, j, &pr[dim], c.beta * rvd[j]);
      if (fabs(rv[dim]) > 1e-15) rv_row_add(&result, j, &vr[j], c.beta * rv[dim]);
    }
    double sk = Sk[dim][j];
    if (fabs(sk) > 1e-15) rv_row_add(&result, j, &dgd, sk);
    if (fabs(gamma_dot) > 1e-15 && dim != j) rv_row_add(&result, j, &pr[3 - dim - j], gamma_dot * rv_sign(dim, j));
    double skd = Skd[dim][j];
    if (fabs(skd) > 1e-15 && fabs(c.gamma) > 1e-15 && theta > RV_EPS) rv_row_add(&result, j, &nhat, c.dgamma * skd);
    if (fabs(c.gamma) > 1e-15 && dim != j) rv_row_add(&result, j, &vr[3 - dim - j], c.gamma * rv_sign(dim, j));
  }
  for (int l = 0; l < 3; ++l) { sp_free(&pr[l]); sp_free(&vr[l]); }
  sp_free(&dad); sp_free(&dbd); sp_free(&dgd); sp_free(&nhat); sp_free(&jac_pos); sp_free(&jac_vel);
  return result;
}

/* GetDerivOfAngVelWrtNodes, :508-528 */
static spmat rv_d_angvel(const Euler* e, double t) {
  spmat jac = sp_copy(&e->jac_struct);
  double st[3][3], JL[3][3]; spline_point(e->euler, t, st);
  spmat vel = sp_from_dense(1, 3, st[kVel], 1);
  spmat dVel = spline_jac(e->euler, t, kVel);
  rv_left_jac(st[kPos], JL);
  spmat JLdv = rv_dense_times_sparse(JL, &dVel);
  for (int dim = X; dim <= Z; ++dim) {
    spmat dJL = rv_dJL(e, t, dim);
    spmat a = sp_mul(&vel, &dJL), b = sp_row_of(&JLdv, dim);
    spmat s = sp_lincomb(&a, 1.0, &b, 1.0);
    sp_set_row_from(&jac, dim, &s);
    sp_free(&dJL); sp_free(&a); sp_free(&b); sp_free(&s);
  }
  rv_full_pattern(e, t, &jac);
  sp_free(&vel); sp_free(&dVel); sp_free(&JLdv);
  return jac;
}

/* GetDerivOfAngAccWrtNodes, :530-561 */
static spmat rv_d_angacc(const Euler* e, double t) {
  spmat jac = sp_copy(&e->jac_struct);
  double st[3][3], JL[3][3], JLd[3][3]; spline_point(e->euler, t, st);
  spmat vel = sp_from_dense(1, 3, st[kVel], 1), acc = sp_from_dense(1, 3, st[kAcc], 1);
  spmat dVel = spline_jac(e->euler, t, kVel), dAcc = spline_jac(e->euler, t, kAcc);
  rv_left_jac(st[kPos], JL); rv_left_jac_dot(st[kPos], st[kVel], JLd);
  spmat JLd_dv = rv_dense_times_sparse(JLd, &dVel), JL_da = rv_dense_times_sparse(JL, &dAcc);
  for (int dim = X; dim <= Z; ++dim) {
    spmat dJLd = rv_dJLdot(e, t, dim), dJL = rv_dJL(e, t, dim);
    spmat t1 = sp_mul(&vel, &dJLd), t2 = sp_row_of(&JLd_dv, dim), t3 = sp_mul(&acc, &dJL), t4 = sp_row_of(&JL_da, dim);
    spmat s = sp_lincomb(&t1, 1.0, &t2, 1.0);
    sp_add_inplace(&s, &t3, 1.0); sp_add_inplace(&s, &t4, 1.0);
    sp_set_row_from(&jac, dim, &s);
    sp_free(&dJLd); sp_free(&dJL); sp_free(&t1); sp_free(&t2); sp_free(&t3); sp_free(&t4); sp_free(&s);
  }
  rv_full_pattern(e, t, &jac);
  sp_free(&vel); sp_free(&acc); sp_free(&dVel); sp_free(&dAcc); sp_free(&JLd_dv); sp_free(&JL_da);
  return jac;
}

/* EulerConverter::GetM, euler_converter.cc:133-148 */
static spmat eu_M(const double xyz[3]) {
  double z = xyz[Z], y = xyz[Y];
  spmat M = sp_zero(3, 3);
  *sp_coeffref(&M, 0, Y) = -sin(z); *sp_coeffref(&M, 0, X) = cos(y) * cos(z);
  *sp_coeffref(&M, 1, Y) = cos(z);  *sp_coeffref(&M, 1, X) = cos(y) * sin(z);
  *sp_coeffref(&M, 2, Z) = 1.0;     *sp_coeffref(&M, 2, X) = -sin(y);
  return M;
}
/* EulerConverter::GetMdot, euler_converter.cc:150-166 */
static spmat eu_Mdot(const double xyz[3], const double xyzd[3]) {
  double z = xyz[Z], zd = xyzd[Z], y = xyz[Y], yd = xyzd[Y];
  spmat M = sp_zero(3, 3);
  *sp_coeffref(&M, 0, Y) = -cos(z) * zd; *sp_coeffref(&M, 0, X) = -cos(z) * sin(y) * yd - cos(y) * sin(z) * zd;
  *sp_coeffref(&M, 1, Y) = -sin(z) * zd; *sp_coeffref(&M, 1, X) = cos(y) * cos(z) * zd - sin(y) * sin(z) * yd;
  *sp_coeffref(&M, 2, X) = -cos(y) * yd;
  return M;
}
/* GetRotationMatrixBaseToWorld(t), euler_converter.cc:200-205 -> dense + sparseView(1,-1) */
static void eu_R_t(const Euler* e, double t, double R[3][3]) {
  if (e->rotvec) { rv_R_t(e, t, R); return; }
  double st[3][3]; spline_point(e->euler, t, st);
  euler_R(st[kPos], R);
}
static spmat eu_R_sparse(const double R[3][3]) { return sp_from_dense(3, 3, &R[0][0], 1); }

/* GetAngularVelocityInWorld, :58-70 ; GetAngularAccelerationInWorld, :72-83 */
static void eu_omega(const Euler* e, double t, double w[3]) {
  if (e->rotvec) { rv_omega(e, t, w); return; }
  double st[3][3]; spline_point(e->euler, t, st);
  spmat M = eu_M(st[kPos]); sp_mul_vec(&M, st[kVel], w); sp_free(&M);
}
static void eu_omega_dot(const Euler* e, double t, double wd[3]) {
  if (e->rotvec) { rv_omega_dot(e, t, wd); return; }
  double st[3][3]; spline_point(e->euler, t, st);
  spmat Md = eu_Mdot(st[kPos], st[kVel]), M = eu_M(st[kPos]);
  double a[3], b[3];
  sp_mul_vec(&Md, st[kVel], a); sp_mul_vec(&M, st[kAcc], b);
  for (int k = 0; k < 3; ++k) wd[k] = a[k] + b[k];
  sp_free(&Md); sp_free(&M);
}

/* EulerConverter::GetJac, euler_converter.cc:306-310 */
static spmat eu_getjac(const Euler* e, double t, int deriv, int dim) {
  spmat J = spline_jac(e->euler, t, deriv);
  spmat r = sp_row_of(&J, dim);
  sp_free(&J);
  return r;
}

/* linear combination of 1 x n rows: sum_k c[k] * r[k] (union structure) */
static spmat rows_lc(int n, const double* c, spmat* const* r) {
  spmat acc = sp_scale(r[0], c[0]);
  for (int k = 1; k < n; ++k) sp_add_inplace(&acc, r[k], c[k]);
  return acc;
}

/* EulerConverter::GetDerivMwrtNodes, euler_converter.cc:168-198 */
static spmat eu_dM(const Euler* e, double t, int dim) {
  double st[3][3]; spline_point(e->euler, t, st);
  double z = st[kPos][Z], y = st[kPos][Y];
  spmat jz = eu_getjac(e, t, kPos, Z), jy = eu_getjac(e, t, kPos, Y);
  spmat jac = sp_copy(&e->jac_struct);
  if (dim == X) {
    spmat a = sp_scale(&jz, -cos(z));
    double c[2] = {-cos(z) * sin(y), -(cos(y) * sin(z))}; spmat* r[2] = {&jy, &jz};
    spmat b = rows_lc(2, c, r);
    sp_set_row_from(&jac, Y, &a); sp_set_row_from(&jac, X, &b); sp_free(&a); sp_free(&b);
  } else if (dim == Y) {
    spmat a = sp_scale(&jz, -sin(z));
    double c[2] = {cos(y) * cos(z), -(sin(y) * sin(z))}; spmat* r[2] = {&jz, &jy};
    spmat b = rows_lc(2, c, r);
    sp_set_row_from(&jac, Y, &a); sp_set_row_from(&jac, X, &b); sp_free(&a); sp_free(&b);
  } else {
    spmat b = sp_scale(&jy, -cos(y));
    sp_set_row_from(&jac, X, &b); sp_free(&b);
  }
  sp_free(&jz); sp_free(&jy);
  return jac;
}

/* EulerConverter::GetDerivMdotwrtNodes, euler_converter.cc:270-304 */
static spmat eu_dMdot(const Euler* e, double t, int dim) {
  double st[3][3]; spline_point(e->euler, t, st);
  double z = st[kPos][Z], zd = st[kVel][Z], y = st[kPos][Y], yd = st[kVel][Y];
  spmat jz = eu_getjac(e, t, kPos, Z), jy = eu_getjac(e, t, kPos, Y);
  spmat jzd = eu_getjac(e, t, kVel, Z), jyd = eu_getjac(e, t, kVel, Y);
  spmat jac = sp_copy(&e->jac_struct);
  if (dim == X) {
    double c1[2] = {sin(z) * zd, -cos(z)}; spmat* r1[2] = {&jz, &jzd};
    double c2[6] = {sin(y) * sin(z) * yd, -(cos(y) * sin(z)), -(cos(y) * cos(z) * yd), -(cos(y) * cos(z) * zd), -(cos(z) * sin(y)), sin(y) * sin(z) * zd};
    spmat* r2[6] = {&jz, &jzd, &jy, &jz, &jyd, &jy};
    spmat a = rows_lc(2, c1, r1), b = rows_lc(6, c2, r2);
    sp_set_row_from(&jac, Y, &a); sp_set_row_from(&jac, X, &b); sp_free(&a); sp_free(&b);
  } else if (dim == Y) {
    double c1[2] = {-sin(z), -(cos(z) * zd)}; spmat* r1[2] = {&jzd, &jz};
    double c2[6] = {cos(y) * cos(z), -(sin(y) * sin(z)), -(cos(y) * sin(z) * yd), -(cos(z) * sin(y) * yd), -(cos(z) * sin(y) * zd), -(cos(y) * sin(z) * zd)};
    spmat* r2[6] = {&jzd, &jyd, &jy, &jz, &jy, &jz};
    spmat a = rows_lc(2, c1, r1), b = rows_lc(6, c2, r2);
    sp_set_row_from(&jac, Y, &a); sp_set_row_from(&jac, X, &b); sp_free(&a); sp_free(&b);
  } else {
    double c2[2] = {sin(y) * yd, -cos(y)}; spmat* r2[2] = {&jy, &jyd};
    spmat b = rows_lc(2, c2, r2);
    sp_set_row_from(&jac, X, &b); sp_free(&b);
  }
  sp_free(&jz); sp_free(&jy); sp_free(&jzd); sp_free(&jyd);
  return jac;
}

/* EulerConverter::GetDerivOfAngVelWrtNodes, euler_converter.cc:85-102 */
static spmat eu_d_angvel(const Euler* e, double t) {
  if (e->rotvec) return rv_d_angvel(e, t);
  spmat jac = sp_copy(&e->jac_struct);
  double st[3][3]; spline_point(e->euler, t, st);
  spmat vel = sp_from_dense(1, 3, st[kVel], 1);
  spmat dVel = spline_jac(e->euler, t, kVel);
  spmat M = eu_M(st[kPos]);
  for (int dim = X; dim <= Z; ++dim) {
    spmat dM = eu_dM(e, t, dim);
    spmat a = sp_mul(&vel, &dM);
    spmat Mr = sp_row_of(&M, dim);
    spmat b = sp_mul(&Mr, &dVel);
    spmat s = sp_lincomb(&a, 1.0, &b, 1.0);
    sp_set_row_from(&jac, dim, &s);
    sp_free(&dM); sp_free(&a); sp_free(&Mr); sp_free(&b); sp_free(&s);
  }
  sp_free(&vel); sp_free(&dVel); sp_free(&M);
  return jac;
}

/* EulerConverter::GetDerivOfAngAccWrtNodes, euler_converter.cc:104-131 */
static spmat eu_d_angacc(const Euler* e, double t) {
  if (e->rotvec) return rv_d_angacc(e, t);
  spmat jac = sp_copy(&e->jac_struct);
  double st[3][3]; spline_point(e->euler, t, st);
  spmat vel = sp_from_dense(1, 3, st[kVel], 1);
  spmat acc = sp_from_dense(1, 3, st[kAcc], 1);
  spmat dVel = spline_jac(e->euler, t, kVel);
  spmat dAcc = spline_jac(e->euler, t, kAcc);
  spmat M = eu_M(st[kPos]), Md = eu_Mdot(st[kPos], st[kVel]);
  for (int dim = X; dim <= Z; ++dim) {
    spmat dMd = eu_dMdot(e, t, dim), dM = eu_dM(e, t, dim);
    spmat t1 = sp_mul(&vel, &dMd);
    spmat Mdr = sp_row_of(&Md, dim); spmat t2 = sp_mul(&Mdr, &dVel);
    spmat t3 = sp_mul(&acc, &dM);
    spmat Mr = sp_row_of(&M, dim); spmat t4 = sp_mul(&Mr, &dAcc);
    spmat s = sp_lincomb(&t1, 1.0, &t2, 1.0);
    sp_add_inplace(&s, &t3, 1.0); sp_add_inplace(&s, &t4, 1.0);
    sp_set_row_from(&jac, dim, &s);
    sp_free(&dMd); sp_free(&dM); sp_free(&t1); sp_free(&Mdr); sp_free(&t2); sp_free(&t3); sp_free(&Mr); sp_free(&t4); sp_free(&s);
  }
  sp_free(&vel); sp_free(&acc); sp_free(&dVel); sp_free(&dAcc); sp_free(&M); sp_free(&Md);
  return jac;
}

/* EulerConverter::GetDerivativeOfRotationMatrixWrtNodes, euler_converter.cc:241-268 */
static void eu_dR(const Euler* e, double t, spmat Rd[3][3]) {
  double st[3][3]; spline_point(e->euler, t, st);
  double x = st[kPos][X], y = st[kPos][Y], z = st[kPos][Z];
  spmat jx = eu_getjac(e, t, kPos, X), jy = eu_getjac(e, t, kPos, Y), jz = eu_getjac(e, t, kPos, Z);
  { double c[2] = {-(cos(z) * sin(y)), -(cos(y) * sin(z))}; spmat* r[2] = {&jy, &jz}; Rd[X][X] = rows_lc(2, c, r); }
  { double c[5] = {sin(x) * sin(z), -(cos(x) * cos(z)), -(sin(x) * sin(y) * sin(z)), cos(x) * cos(z) * sin(y), cos(y) * cos(z) * sin(x)};
    spmat* r[5] = {&jx, &jz, &jz, &jx, &jy}; Rd[X][Y] = rows_lc(5, c, r); }
  { double c[5] = {cos(x) * sin(z), cos(z) * sin(x), -(cos(z) * sin(x) * sin(y)), -(cos(x) * sin(y) * sin(z)), cos(x) * cos(y) * cos(z)};
    spmat* r[5] = {&jx, &jz, &jx, &jz, &jy}; Rd[X][Z] = rows_lc(5, c, r); }
  { double c[2] = {cos(y) * cos(z), -(sin(y) * sin(z))}; spmat* r[2] = {&jz, &jy}; Rd[Y][X] = rows_lc(2, c, r); }
  { double c[5] = {cos(x) * sin(y) * sin(z), -(cos(x) * sin(z)), -(cos(z) * sin(x)), cos(y) * sin(x) * sin(z), cos(z) * sin(x) * sin(y)};
    spmat* r[5] = {&jx, &jz, &jx, &jy, &jz}; Rd[Y][Y] = rows_lc(5, c, r); }
  { double c[5] = {sin(x) * sin(z), -(cos(x) * cos(z)), -(sin(x) * sin(y) * sin(z)), cos(x) * cos(y) * sin(z), cos(x) * cos(z) * sin(y)};
    spmat* r[5] = {&jz, &jx, &jx, &jy, &jz}; Rd[Y][Z] = rows_lc(5, c, r); }
  { Rd[Z][X] = sp_scale(&jy, -cos(y)); }
  { double c[2] = {cos(x) * cos(y), -(sin(x) * sin(y))}; spmat* r[2] = {&jx, &jy}; Rd[Z][Y] = rows_lc(2, c, r); }
  { double c[2] = {-(cos(y) * sin(x)), -(cos(x) * sin(y))}; spmat* r[2] = {&jx, &jy}; Rd[Z][Z] = rows_lc(2, c, r); }
  sp_free(&jx); sp_free(&jy); sp_free(&jz);
}

/* EulerConverter::DerivOfRotVecMult, euler_converter.cc:223-239 */
static spmat eu_d_rotvec(const Euler* e, double t, const double v[3], int inverse) {
  if (e->rotvec) return rv_d_rotvec(e, t, v, inverse);
  spmat Rd[3][3]; eu_dR(e, t, Rd);
  spmat jac = sp_copy(&e->jac_struct);
  for (int row = X; row <= Z; ++row)
    for (int col = X; col <= Z; ++col) {
      const spmat* jr = inverse ? &Rd[col][row] : &Rd[row][col];
      spmat cur = sp_row_of(&jac, row);
      sp_add_inplace(&cur, jr, v[col]);
      sp_set_row_from(&jac, row, &cur);
      sp_free(&cur);
    }
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) sp_free(&Rd[i][j]);
  return jac;
}

/* =============================================================================================
 * SingleRigidBodyDynamics (src/models/single_rigid_body_dynamics.cc, dynamic_model.cc)
 * ===========================================================================================*/
typedef struct {
  double m, g;
  spmat I_b;                                  /* inertia_b.sparseView()  (:69-74)          */
  int n_ee;
  double com_pos[3], com_acc[3], R[3][3], omega[3], omega_dot[3];
  double f[MAXE][3], p[MAXE][3], tau[MAXE][3];
} Model;

/* Cross, single_rigid_body_dynamics.cc:47-57 */
static spmat cross_mat(const double in[3]) {
  spmat o = sp_zero(3, 3);
  *sp_coeffref(&o, 0, 1) = -in[2]; *sp_coeffref(&o, 0, 2) = in[1];
  *sp_coeffref(&o, 1, 0) = in[2];  *sp_coeffref(&o, 1, 2) = -in[0];
  *sp_coeffref(&o, 2, 0) = -in[1]; *sp_coeffref(&o, 2, 1) = in[0];
  return o;
}

/* I_w = w_R_b_.sparseView() * I_b * w_R_b_.transpose().sparseView()  (:92, :128) */
static spmat model_Iw(const Model* M) {
  double Rt[3][3];
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Rt[i][j] = M->R[j][i];
  spmat Rs = sp_from_dense(3, 3, &M->R[0][0], 0), Rts = sp_from_dense(3, 3, &Rt[0][0], 0);
  spmat a = sp_mul(&Rs, &M->I_b), Iw = sp_mul(&a, &Rts);
  sp_free(&Rs); sp_free(&Rts); sp_free(&a);
  return Iw;
}

static void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
}

/* SingleRigidBodyDynamics::GetDynamicViolation, single_rigid_body_dynamics.cc:76-102 */
static void model_violation(const Model* M, double acc[6]) {
  double fs[3] = {0, 0, 0}, ts[3] = {0, 0, 0};
  for (int ee = 0; ee < M->n_ee; ++ee) {
    double r[3], c[3];
    for (int k = 0; k < 3; ++k) r[k] = M->com_pos[k] - M->p[ee][k];
    cross3(M->f[ee], r, c);
    for (int k = 0; k < 3; ++k) { ts[k] += c[k] + M->tau[ee][k]; fs[k] += M->f[ee][k]; }
  }
  spmat Iw = model_Iw(M);
  double a[3], Iww[3], b[3];
  sp_mul_vec(&Iw, M->omega_dot, a);
  sp_mul_vec(&Iw, M->omega, Iww);
  spmat C = cross_mat(M->omega); sp_mul_vec(&C, Iww, b);
  for (int k = 0; k < 3; ++k) acc[AX + k] = a[k] + b[k] - ts[k];
  double grav[3] = {0.0, 0.0, -M->m * M->g};
  for (int k = 0; k < 3; ++k) acc[LX + k] = M->m * M->com_acc[k] - fs[k] - grav[k];
  sp_free(&Iw); sp_free(&C);
}

/* SingleRigidBodyDynamics::GetJacobianWrtBaseLin, :104-122 */
static spmat model_jac_base_lin(const Model* M, const spmat* jpos, const spmat* jacc) {
  int n = jpos->cols;
  spmat sum = sp_zero(3, n);
  for (int ee = 0; ee < M->n_ee; ++ee) {
    spmat C = cross_mat(M->f[ee]);
    spmat jt = sp_mul(&C, jpos);
    sp_add_inplace(&sum, &jt, 1.0);
    sp_free(&C); sp_free(&jt);
  }
  spmat jac = sp_zero(6, n);
  spmat a = sp_scale(&sum, -1.0), b = sp_scale(jacc, M->m);
  sp_set_rows(&jac, AX, &a); sp_set_rows(&jac, LX, &b);
  sp_free(&sum); sp_free(&a); sp_free(&b);
  return jac;
}

/* SingleRigidBodyDynamics::GetJacobianWrtBaseAng, :124-166 */
static spmat model_jac_base_ang(const Model* M, const Euler* e, double t) {
  spmat Iw = model_Iw(M);
  double RtW[3], v11[3], v21[3], tmp[3];
  /* v11 = I_b * w_R_b_^T * omega_dot */
  for (int i = 0; i < 3; ++i) RtW[i] = M->R[0][i] * M->omega_dot[0] + M->R[1][i] * M->omega_dot[1] + M->R[2][i] * M->omega_dot[2];
  sp_mul_vec(&M->I_b, RtW, v11);
  spmat jac11 = eu_d_rotvec(e, t, v11, 0);
  spmat Rs = sp_from_dense(3, 3, &M->R[0][0], 0);
  spmat RI = sp_mul(&Rs, &M->I_b);
  spmat d12 = eu_d_rotvec(e, t, M->omega_dot, 1);
  spmat jac12 = sp_mul(&RI, &d12);
  spmat jaa = eu_d_angacc(e, t);
  spmat jac13 = sp_mul(&Iw, &jaa);
  spmat jac1 = sp_lincomb(&jac11, 1.0, &jac12, 1.0); sp_add_inplace(&jac1, &jac13, 1.0);

  for (int i = 0; i < 3; ++i) tmp[i] = M->R[0][i] * M->omega[0] + M->R[1][i] * M->omega[1] + M->R[2][i] * M->omega[2];
  sp_mul_vec(&M->I_b, tmp, v21);
  spmat jac21 = eu_d_rotvec(e, t, v21, 0);
  spmat d22 = eu_d_rotvec(e, t, M->omega, 1);
  spmat jac22 = sp_mul(&RI, &d22);
  spmat jav = eu_d_angvel(e, t);
  spmat jac23 = sp_mul(&Iw, &jav);
  spmat s = sp_lincomb(&jac21, 1.0, &jac22, 1.0); sp_add_inplace(&s, &jac23, 1.0);
  spmat Cw = cross_mat(M->omega);
  double Iww[3]; sp_mul_vec(&Iw, M->omega, Iww);
  spmat CIw = cross_mat(Iww);
  spmat p1 = sp_mul(&Cw, &s), p2 = sp_mul(&CIw, &jav);
  spmat jac2 = sp_lincomb(&p1, 1.0, &p2, -1.0);
  spmat jac = sp_zero(6, jav.cols);
  spmat top = sp_lincomb(&jac1, 1.0, &jac2, 1.0);
  sp_set_rows(&jac, AX, &top);
  spmat* fr[] = {&Iw, &jac11, &Rs, &RI, &d12, &jac12, &jaa, &jac13, &jac1, &jac21, &d22, &jac22, &jav, &jac23, &s, &Cw, &CIw, &p1, &p2, &jac2, &top};
  for (size_t i = 0; i < sizeof(fr) / sizeof(fr[0]); ++i) sp_free(fr[i]);
  return jac;
}

/* SingleRigidBodyDynamics::GetJacobianWrtForce, :168-180 */
static spmat model_jac_force(const Model* M, const spmat* jf, int ee) {
  double r[3]; for (int k = 0; k < 3; ++k) r[k] = M->com_pos[k] - M->p[ee][k];
  spmat C = cross_mat(r), Cn = sp_scale(&C, -1.0);
  spmat jt = sp_mul(&Cn, jf);
  spmat jac = sp_zero(6, jf->cols);
  spmat a = sp_scale(&jt, -1.0), b = sp_scale(jf, -1.0);
  sp_set_rows(&jac, AX, &a); sp_set_rows(&jac, LX, &b);
  sp_free(&C); sp_free(&Cn); sp_free(&jt); sp_free(&a); sp_free(&b);
  return jac;
}
/* SingleRigidBodyDynamics::GetJacobianWrtTorque, :182-191 */
static spmat model_jac_torque(const spmat* jt) {
  spmat jac = sp_zero(6, jt->cols);
  spmat a = sp_scale(jt, -1.0);
  sp_set_rows(&jac, AX, &a); sp_free(&a);
  return jac;
}
/* SingleRigidBodyDynamics::GetJacobianWrtEEPos, :193-204 */
static spmat model_jac_eepos(const Model* M, const spmat* jp, int ee) {
  spmat C = cross_mat(M->f[ee]);
  spmat njp = sp_scale(jp, -1.0);
  spmat jt = sp_mul(&C, &njp);
  spmat jac = sp_zero(6, jt.cols);
  spmat a = sp_scale(&jt, -1.0);
  sp_set_rows(&jac, AX, &a);
  sp_free(&C); sp_free(&njp); sp_free(&jt); sp_free(&a);
  return jac;
}

/* =============================================================================================
 * Problem: variable sets, spline holder, constraint sets, ifopt assembly
 * ===========================================================================================*/
typedef struct {
  int kind, ee, n, col0;
  NodesVar* nv; PhaseDur* pd;
} VarSet;

typedef struct {
  int kind, ee, rows, row0;
  double T, dt, p[6];
  int ip[9];                       /* EELinearConstraint: target, deriv, n_terms, ee*3+dim    */
  int n_dts; double* dts;          /* TimeDiscretizationConstraint::dts_                    */
  int n_ids; int* ids;             /* node ids (force/terrain/swing/base-height)           */
  /* SplineAccConstraint (spline_acc_constraint.cc:34-46) */
  const Spline* acc_spline; int acc_varset_kind; int n_junctions; double* acc_T;
  int role;                        /* towr_constraint_role: soft sets are not part of g / J     */
  int lin_vs; double* lin_M;       /* LinearEqualityConstraint: variable set index, M (rows x n_set) */
} Cons;

struct oracle_s {
  towr_problem_desc_t d;
  Terrain terrain;
  int n_ee;
  NodesVar *base_lin, *base_ang, *motion[MAXE], *ang[MAXE], *force[MAXE], *torque[MAXE];
  PhaseDur* pd[MAXE];
  Spline *s_lin, *s_ang, *s_motion[MAXE], *s_ang_ee[MAXE], *s_force[MAXE], *s_torque[MAXE];
  Euler euler;
  Model model;
  int n_vs; VarSet vs[TOWR_MAX_VARSETS];
  int n_cons; Cons cons[TOWR_MAX_CONSTRAINTS];
  int n, m;
  double* x;                        /* the current x (LinearEqualityConstraint reads its set's values) */
  double* soft_b[TOWR_MAX_COSTS];   /* SoftConstraint terms: b = (upper + lower) / 2 per wrapped row   */
};

/* TimeDiscretizationConstraint ctor, time_discretization_constraint.cc:37-50 */
static void make_dts(Cons* c) {
  int steps = (int)floor(c->T / c->dt);
  c->dts = (double*)malloc(sizeof(double) * (size_t)(steps + 2));
  double t = 0.0;
  c->n_dts = 0;
  c->dts[c->n_dts++] = t;
  for (int i = 0; i < steps; ++i) { t += c->dt; c->dts[c->n_dts++] = t; }
  c->dts[c->n_dts++] = c->T;
}

/* DynamicConstraint::UpdateModel, dynamic_constraint.cc:128-148 */
static void dyn_update_model(oracle_t* o, double t) {
  Model* M = &o->model;
  double st[3][3];
  spline_point(o->s_lin, t, st);
  memcpy(M->com_pos, st[kPos], sizeof(double[3])); memcpy(M->com_acc, st[kAcc], sizeof(double[3]));
  eu_R_t(&o->euler, t, M->R);
  eu_omega(&o->euler, t, M->omega);
  eu_omega_dot(&o->euler, t, M->omega_dot);
  for (int ee = 0; ee < o->n_ee; ++ee) {
    spline_point(o->s_force[ee], t, st);  memcpy(M->f[ee], st[kPos], sizeof(double[3]));
    spline_point(o->s_torque[ee], t, st); memcpy(M->tau[ee], st[kPos], sizeof(double[3]));
    spline_point(o->s_motion[ee], t, st); memcpy(M->p[ee], st[kPos], sizeof(double[3]));
  }
}

/* ---------------------------------------------------------------- GetValues per set ------ */
static void cons_values(oracle_t* o, const Cons* c, double* g) {
  const Terrain* T = &o->terrain;
  switch (c->kind) {
    case TOWR_C_DYNAMIC:          /* dynamic_constraint.cc:63-68 */
      for (int k = 0; k < c->n_dts; ++k) { dyn_update_model(o, c->dts[k]); model_violation(&o->model, &g[6 * k]); }
      break;
    case TOWR_C_RANGE_OF_MOTION:  /* range_of_motion_constraint.cc:72-83 */
      for (int k = 0; k < c->n_dts; ++k) {
        double t = c->dts[k], b[3][3], e[3][3], R[3][3];
        spline_point(o->s_lin, t, b); spline_point(o->s_motion[c->ee], t, e);
        eu_R_t(&o->euler, t, R);
        double v[3]; for (int q = 0; q < 3; ++q) v[q] = e[kPos][q] - b[kPos][q];
        for (int i = 0; i < 3; ++i) g[3 * k + i] = R[0][i] * v[0] + R[1][i] * v[1] + R[2][i] * v[2];
      }
      break;
    case TOWR_C_FORCE_DISCRETIZED: { /* force_constraint_discretized.cc:97-117 */
      double mu = T->friction_coeff;
      for (int k = 0; k < c->n_dts; ++k) {
        double t = c->dts[k], p[3][3], f[3][3], n[3], t1[3], t2[3];
        spline_point(o->s_motion[c->ee], t, p); spline_point(o->s_force[c->ee], t, f);
        ter_nbasis(T, NORMAL, p[kPos][X], p[kPos][Y], n);
        ter_nbasis(T, TANGENT1, p[kPos][X], p[kPos][Y], t1);
        ter_nbasis(T, TANGENT2, p[kPos][X], p[kPos][Y], t2);
        double* F = f[kPos]; int r = 5 * k;
        g[r++] = F[0] * n[0] + F[1] * n[1] + F[2] * n[2];
        g[r++] = F[0] * (t1[0] - mu * n[0]) + F[1] * (t1[1] - mu * n[1]) + F[2] * (t1[2] - mu * n[2]);
        g[r++] = F[0] * (t1[0] + mu * n[0]) + F[1] * (t1[1] + mu * n[1]) + F[2] * (t1[2] + mu * n[2]);
        g[r++] = F[0] * (t2[0] - mu * n[0]) + F[1] * (t2[1] - mu * n[1]) + F[2] * (t2[2] - mu * n[2]);
        g[r++] = F[0] * (t2[0] + mu * n[0]) + F[1] * (t2[1] + mu * n[1]) + F[2] * (t2[2] + mu * n[2]);
      }
      break;
    }
    case TOWR_C_FORCE: {          /* force_constraint.cc:62-89 */
      double mu = T->friction_coeff;
      const NodesVar* fv = o->force[c->ee]; const NodesVar* mv = o->motion[c->ee];
      int row = 0;
      for (int i = 0; i < c->n_ids; ++i) {
        int fid = c->ids[i], phase = nv_get_phase(fv, fid);
        const double* p = mv->nodes[nv_node_at_start_of_phase(mv, phase)][kPos];
        double n[3], t1[3], t2[3]; const double* F = fv->nodes[fid][kPos];
        ter_nbasis(T, NORMAL, p[X], p[Y], n);
        g[row++] = F[0] * n[0] + F[1] * n[1] + F[2] * n[2];
        ter_nbasis(T, TANGENT1, p[X], p[Y], t1);
        g[row++] = F[0] * (t1[0] - mu * n[0]) + F[1] * (t1[1] - mu * n[1]) + F[2] * (t1[2] - mu * n[2]);
        g[row++] = F[0] * (t1[0] + mu * n[0]) + F[1] * (t1[1] + mu * n[1]) + F[2] * (t1[2] + mu * n[2]);
        ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
        g[row++] = F[0] * (t2[0] - mu * n[0]) + F[1] * (t2[1] - mu * n[1]) + F[2] * (t2[2] - mu * n[2]);
        g[row++] = F[0] * (t2[0] + mu * n[0]) + F[1] * (t2[1] + mu * n[1]) + F[2] * (t2[2] + mu * n[2]);
      }
      break;
    }
    case TOWR_C_TERRAIN: {        /* terrain_constraint.cc:61-74 */
      const NodesVar* mv = o->motion[c->ee];
      for (int i = 0; i < c->n_ids; ++i) { const double* p = mv->nodes[c->ids[i]][kPos]; g[i] = p[Z] - ter_h(T, p[X], p[Y]); }
      break;
    }
    case TOWR_C_BASE_MOTION:      /* base_motion_constraint.cc:60-66 */
      for (int k = 0; k < c->n_dts; ++k) {
        double a[3][3], b[3][3];
        spline_point(o->s_lin, c->dts[k], a); spline_point(o->s_ang, c->dts[k], b);
        for (int q = 0; q < 3; ++q) { g[6 * k + LX + q] = a[kPos][q]; g[6 * k + AX + q] = b[kPos][q]; }
      }
      break;
    case TOWR_C_SPLINE_ACC:       /* spline_acc_constraint.cc:48-64 */
      for (int j = 0; j < c->n_junctions; ++j) {
        double a[3][3], b[3][3];
        poly_get_point(&c->acc_spline->polys[j], c->acc_T[j], a);
        poly_get_point(&c->acc_spline->polys[j + 1], 0.0, b);
        for (int q = 0; q < 3; ++q) g[3 * j + q] = a[kAcc][q] - b[kAcc][q];
      }
      break;
    case TOWR_C_BASE_HEIGHT:      /* base_height_constraint.cc:58-71 */
      for (int i = 0; i < c->n_ids; ++i) {
        const double* p = o->base_lin->nodes[c->ids[i]][kPos];
        g[i] = p[Z] - ter_h(T, p[X], p[Y]) - c->p[0];
      }
      break;
    case TOWR_C_SWING: {          /* swing_constraint.cc:54-78 */
      const NodesVar* mv = o->motion[c->ee]; double tsw = c->p[0];
      int row = 0;
      for (int i = 0; i < c->n_ids; ++i) {
        int id = c->ids[i];
        const double* prev = mv->nodes[id - 1][kPos]; const double* next = mv->nodes[id + 1][kPos];
        for (int dim = X; dim <= Y; ++dim) {
          double dist = next[dim] - prev[dim], center = prev[dim] + 0.5 * dist, vdes = dist / tsw;
          g[row++] = mv->nodes[id][kPos][dim] - center;
          g[row++] = mv->nodes[id][kVel][dim] - vdes;
        }
      }
      break;
    }
    case TOWR_C_TORQUE_DISCRETIZED: { /* torque_constraint_discretized.cc:101-122 */
      double mu = T->friction_coeff, kf = c->p[4];
      for (int k = 0; k < c->n_dts; ++k) {
        double t = c->dts[k], p[3][3], f[3][3], tq[3][3], n[3], t1[3], t2[3];
        spline_point(o->s_motion[c->ee], t, p); spline_point(o->s_force[c->ee], t, f); spline_point(o->s_torque[c->ee], t, tq);
        ter_nbasis(T, NORMAL, p[kPos][X], p[kPos][Y], n);
        ter_nbasis(T, TANGENT1, p[kPos][X], p[kPos][Y], t1);
        ter_nbasis(T, TANGENT2, p[kPos][X], p[kPos][Y], t2);
        double tau_t1 = dot3(tq[kPos], t1), tau_t2 = dot3(tq[kPos], t2), tau_n = dot3(tq[kPos], n), f_n = dot3(f[kPos], n);
        double tz_lim = kf * mu * f_n;
        g[4 * k + 0] = tau_t1; g[4 * k + 1] = tau_t2; g[4 * k + 2] = tau_n - tz_lim; g[4 * k + 3] = -tau_n - tz_lim;
      }
      break;
    }
    case TOWR_C_TORQUE: {         /* torque_constraint.cc:68-103 */
      const NodesVar* tv = o->torque[c->ee]; const NodesVar* mv = o->motion[c->ee];
      for (int i = 0; i < c->n_ids; ++i) {
        int tid = c->ids[i], phase = nv_get_phase(tv, tid);
        const double* p = mv->nodes[nv_node_at_start_of_phase(mv, phase)][kPos];
        const double* tau = tv->nodes[tid][kPos];
        double n[3], t1[3], t2[3];
        ter_nbasis(T, NORMAL, p[X], p[Y], n); ter_nbasis(T, TANGENT1, p[X], p[Y], t1); ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
        g[3 * i + 0] = dot3(tau, t1); g[3 * i + 1] = dot3(tau, t2); g[3 * i + 2] = dot3(tau, n);
      }
      break;
    }
    case TOWR_C_TERRAIN_HARD:     /* terrain_constraint_hard.cc:50-72 */
      for (int k = 0; k < c->n_dts; ++k) {
        double st[3][3], n[3], t1[3], t2[3];
        spline_point(o->s_motion[c->ee], c->dts[k], st);
        const double* p = st[kPos]; const double* v = st[kVel];
        ter_nbasis(T, NORMAL, p[X], p[Y], n); ter_nbasis(T, TANGENT1, p[X], p[Y], t1); ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
        double vt1 = dot3(v, t1), vt2 = dot3(v, t2), vtm = sqrt(vt1 * vt1 + vt2 * vt2);
        double dz = p[Z] - ter_h(T, p[X], p[Y]), kc = 0.02, a = kc * vtm;
        g[k] = dz - (a < kc ? a : kc);   /* std::min(k*|v_t|, k_coeff_) */
      }
      break;
    case TOWR_C_EE_LINEAR:        /* ee_linear_constraint.cc:19-28 */
      for (int k = 0; k < c->n_dts; ++k) {
        double val = 0.0;
        for (int q = 0; q < c->ip[2]; ++q) {
          int ee = c->ip[3 + q] / 3, dim = c->ip[3 + q] % 3; double st[3][3];
          spline_point(c->ip[0] == 0 ? o->s_motion[ee] : o->s_ang_ee[ee], c->dts[k], st);
          val += c->p[q] * (c->ip[1] == 0 ? st[kPos][dim] : st[kVel][dim]);
        }
        g[k] = val;
      }
      break;
    case TOWR_C_TOTAL_DURATION: { /* total_duration_constraint.cc:49-55 */
      const PhaseDur* p = o->pd[c->ee]; double s = 0.0;
      for (int i = 0; i < p->n - 1; ++i) s += p->d[i];
      g[0] = s;
      break;
    }
    case TOWR_C_LINEAR_EQ: {      /* linear_constraint.cc:47-52: M * (the set's values), dense */
      const VarSet* v = &o->vs[c->lin_vs];
      const double* xs = o->x + v->col0;
      for (int i = 0; i < c->rows; ++i) {
        double s = 0.0;
        for (int j = 0; j < v->n; ++j) s += c->lin_M[(size_t)i * v->n + j] * xs[j];
        g[i] = s;
      }
      break;
    }
  }
}

/* ------------------------------------------------------ FillJacobianBlock per set -------- */
static int vs_is(const VarSet* v, int kind, int ee) { return v->kind == kind && (kind <= TOWR_VAR_BASE_ANG || v->ee == ee); }

/* DynamicConstraint::UpdateJacobianAtInstance, dynamic_constraint.cc:77-126 */
static void dyn_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  dyn_update_model(o, t);
  int n = jac->cols;
  spmat jm = sp_zero(6, n);
  if (v->kind == TOWR_VAR_BASE_LIN) {
    spmat jp = spline_jac(o->s_lin, t, kPos), ja = spline_jac(o->s_lin, t, kAcc);
    sp_free(&jm); jm = model_jac_base_lin(&o->model, &jp, &ja);
    sp_free(&jp); sp_free(&ja);
  }
  if (v->kind == TOWR_VAR_BASE_ANG) { sp_free(&jm); jm = model_jac_base_ang(&o->model, &o->euler, t); }
  for (int ee = 0; ee < o->n_ee; ++ee) {
    if (vs_is(v, TOWR_VAR_EE_FORCE, ee)) {
      spmat jf = spline_jac(o->s_force[ee], t, kPos); sp_free(&jm); jm = model_jac_force(&o->model, &jf, ee); sp_free(&jf);
    }
    if (vs_is(v, TOWR_VAR_EE_TORQUE, ee)) {
      spmat jt = spline_jac(o->s_torque[ee], t, kPos); sp_free(&jm); jm = model_jac_torque(&jt); sp_free(&jt);
    }
    if (vs_is(v, TOWR_VAR_EE_MOTION, ee)) {
      spmat jp = spline_jac(o->s_motion[ee], t, kPos); sp_free(&jm); jm = model_jac_eepos(&o->model, &jp, ee); sp_free(&jp);
    }
    if (vs_is(v, TOWR_VAR_EE_SCHEDULE, ee)) {
      spmat jfd = spline_jac_pos_wrt_durations(o->s_force[ee], t);
      spmat a = model_jac_force(&o->model, &jfd, ee); sp_add_inplace(&jm, &a, 1.0);
      spmat jxd = spline_jac_pos_wrt_durations(o->s_motion[ee], t);
      spmat b = model_jac_eepos(&o->model, &jxd, ee); sp_add_inplace(&jm, &b, 1.0);
      sp_free(&jfd); sp_free(&a); sp_free(&jxd); sp_free(&b);
      /* NOTE: reference omits the torque term here (quirk A22 ii), reproduced */
    }
  }
  (void)c;
  sp_set_rows(jac, 6 * k, &jm);
  sp_free(&jm);
}

/* RangeOfMotionConstraint::UpdateJacobianAtInstance, range_of_motion_constraint.cc:105-131 */
static void rom_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  double R[3][3]; eu_R_t(&o->euler, t, R);
  spmat Rs = eu_R_sparse(R), bRw = sp_transpose(&Rs);
  int row = 3 * k;
  if (v->kind == TOWR_VAR_BASE_LIN) {
    spmat m1 = sp_scale(&bRw, -1.0), J = spline_jac(o->s_lin, t, kPos), r = sp_mul(&m1, &J);
    sp_set_rows(jac, row, &r); sp_free(&m1); sp_free(&J); sp_free(&r);
  }
  if (v->kind == TOWR_VAR_BASE_ANG) {
    double b[3][3], e[3][3], rW[3];
    spline_point(o->s_lin, t, b); spline_point(o->s_motion[c->ee], t, e);
    for (int q = 0; q < 3; ++q) rW[q] = e[kPos][q] - b[kPos][q];
    spmat r = eu_d_rotvec(&o->euler, t, rW, 1);
    sp_set_rows(jac, row, &r); sp_free(&r);
  }
  if (vs_is(v, TOWR_VAR_EE_MOTION, c->ee)) {
    spmat J = spline_jac(o->s_motion[c->ee], t, kPos), r = sp_mul(&bRw, &J);
    sp_set_rows(jac, row, &r); sp_free(&J); sp_free(&r);
  }
  if (vs_is(v, TOWR_VAR_EE_SCHEDULE, c->ee)) {
    spmat J = spline_jac_pos_wrt_durations(o->s_motion[c->ee], t), r = sp_mul(&bRw, &J);
    sp_set_rows(jac, row, &r); sp_free(&J); sp_free(&r);
  }
  sp_free(&Rs); sp_free(&bRw);
}

/* AccumulateLinearFormJacobian / AccumulateScaledRowJacobian, force_constraint_discretized.cc:38-67 */
static void acc_linear_form(const spmat* J, const double b[3], int dst, spmat* out) {
  for (int r = 0; r < J->rows; ++r)
    for (int q = 0; q < J->r[r].n; ++q) *sp_coeffref(out, dst, J->r[r].e[q].col) += b[r] * J->r[r].e[q].val;
}
static void acc_scaled_row(const spmat* J, int src, double s, int dst, spmat* out) {
  if (s == 0.0) return;
  for (int r = 0; r < J->rows; ++r)
    for (int q = 0; q < J->r[r].n; ++q)
      if (r == src) *sp_coeffref(out, dst, J->r[r].e[q].col) += s * J->r[r].e[q].val;
}

/* F . (a + s*b) */
static double fdot(const double F[3], const double a[3], double s, const double b[3]) {
  double t[3] = {a[0] + s * b[0], a[1] + s * b[1], a[2] + s * b[2]};
  return dot3(F, t);
}

/* ForceConstraintDiscretized::UpdateJacobianAtInstance, force_constraint_discretized.cc:131-221 */
static void fdisc_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  const Terrain* T = &o->terrain; double mu = T->friction_coeff;
  double p[3][3], f[3][3], n[3], t1[3], t2[3], b[5][3];
  spline_point(o->s_motion[c->ee], t, p); spline_point(o->s_force[c->ee], t, f);
  ter_nbasis(T, NORMAL, p[kPos][X], p[kPos][Y], n);
  ter_nbasis(T, TANGENT1, p[kPos][X], p[kPos][Y], t1);
  ter_nbasis(T, TANGENT2, p[kPos][X], p[kPos][Y], t2);
  for (int q = 0; q < 3; ++q) {
    b[0][q] = n[q]; b[1][q] = t1[q] - mu * n[q]; b[2][q] = t1[q] + mu * n[q];
    b[3][q] = t2[q] - mu * n[q]; b[4][q] = t2[q] + mu * n[q];
  }
  int r0 = 5 * k;
  if (vs_is(v, TOWR_VAR_EE_FORCE, c->ee)) {
    spmat Jf = spline_jac(o->s_force[c->ee], t, kPos);
    for (int i = 0; i < 5; ++i) acc_linear_form(&Jf, b[i], r0 + i, jac);
    sp_free(&Jf);
  }
  int is_m = vs_is(v, TOWR_VAR_EE_MOTION, c->ee), is_s = vs_is(v, TOWR_VAR_EE_SCHEDULE, c->ee);
  if (is_m || is_s) {
    spmat Jp, Jfd;
    if (is_s) {
      Jfd = spline_jac_pos_wrt_durations(o->s_force[c->ee], t);
      for (int i = 0; i < 5; ++i) acc_linear_form(&Jfd, b[i], r0 + i, jac);
      sp_free(&Jfd);
      Jp = spline_jac_pos_wrt_durations(o->s_motion[c->ee], t);
    } else {
      Jp = spline_jac(o->s_motion[c->ee], t, kPos);
    }
    for (int dim = X; dim <= Y; ++dim) {
      double dn[3], dt1[3], dt2[3], s[5];
      ter_d_nbasis(T, NORMAL, dim, p[kPos][X], p[kPos][Y], dn);
      ter_d_nbasis(T, TANGENT1, dim, p[kPos][X], p[kPos][Y], dt1);
      ter_d_nbasis(T, TANGENT2, dim, p[kPos][X], p[kPos][Y], dt2);
      s[0] = dot3(f[kPos], dn);
      s[1] = fdot(f[kPos], dt1, -mu, dn);
      s[2] = fdot(f[kPos], dt1, mu, dn);
      s[3] = fdot(f[kPos], dt2, -mu, dn);
      s[4] = fdot(f[kPos], dt2, mu, dn);
      for (int i = 0; i < 5; ++i) acc_scaled_row(&Jp, dim, s[i], r0 + i, jac);
    }
    sp_free(&Jp);
  }
}

/* ForceConstraint::FillJacobianBlock, force_constraint.cc:107-171 */
static void force_node_jac(oracle_t* o, const Cons* c, const VarSet* v, spmat* jac) {
  const Terrain* T = &o->terrain; double mu = T->friction_coeff;
  const NodesVar* fv = o->force[c->ee]; const NodesVar* mv = o->motion[c->ee];
  if (vs_is(v, TOWR_VAR_EE_FORCE, c->ee)) {
    int row = 0;
    for (int i = 0; i < c->n_ids; ++i) {
      int fid = c->ids[i], phase = nv_get_phase(fv, fid);
      const double* p = mv->nodes[nv_node_at_start_of_phase(mv, phase)][kPos];
      double n[3], t1[3], t2[3];
      ter_nbasis(T, NORMAL, p[X], p[Y], n); ter_nbasis(T, TANGENT1, p[X], p[Y], t1); ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
      for (int dim = X; dim <= Z; ++dim) {
        int idx = nv_opt_index(fv, fid, kPos, dim), rr = row;
        *sp_coeffref(jac, rr++, idx) = n[dim];
        *sp_coeffref(jac, rr++, idx) = t1[dim] - mu * n[dim];
        *sp_coeffref(jac, rr++, idx) = t1[dim] + mu * n[dim];
        *sp_coeffref(jac, rr++, idx) = t2[dim] - mu * n[dim];
        *sp_coeffref(jac, rr++, idx) = t2[dim] + mu * n[dim];
      }
      row += 5;
    }
  }
  if (vs_is(v, TOWR_VAR_EE_MOTION, c->ee)) {
    int row = 0;
    for (int i = 0; i < c->n_ids; ++i) {
      int fid = c->ids[i], phase = nv_get_phase(fv, fid);
      int ee_node = nv_node_at_start_of_phase(mv, phase);
      const double* p = mv->nodes[ee_node][kPos]; const double* F = fv->nodes[fid][kPos];
      for (int dim = X; dim <= Y; ++dim) {
        double dn[3], dt1[3], dt2[3];
        ter_d_nbasis(T, NORMAL, dim, p[X], p[Y], dn);
        ter_d_nbasis(T, TANGENT1, dim, p[X], p[Y], dt1);
        ter_d_nbasis(T, TANGENT2, dim, p[X], p[Y], dt2);
        int idx = nv_opt_index(mv, ee_node, kPos, dim), rr = row;
        *sp_coeffref(jac, rr++, idx) = dot3(F, dn);
        *sp_coeffref(jac, rr++, idx) = fdot(F, dt1, -mu, dn);
        *sp_coeffref(jac, rr++, idx) = fdot(F, dt1, mu, dn);
        *sp_coeffref(jac, rr++, idx) = fdot(F, dt2, -mu, dn);
        *sp_coeffref(jac, rr++, idx) = fdot(F, dt2, mu, dn);
      }
      row += 5;
    }
  }
}

/* TorqueConstraintDiscretized::UpdateJacobianAtInstance, torque_constraint_discretized.cc:135-235 */
static void tqdisc_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  const Terrain* T = &o->terrain; double mu = T->friction_coeff, kf = c->p[4];
  double p[3][3], f[3][3], tq[3][3], n[3], t1[3], t2[3], mn[3], b[3];
  spline_point(o->s_motion[c->ee], t, p); spline_point(o->s_force[c->ee], t, f); spline_point(o->s_torque[c->ee], t, tq);
  ter_nbasis(T, NORMAL, p[kPos][X], p[kPos][Y], n);
  ter_nbasis(T, TANGENT1, p[kPos][X], p[kPos][Y], t1);
  ter_nbasis(T, TANGENT2, p[kPos][X], p[kPos][Y], t2);
  for (int q = 0; q < 3; ++q) { mn[q] = -n[q]; b[q] = -kf * mu * n[q]; }
  int r0 = 4 * k, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3;
  int is_t = vs_is(v, TOWR_VAR_EE_TORQUE, c->ee), is_f = vs_is(v, TOWR_VAR_EE_FORCE, c->ee);
  int is_m = vs_is(v, TOWR_VAR_EE_MOTION, c->ee), is_s = vs_is(v, TOWR_VAR_EE_SCHEDULE, c->ee);
  if (is_t || is_s) {
    spmat J = is_t ? spline_jac(o->s_torque[c->ee], t, kPos) : spline_jac_pos_wrt_durations(o->s_torque[c->ee], t);
    acc_linear_form(&J, t1, r0, jac); acc_linear_form(&J, t2, r1, jac);
    acc_linear_form(&J, n, r2, jac); acc_linear_form(&J, mn, r3, jac);
    sp_free(&J);
  }
  if (is_f || is_s) {
    spmat J = is_f ? spline_jac(o->s_force[c->ee], t, kPos) : spline_jac_pos_wrt_durations(o->s_force[c->ee], t);
    acc_linear_form(&J, b, r2, jac); acc_linear_form(&J, b, r3, jac);
    sp_free(&J);
  }
  if (is_m || is_s) {
    spmat Jp = is_m ? spline_jac(o->s_motion[c->ee], t, kPos) : spline_jac_pos_wrt_durations(o->s_motion[c->ee], t);
    for (int dim = X; dim <= Y; ++dim) {
      double dn[3], dt1[3], dt2[3];
      ter_d_nbasis(T, NORMAL, dim, p[kPos][X], p[kPos][Y], dn);
      ter_d_nbasis(T, TANGENT1, dim, p[kPos][X], p[kPos][Y], dt1);
      ter_d_nbasis(T, TANGENT2, dim, p[kPos][X], p[kPos][Y], dt2);
      double s_tx = dot3(tq[kPos], dt1), s_ty = dot3(tq[kPos], dt2), s_tau_n = dot3(tq[kPos], dn);
      double s_lim = kf * mu * dot3(f[kPos], dn);
      acc_scaled_row(&Jp, dim, s_tx, r0, jac);
      acc_scaled_row(&Jp, dim, s_ty, r1, jac);
      acc_scaled_row(&Jp, dim, s_tau_n - s_lim, r2, jac);
      acc_scaled_row(&Jp, dim, -s_tau_n - s_lim, r3, jac);
    }
    sp_free(&Jp);
  }
}

/* TerrainConstraintHard::UpdateJacobianAtInstance, terrain_constraint_hard.cc:84-132 */
static void thard_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  if (!vs_is(v, TOWR_VAR_EE_MOTION, c->ee)) return;
  const Terrain* T = &o->terrain;
  double st[3][3], n[3], t1[3], t2[3];
  spline_point(o->s_motion[c->ee], t, st);
  const double* p = st[kPos]; const double* vel = st[kVel];
  ter_nbasis(T, NORMAL, p[X], p[Y], n); ter_nbasis(T, TANGENT1, p[X], p[Y], t1); ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
  double vt1 = dot3(vel, t1), vt2 = dot3(vel, t2), vtm = sqrt(vt1 * vt1 + vt2 * vt2), kc = 0.02;
  spmat jp = spline_jac(o->s_motion[c->ee], t, kPos), jv = spline_jac(o->s_motion[c->ee], t, kVel);
  spmat row = sp_row_of(&jp, Z);
  for (int dim = X; dim <= Y; ++dim) {
    spmat r = sp_row_of(&jp, dim);
    sp_add_inplace(&row, &r, -ter_dh(T, dim, p[X], p[Y]));   /* -= terrain_deriv * jac_pos.row(dim) */
    sp_free(&r);
  }
  if (vtm > 1e-6 && kc * vtm < 0.05 - 1e-6) {
    double td[3];
    for (int q = 0; q < 3; ++q) td[q] = (vt1 * t1[q] + vt2 * t2[q]) / vtm;
    for (int dim = X; dim <= Z; ++dim) {
      spmat r = sp_row_of(&jv, dim);
      sp_add_inplace(&row, &r, -(kc * td[dim]));
      sp_free(&r);
    }
  }
  sp_set_rows(jac, k, &row);
  sp_free(&row); sp_free(&jp); sp_free(&jv);
}

/* EELinearConstraint::UpdateJacobianAtInstance, ee_linear_constraint.cc:37-48 */
static void eelin_jac_instance(oracle_t* o, const Cons* c, double t, int k, const VarSet* v, spmat* jac) {
  const int kind = c->ip[0] == 0 ? TOWR_VAR_EE_MOTION : TOWR_VAR_EE_ANG;
  spmat row = sp_zero(1, jac->cols);
  int any = 0;
  for (int q = 0; q < c->ip[2]; ++q) {
    int ee = c->ip[3 + q] / 3, dim = c->ip[3 + q] % 3;
    if (!vs_is(v, kind, ee)) continue;
    spmat J = spline_jac(kind == TOWR_VAR_EE_MOTION ? o->s_motion[ee] : o->s_ang_ee[ee], t, c->ip[1] == 0 ? kPos : kVel);
    spmat r = sp_row_of(&J, dim);
    sp_add_inplace(&row, &r, c->p[q]);
    sp_free(&J); sp_free(&r);
    any = 1;
  }
  if (any) sp_set_rows(jac, k, &row);
  sp_free(&row);
}

static void cons_fill_jac(oracle_t* o, const Cons* c, const VarSet* v, spmat* jac) {
  const Terrain* T = &o->terrain;
  switch (c->kind) {
    case TOWR_C_DYNAMIC:           /* TimeDiscretizationConstraint::FillJacobianBlock, :89-96 */
      for (int k = 0; k < c->n_dts; ++k) dyn_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_RANGE_OF_MOTION:
      for (int k = 0; k < c->n_dts; ++k) rom_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_FORCE_DISCRETIZED:
      for (int k = 0; k < c->n_dts; ++k) fdisc_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_FORCE: force_node_jac(o, c, v, jac); break;
    case TOWR_C_TERRAIN:           /* terrain_constraint.cc:93-111 */
      if (vs_is(v, TOWR_VAR_EE_MOTION, c->ee)) {
        const NodesVar* mv = o->motion[c->ee];
        for (int i = 0; i < c->n_ids; ++i) {
          int id = c->ids[i];
          *sp_coeffref(jac, i, nv_opt_index(mv, id, kPos, Z)) = 1.0;
          const double* p = mv->nodes[id][kPos];
          for (int dim = X; dim <= Y; ++dim)
            *sp_coeffref(jac, i, nv_opt_index(mv, id, kPos, dim)) = -ter_dh(T, dim, p[X], p[Y]);
        }
      }
      break;
    case TOWR_C_BASE_MOTION:       /* base_motion_constraint.cc:75-85 */
      for (int k = 0; k < c->n_dts; ++k) {
        double t = c->dts[k];
        if (v->kind == TOWR_VAR_BASE_ANG) { spmat J = spline_jac(o->s_ang, t, kPos); sp_set_rows(jac, 6 * k + AX, &J); sp_free(&J); }
        if (v->kind == TOWR_VAR_BASE_LIN) { spmat J = spline_jac(o->s_lin, t, kPos); sp_set_rows(jac, 6 * k + LX, &J); sp_free(&J); }
      }
      break;
    case TOWR_C_SPLINE_ACC:        /* spline_acc_constraint.cc:66-80 */
      if (v->kind == c->acc_varset_kind)
        for (int j = 0; j < c->n_junctions; ++j) {
          spmat a = spline_jac_id(c->acc_spline, j, c->acc_T[j], kAcc);
          spmat b = spline_jac_id(c->acc_spline, j + 1, 0.0, kAcc);
          spmat d = sp_lincomb(&a, 1.0, &b, -1.0);
          sp_set_rows(jac, 3 * j, &d);
          sp_free(&a); sp_free(&b); sp_free(&d);
        }
      break;
    case TOWR_C_BASE_HEIGHT:       /* base_height_constraint.cc:90-110 */
      if (v->kind == TOWR_VAR_BASE_LIN)
        for (int i = 0; i < c->n_ids; ++i) {
          int id = c->ids[i];
          *sp_coeffref(jac, i, nv_opt_index(o->base_lin, id, kPos, Z)) = 1.0;
          const double* p = o->base_lin->nodes[id][kPos];
          for (int dim = X; dim <= Y; ++dim)
            *sp_coeffref(jac, i, nv_opt_index(o->base_lin, id, kPos, dim)) = -ter_dh(T, dim, p[X], p[Y]);
        }
      break;
    case TOWR_C_SWING:             /* swing_constraint.cc:86-108 */
      if (vs_is(v, TOWR_VAR_EE_MOTION, c->ee)) {
        const NodesVar* mv = o->motion[c->ee]; double tsw = c->p[0];
        int row = 0;
        for (int i = 0; i < c->n_ids; ++i) {
          int id = c->ids[i];
          for (int dim = X; dim <= Y; ++dim) {
            *sp_coeffref(jac, row, nv_opt_index(mv, id, kPos, dim)) = 1.0;
            *sp_coeffref(jac, row, nv_opt_index(mv, id + 1, kPos, dim)) = -0.5;
            *sp_coeffref(jac, row, nv_opt_index(mv, id - 1, kPos, dim)) = -0.5;
            row++;
            *sp_coeffref(jac, row, nv_opt_index(mv, id, kVel, dim)) = 1.0;
            *sp_coeffref(jac, row, nv_opt_index(mv, id + 1, kPos, dim)) = -1.0 / tsw;
            *sp_coeffref(jac, row, nv_opt_index(mv, id - 1, kPos, dim)) = +1.0 / tsw;
            row++;
          }
        }
      }
      break;
    case TOWR_C_TORQUE_DISCRETIZED:
      for (int k = 0; k < c->n_dts; ++k) tqdisc_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_TERRAIN_HARD:
      for (int k = 0; k < c->n_dts; ++k) thard_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_EE_LINEAR:
      for (int k = 0; k < c->n_dts; ++k) eelin_jac_instance(o, c, c->dts[k], k, v, jac);
      break;
    case TOWR_C_TORQUE: {          /* torque_constraint.cc:129-193 */
      const NodesVar* tv = o->torque[c->ee]; const NodesVar* mv = o->motion[c->ee];
      if (vs_is(v, TOWR_VAR_EE_TORQUE, c->ee))
        for (int i = 0; i < c->n_ids; ++i) {
          int tid = c->ids[i], phase = nv_get_phase(tv, tid);
          const double* p = mv->nodes[nv_node_at_start_of_phase(mv, phase)][kPos];
          double n[3], t1[3], t2[3];
          ter_nbasis(T, NORMAL, p[X], p[Y], n); ter_nbasis(T, TANGENT1, p[X], p[Y], t1); ter_nbasis(T, TANGENT2, p[X], p[Y], t2);
          for (int dim = X; dim <= Z; ++dim) {
            int idx = nv_opt_index(tv, tid, kPos, dim);
            *sp_coeffref(jac, 3 * i + 0, idx) = t1[dim];
            *sp_coeffref(jac, 3 * i + 1, idx) = t2[dim];
            *sp_coeffref(jac, 3 * i + 2, idx) = n[dim];
          }
        }
      if (vs_is(v, TOWR_VAR_EE_MOTION, c->ee))
        for (int i = 0; i < c->n_ids; ++i) {
          int tid = c->ids[i], phase = nv_get_phase(tv, tid);
          int ee_node = nv_node_at_start_of_phase(mv, phase);
          const double* p = mv->nodes[ee_node][kPos];
          const double* tau = tv->nodes[nv_node_at_start_of_phase(tv, phase)][kPos];   /* GetValueAtStartOfPhase (:166) */
          for (int dim = X; dim <= Y; ++dim) {
            double dn[3], dt1[3], dt2[3];
            ter_d_nbasis(T, TANGENT1, dim, p[X], p[Y], dt1);
            ter_d_nbasis(T, TANGENT2, dim, p[X], p[Y], dt2);
            ter_d_nbasis(T, NORMAL, dim, p[X], p[Y], dn);
            int idx = nv_opt_index(mv, ee_node, kPos, dim);
            *sp_coeffref(jac, 3 * i + 0, idx) = dot3(tau, dt1);
            *sp_coeffref(jac, 3 * i + 1, idx) = dot3(tau, dt2);
            *sp_coeffref(jac, 3 * i + 2, idx) = dot3(tau, dn);
          }
        }
      break;
    }
    case TOWR_C_TOTAL_DURATION:    /* total_duration_constraint.cc:66-72 */
      if (vs_is(v, TOWR_VAR_EE_SCHEDULE, c->ee))
        for (int col = 0; col < o->pd[c->ee]->n - 1; ++col) *sp_coeffref(jac, 0, col) = 1.0;
      break;
    case TOWR_C_LINEAR_EQ:         /* linear_constraint.cc:68-76: jac = M.sparseView() (exact zeros pruned) */
      if (v == &o->vs[c->lin_vs])
        for (int i = 0; i < c->rows; ++i)
          for (int j = 0; j < v->n; ++j) {
            const double mij = c->lin_M[(size_t)i * v->n + j];
            if (mij != 0.0) *sp_coeffref(jac, i, j) = mij;
          }
      break;
  }
}

/* ifopt Composite::SetVariables -> each VariableSet::SetVariables */
static void set_variables(oracle_t* o, const double* x) {
  memcpy(o->x, x, sizeof(double) * (size_t)o->n);
  for (int i = 0; i < o->n_vs; ++i) {
    VarSet* v = &o->vs[i];
    if (v->nv) nv_set_variables(v->nv, x + v->col0);
    else pd_set_variables(v->pd, x + v->col0);
  }
}

/* ----------------------------------------------------- triplet assembly (setFromTriplets) -- */
typedef struct { int r, c; double v; } Trip;
typedef struct { Trip* t; long n, cap; } TripList;
static void trip_push(TripList* L, int r, int c, double v) {
  if (L->n == L->cap) { L->cap = L->cap ? 2 * L->cap : 4096; L->t = (Trip*)realloc(L->t, sizeof(Trip) * (size_t)L->cap); }
  L->t[L->n].r = r; L->t[L->n].c = c; L->t[L->n].v = v; L->n++;
}
static int trip_cmp(const void* a, const void* b) {
  const Trip* x = (const Trip*)a; const Trip* y = (const Trip*)b;
  if (x->r != y->r) return x->r < y->r ? -1 : 1;
  return (x->c > y->c) - (x->c < y->c);
}
/* sort + sum duplicates, in place; returns new count */
static long trip_compress(TripList* L) {
  qsort(L->t, (size_t)L->n, sizeof(Trip), trip_cmp);
  long w = 0;
  for (long i = 0; i < L->n; ++i) {
    if (w > 0 && L->t[w - 1].r == L->t[i].r && L->t[w - 1].c == L->t[i].c) L->t[w - 1].v += L->t[i].v;
    else L->t[w++] = L->t[i];
  }
  L->n = w;
  return w;
}

/* ifopt ConstraintSet::GetJacobian (per set, triplets of every FillJacobianBlock) followed by
 * Composite::GetJacobian (row offsets) and Problem::GetJacobianOfConstraints. */
static void build_jacobian(oracle_t* o, TripList* all) {
  all->n = 0;
  for (int ci = 0; ci < o->n_cons; ++ci) {
    Cons* c = &o->cons[ci];
    if (c->role == TOWR_ROLE_SOFT) continue;   /* wrapped by a SoftConstraint cost only */
    TripList L = {0, 0, 0};
    for (int vi = 0; vi < o->n_vs; ++vi) {
      VarSet* v = &o->vs[vi];
      spmat jac = sp_zero(c->rows, v->n);          /* jac.resize(GetRows(), n) */
      cons_fill_jac(o, c, v, &jac);
      for (int r = 0; r < jac.rows; ++r)
        for (int q = 0; q < jac.r[r].n; ++q) trip_push(&L, r, v->col0 + jac.r[r].e[q].col, jac.r[r].e[q].val);
      sp_free(&jac);
    }
    trip_compress(&L);                              /* jacobian.setFromTriplets (per set) */
    for (long i = 0; i < L.n; ++i) trip_push(all, c->row0 + L.t[i].r, L.t[i].c, L.t[i].v);
    free(L.t);
  }
  trip_compress(all);                               /* Composite setFromTriplets */
}

/* ============================================================================================
 * construction (NlpFormulation::GetVariableSets / GetConstraints, nlp_formulation.cc:76-378)
 * ==========================================================================================*/
static void set_err(char* err, int len, const char* msg) { if (err && len > 0) { snprintf(err, (size_t)len, "%s", msg); } }

oracle_t* oracle_create(const towr_problem_desc_t* d, char* err, int errlen) { return oracle_create_ex(d, 0, NULL, err, errlen); }

static const towr_data_t* find_data(int n_data, const towr_data_t* data, int kind, int index) {
  for (int i = 0; i < n_data; ++i) if (data[i].kind == kind && data[i].index == index) return &data[i];
  return NULL;
}

oracle_t* oracle_create_ex(const towr_problem_desc_t* d, int n_data, const towr_data_t* data, char* err, int errlen) {
  if (!d || d->abi_version != TOWR_GPU_ABI_VERSION) { set_err(err, errlen, "bad abi version"); return NULL; }
  if (n_data < 0 || (n_data > 0 && !data)) { set_err(err, errlen, "bad side data"); return NULL; }
  if (d->angular_rep != 0 && d->angular_rep != 1) { set_err(err, errlen, "angular_rep must be 0 (EulerZYX) or 1 (RotationVector)"); return NULL; }
  int E = d->robot.n_ee;
  if (E < 1 || E > MAXE) { set_err(err, errlen, "bad n_ee"); return NULL; }
  oracle_t* o = (oracle_t*)calloc(1, sizeof(oracle_t));
  o->d = *d; o->terrain = d->terrain; o->n_ee = E;
  double T = d->total_time;

  /* Parameters::GetBasePolyDurations, parameters.cc:114-130 */
  double base_d[4096]; int nb = 0;
  { double dt = d->duration_base_polynomial, tl = T, eps = 1e-10;
    while (tl > eps) { base_d[nb++] = tl > dt ? dt : tl; tl -= dt; } }

  o->base_lin = nv_all(TOWR_VAR_BASE_LIN, nb + 1);
  o->base_ang = nv_all(TOWR_VAR_BASE_ANG, nb + 1);
  for (int ee = 0; ee < E; ++ee) {
    int np = d->n_phases[ee], cs = d->contact_at_start[ee];
    o->motion[ee] = nv_phase_based(TOWR_VAR_EE_MOTION, ee, np, cs, d->ee_polynomials_per_swing_phase);
    o->ang[ee] = nv_phase_based(TOWR_VAR_EE_ANG, ee, np, cs, d->ee_polynomials_per_swing_phase);
    o->force[ee] = nv_phase_based(TOWR_VAR_EE_FORCE, ee, np, cs, d->force_polynomials_per_stance_phase);
    o->torque[ee] = nv_phase_based(TOWR_VAR_EE_TORQUE, ee, np, cs, d->torque_polynomials_per_stance_phase);
    PhaseDur* p = (PhaseDur*)calloc(1, sizeof(PhaseDur));  /* PhaseDurations ctor, phase_durations.cc:41-53 */
    p->ee = ee; p->n = np; p->initial_contact = cs;
    double s = 0.0;
    for (int i = 0; i < np; ++i) { p->d[i] = d->phase_durations[ee][i]; s += p->d[i]; }
    p->t_total = s;
    o->pd[ee] = p;
  }

  /* ---- initial values (nlp_formulation.cc:121-346 or procedural_example.cc:134-166) ---- */
  const towr_init_t* in = &d->init;
  const towr_robot_t* rb = &d->robot;
  if (in->mode == TOWR_INIT_FORMULATION) {
    double fx = in->base_lin_p1[X], fy = in->base_lin_p1[Y];
    double fp[3] = {fx, fy, ter_h(&o->terrain, fx, fy) - rb->nominal_stance[0][Z]};
    nv_set_linear(o->base_lin, in->base_lin_p0, fp, T);
    nv_set_linear(o->base_ang, in->base_ang_p0, in->base_ang_p1, T);
    for (int ee = 0; ee < E; ++ee) {
      double yaw[3] = {0.0, 0.0, in->base_ang_p1[Z]}, R[3][3], fe[3];
      euler_R(yaw, R);
      for (int q = 0; q < 3; ++q)
        fe[q] = in->base_lin_p1[q] + (R[q][0] * rb->nominal_stance[ee][0] + R[q][1] * rb->nominal_stance[ee][1] + R[q][2] * rb->nominal_stance[ee][2]);
      double tgt[3] = {fe[X], fe[Y], ter_h(&o->terrain, fe[X], fe[Y])};
      nv_set_linear_rel_base(o->motion[ee], in->ee_p0[ee], tgt, in->base_lin_p0, in->base_lin_p1,
                             in->base_ang_p0, in->base_ang_p1, T);
      nv_set_linear(o->ang[ee], in->base_ang_p0, in->base_ang_p1, T);
      double fs[3] = {0.0, 0.0, rb->mass * rb->gravity / E};
      nv_set_linear(o->force[ee], fs, fs, T);
      double z3[3] = {0, 0, 0};
      nv_set_linear(o->torque[ee], z3, z3, T);
    }
  } else {
    nv_set_linear(o->base_lin, in->base_lin_p0, in->base_lin_p1, T);
    nv_set_linear(o->base_ang, in->base_ang_p0, in->base_ang_p1, T);
    for (int ee = 0; ee < E; ++ee) {
      nv_set_linear(o->motion[ee], in->ee_p0[ee], in->ee_p1[ee], T);
      nv_set_linear(o->ang[ee], in->base_ang_p0, in->base_ang_p1, T);
      double fs[3] = {0.0, 0.0, rb->mass * rb->gravity / E}, z3[3] = {0, 0, 0};
      nv_set_linear(o->force[ee], fs, fs, T);
      nv_set_linear(o->torque[ee], z3, z3, T);
    }
  }

  /* ---- SplineHolder, spline_holder.cc:35-69 ---- */
  o->s_lin = spline_new(o->base_lin, base_d, NULL);
  o->s_ang = spline_new(o->base_ang, base_d, NULL);
  for (int ee = 0; ee < E; ++ee) {
    double pd[1024];
    PhaseDur* p = d->optimize_timings ? o->pd[ee] : NULL;
    NodesVar* sets[4] = {o->motion[ee], o->ang[ee], o->force[ee], o->torque[ee]};
    Spline** dst[4] = {&o->s_motion[ee], &o->s_ang_ee[ee], &o->s_force[ee], &o->s_torque[ee]};
    for (int q = 0; q < 4; ++q) {
      nv_phase_to_poly_durations(sets[q], o->pd[ee]->d, pd);
      *dst[q] = spline_new(sets[q], pd, p);
    }
  }
  o->euler.euler = o->s_ang;
  o->euler.jac_struct = sp_zero(3, o->base_ang->n_rows);   /* euler_converter.cc:38-42, rotvec_converter.cc:12-16 */
  o->euler.rotvec = d->angular_rep == 1;                     /* nlp_formulation.cc:113-116 */

  /* ---- model (SingleRigidBodyDynamics ctor + BuildInertiaTensor, :36-74) ---- */
  o->model.m = rb->mass; o->model.g = rb->gravity; o->model.n_ee = E;
  { const double* I = rb->inertia;
    double Ib[9] = {I[0], -I[3], -I[4], -I[3], I[1], -I[5], -I[4], -I[5], I[2]};
    o->model.I_b = sp_from_dense(3, 3, Ib, 0); }

  /* ---- variable sets in AddVariableSet order ---- */
  int col = 0;
  o->n_vs = d->n_varsets;
  for (int i = 0; i < d->n_varsets; ++i) {
    VarSet* v = &o->vs[i];
    v->kind = d->varsets[i].kind; v->ee = d->varsets[i].ee;
    if (v->kind != TOWR_VAR_BASE_LIN && v->kind != TOWR_VAR_BASE_ANG && (v->ee < 0 || v->ee >= E)) { set_err(err, errlen, "bad varset ee"); oracle_destroy(o); return NULL; }
    switch (v->kind) {
      case TOWR_VAR_BASE_LIN: v->nv = o->base_lin; break;
      case TOWR_VAR_BASE_ANG: v->nv = o->base_ang; break;
      case TOWR_VAR_EE_MOTION: v->nv = o->motion[v->ee]; break;
      case TOWR_VAR_EE_ANG: v->nv = o->ang[v->ee]; break;
      case TOWR_VAR_EE_FORCE: v->nv = o->force[v->ee]; break;
      case TOWR_VAR_EE_TORQUE: v->nv = o->torque[v->ee]; break;
      case TOWR_VAR_EE_SCHEDULE: v->pd = o->pd[v->ee]; break;
      default: set_err(err, errlen, "bad varset kind"); oracle_destroy(o); return NULL;
    }
    v->n = v->nv ? v->nv->n_rows : v->pd->n - 1;
    v->col0 = col; col += v->n;
  }
  o->n = col;
  o->x = (double*)calloc((size_t)(col > 0 ? col : 1), sizeof(double));

  /* ---- cost terms ---- */
  if (d->n_costs < 0 || d->n_costs > TOWR_MAX_COSTS) { set_err(err, errlen, "bad n_costs"); oracle_destroy(o); return NULL; }
  for (int i = 0; i < d->n_costs; ++i) {
    const towr_cost_t* c = &d->costs[i];
    int ok = c->kind >= TOWR_COST_NODE && c->kind <= TOWR_COST_SOFT;
    if (c->kind == TOWR_COST_BASE_HEIGHT) ok = ok && c->dt > 0.0;   /* the reference loops forever otherwise */
    if (c->kind == TOWR_COST_SOFT) ok = ok && c->ip[0] >= 0 && c->ip[0] < d->n_constraints;
    if (c->kind == TOWR_COST_NODE)
      ok = ok && c->ip[0] >= TOWR_VAR_BASE_LIN && c->ip[0] <= TOWR_VAR_EE_TORQUE && c->ip[1] >= 0 && c->ip[1] <= 1 &&
           c->ip[2] >= 0 && c->ip[2] <= 2 && (c->ip[0] <= TOWR_VAR_BASE_ANG || (c->ee >= 0 && c->ee < E));
    if (c->kind == TOWR_COST_EE_BASE_POS) ok = ok && c->ee >= 0 && c->ee < E;
    if (!ok) { set_err(err, errlen, "bad cost term"); oracle_destroy(o); return NULL; }
  }

  /* ---- constraint sets in AddConstraintSet order ---- */
  int row = 0;
  o->n_cons = d->n_constraints;
  for (int i = 0; i < d->n_constraints; ++i) {
    Cons* c = &o->cons[i];
    const towr_constraint_t* s = &d->constraints[i];
    c->kind = s->kind; c->ee = s->ee; c->T = s->T; c->dt = s->dt;
    memcpy(c->p, s->p, sizeof(c->p));
    memcpy(c->ip, s->ip, sizeof(c->ip));
    c->role = s->role;
    if (c->role != TOWR_ROLE_HARD && c->role != TOWR_ROLE_SOFT) { set_err(err, errlen, "bad constraint role"); oracle_destroy(o); return NULL; }
    switch (c->kind) {
      case TOWR_C_TORQUE_DISCRETIZED: make_dts(c); c->rows = 4 * c->n_dts; break;      /* torque_constraint_discretized.cc:92-93 */
      case TOWR_C_TERRAIN_HARD: make_dts(c); c->rows = c->n_dts; break;                /* terrain_constraint_hard.cc:47 */
      case TOWR_C_EE_LINEAR:      /* ee_linear_constraint.cc:15-16 */
        if (c->ip[2] < 1 || c->ip[2] > 6 || c->ip[0] < 0 || c->ip[0] > 1 || c->ip[1] < 0 || c->ip[1] > 1) { set_err(err, errlen, "bad EELinear definition"); oracle_destroy(o); return NULL; }
        for (int q = 0; q < c->ip[2]; ++q)
          if (c->ip[3 + q] < 0 || c->ip[3 + q] >= 3 * E) { set_err(err, errlen, "bad EELinear term"); oracle_destroy(o); return NULL; }
        make_dts(c); c->rows = c->n_dts; break;
      case TOWR_C_TORQUE: {       /* TorqueConstraint::InitVariableDependedQuantities, torque_constraint.cc:56-66 */
        NodesVar* tv = o->torque[c->ee];
        c->ids = (int*)malloc(sizeof(int) * (size_t)tv->n_nodes);
        for (int id = 0; id < tv->n_nodes; ++id) if (!nv_is_constant_node(tv, id)) c->ids[c->n_ids++] = id;
        c->rows = 3 * c->n_ids;
        break;
      }
      case TOWR_C_DYNAMIC: make_dts(c); c->rows = 6 * c->n_dts; break;                 /* :54 */
      case TOWR_C_RANGE_OF_MOTION: make_dts(c); c->rows = 3 * c->n_dts; break;         /* :55 */
      case TOWR_C_FORCE_DISCRETIZED: make_dts(c); c->rows = 5 * c->n_dts; break;       /* :88 */
      case TOWR_C_BASE_MOTION: make_dts(c); c->rows = 6 * c->n_dts; break;             /* :57 */
      case TOWR_C_FORCE: {        /* ForceConstraint::InitVariableDependedQuantities, :50-60 */
        NodesVar* fv = o->force[c->ee];
        c->ids = (int*)malloc(sizeof(int) * (size_t)fv->n_nodes);
        for (int id = 0; id < fv->n_nodes; ++id) if (!nv_is_constant_node(fv, id)) c->ids[c->n_ids++] = id;
        c->rows = 5 * c->n_ids;
        break;
      }
      case TOWR_C_TERRAIN: {      /* TerrainConstraint::InitVariableDependedQuantities, :48-59 */
        NodesVar* mv = o->motion[c->ee];
        c->ids = (int*)malloc(sizeof(int) * (size_t)mv->n_nodes);
        for (int id = 1; id < mv->n_nodes; ++id) c->ids[c->n_ids++] = id;
        c->rows = c->n_ids;
        break;
      }
      case TOWR_C_BASE_HEIGHT: {  /* BaseHeightConstraint::InitVariableDependedQuantities, :45-56 */
        c->ids = (int*)malloc(sizeof(int) * (size_t)o->base_lin->n_nodes);
        for (int id = 1; id < o->base_lin->n_nodes; ++id) c->ids[c->n_ids++] = id;
        c->rows = c->n_ids;
        break;
      }
      case TOWR_C_SWING: {        /* SwingConstraint::InitVariableDependedQuantities, :41-52 */
        NodesVar* mv = o->motion[c->ee];
        c->ids = (int*)malloc(sizeof(int) * (size_t)mv->n_nodes);
        for (int id = 0; id < mv->n_nodes; ++id) if (!nv_is_constant_node(mv, id)) c->ids[c->n_ids++] = id;
        for (int q = 0; q < c->n_ids; ++q)
          if (c->ids[q] == 0 || c->ids[q] == mv->n_nodes - 1) { set_err(err, errlen, "swing node at trajectory boundary (reference indexes out of range)"); oracle_destroy(o); return NULL; }
        c->rows = c->n_ids * 2 * 2;
        break;
      }
      case TOWR_C_SPLINE_ACC: {   /* SplineAccConstraint ctor, :34-46 */
        c->acc_spline = c->ee == 0 ? o->s_lin : o->s_ang;
        c->acc_varset_kind = c->ee == 0 ? TOWR_VAR_BASE_LIN : TOWR_VAR_BASE_ANG;
        c->n_junctions = c->acc_spline->n_polys - 1;
        c->acc_T = (double*)malloc(sizeof(double) * (size_t)c->acc_spline->n_polys);
        spline_durations(c->acc_spline, c->acc_T);
        c->rows = 3 * c->n_junctions;
        break;
      }
      case TOWR_C_TOTAL_DURATION: c->rows = 1; break;
      case TOWR_C_LINEAR_EQ: {    /* LinearEqualityConstraint ctor, linear_constraint.cc:35-45 */
        const towr_data_t* m = find_data(n_data, data, TOWR_DATA_LINEAR_M, i);
        if (c->ip[0] < 0 || c->ip[0] >= o->n_vs || c->ip[1] < 0 || !m || !m->data ||
            m->count != (int64_t)c->ip[1] * o->vs[c->ip[0]].n) { set_err(err, errlen, "bad LinearEquality constraint or matrix"); oracle_destroy(o); return NULL; }
        c->lin_vs = c->ip[0]; c->rows = c->ip[1];
        c->lin_M = (double*)malloc(sizeof(double) * (size_t)(m->count > 0 ? m->count : 1));
        memcpy(c->lin_M, m->data, sizeof(double) * (size_t)m->count);
        break;
      }
      default: set_err(err, errlen, "unsupported constraint kind"); oracle_destroy(o); return NULL;
    }
    if (c->role == TOWR_ROLE_SOFT) { c->row0 = -1; continue; }   /* not a row block of g */
    c->row0 = row; row += c->rows;
  }
  o->m = row;
  /* SoftConstraint ctor (soft_constraint.cc:34-50): b = (upper + lower) / 2 of the wrapped set */
  for (int i = 0; i < d->n_costs; ++i) {
    if (d->costs[i].kind != TOWR_COST_SOFT) continue;
    const Cons* w = &o->cons[d->costs[i].ip[0]];
    const towr_data_t* b = find_data(n_data, data, TOWR_DATA_SOFT_BOUNDS, i);
    if (!b || !b->data || b->count != 2 * (int64_t)w->rows) { set_err(err, errlen, "SoftConstraint term without bounds of its set's size"); oracle_destroy(o); return NULL; }
    o->soft_b[i] = (double*)malloc(sizeof(double) * (size_t)(w->rows > 0 ? w->rows : 1));
    for (int r = 0; r < w->rows; ++r) o->soft_b[i][r] = (b->data[w->rows + r] + b->data[r]) / 2.;
  }
  return o;
}

static void nv_free(NodesVar* v) { if (!v) return; free(v->nodes); free(v->nvi_n); free(v->nvi); free(v->pinfo); free(v); }
static void spline_free(Spline* s) { if (!s) return; free(s->polys); sp_free(&s->jac_struct); free(s); }

void oracle_destroy(oracle_t* o) {
  if (!o) return;
  for (int i = 0; i < o->n_cons; ++i) { free(o->cons[i].dts); free(o->cons[i].ids); free(o->cons[i].acc_T); free(o->cons[i].lin_M); }
  for (int i = 0; i < TOWR_MAX_COSTS; ++i) free(o->soft_b[i]);
  free(o->x);
  spline_free(o->s_lin); spline_free(o->s_ang);
  for (int ee = 0; ee < MAXE; ++ee) {
    spline_free(o->s_motion[ee]); spline_free(o->s_ang_ee[ee]); spline_free(o->s_force[ee]); spline_free(o->s_torque[ee]);
    nv_free(o->motion[ee]); nv_free(o->ang[ee]); nv_free(o->force[ee]); nv_free(o->torque[ee]); free(o->pd[ee]);
  }
  nv_free(o->base_lin); nv_free(o->base_ang);
  sp_free(&o->euler.jac_struct); sp_free(&o->model.I_b);
  free(o);
}


/* =============================================================================================
 * Cost terms (NlpFormulation::GetCosts, nlp_formulation.cc:604-680; towr/src/costs/):
 * IpoptAdapter::eval_f = sum of every term's GetCost, eval_grad_f = the dense sum of their
 * FillJacobianBlock rows.
 * ===========================================================================================*/
/* GetSampleTimes (energy_cost.cc:41-55 and identical copies): t = 0, dt, ... while t <= T + 1e-9,
 * accumulated; T = base_linear_->GetTotalTime() (the sum of the base polynomial durations) */
static int cost_times(const oracle_t* o, double dt, double** out) {
  double T = 0.0;
  for (int i = 0; i < o->s_lin->n_polys; ++i) T += o->s_lin->polys[i].T;
  int cap = dt > 0.0 ? (int)(T / dt) + 4 : 2, n = 0;
  double* ts = (double*)malloc(sizeof(double) * (size_t)cap);
  if (dt <= 0.0) { ts[n++] = 0.0; ts[n++] = T; }
  else for (double t = 0.0; t <= T + 1e-9; t += dt) ts[n++] = t;
  *out = ts;
  return n;
}

/* PhaseDurations::IsContactPhase, phase_durations.cc:120-124 */
static int pd_is_contact(const PhaseDur* p, double t) {
  int id = get_segment_id(t, p->d, p->n);
  return id % 2 == 0 ? p->initial_contact : !p->initial_contact;
}

static const NodesVar* cost_nodes(const oracle_t* o, int kind, int ee) {
  switch (kind) {
    case TOWR_VAR_BASE_LIN: return o->base_lin;
    case TOWR_VAR_BASE_ANG: return o->base_ang;
    case TOWR_VAR_EE_MOTION: return o->motion[ee];
    case TOWR_VAR_EE_ANG: return o->ang[ee];
    case TOWR_VAR_EE_FORCE: return o->force[ee];
    case TOWR_VAR_EE_TORQUE: return o->torque[ee];
  }
  return NULL;
}

static int varset_col0(const oracle_t* o, int kind, int ee) {
  for (int i = 0; i < o->n_vs; ++i) if (vs_is(&o->vs[i], kind, ee)) return o->vs[i].col0;
  return -1;
}

/* grad[col0 + col] += s * J[r][col] for every entry of row r of a 3 x n Jacobian */
static void grad_add_rows(double* grad, int col0, const spmat* J, const double m[3]) {
  if (col0 < 0) return;
  for (int r = 0; r < J->rows; ++r)
    for (int q = 0; q < J->r[r].n; ++q) grad[col0 + J->r[r].e[q].col] += m[r] * J->r[r].e[q].val;
}

/* value of one term, and (grad != NULL) its gradient added into grad */
static double cost_term(oracle_t* o, int ci, double* grad) {
  const towr_cost_t* c = &o->d.costs[ci];
  double cost = 0.0;   /* NodeCost::GetCost leaves its accumulator uninitialised (node_cost.cc:58): 0 here */
  switch (c->kind) {
    case TOWR_COST_NODE: {          /* node_cost.cc:55-79 */
      const NodesVar* v = cost_nodes(o, c->ip[0], c->ee);
      int deriv = c->ip[1], dim = c->ip[2];
      for (int id = 0; id < v->n_nodes; ++id) cost += c->weight * pow(v->nodes[id][deriv][dim], 2);
      int col0 = varset_col0(o, c->ip[0], c->ee);
      if (grad && col0 >= 0) {
        Nvi l[2];
        for (int i = 0; i < v->n_rows; ++i) {
          int nl = nv_info(v, i, l);
          for (int q = 0; q < nl; ++q)
            if (l[q].deriv == deriv && l[q].dim == dim) grad[col0 + i] += c->weight * 2.0 * v->nodes[l[q].id][deriv][dim];
        }
      }
      break;
    }
    case TOWR_COST_ENERGY: {        /* energy_cost.cc:57-152 */
      if (c->weight <= 0.0) break;
      double* ts; int nt = cost_times(o, c->dt, &ts);
      double tw = c->p[0], wdt = c->weight * (c->dt > 0.0 ? c->dt : 1.0);
      for (int k = 0; k < nt; ++k) {
        double inst = 0.0, t = ts[k];
        for (int ee = 0; ee < o->n_ee; ++ee) {
          double f[3][3], tq[3][3];
          spline_point(o->s_force[ee], t, f); spline_point(o->s_torque[ee], t, tq);
          inst += dot3(f[kPos], f[kPos]) + tw * dot3(tq[kPos], tq[kPos]);
          if (!grad) continue;
          double mf[3], mt[3];
          for (int r = 0; r < 3; ++r) { mf[r] = (2.0 * wdt) * f[kPos][r]; mt[r] = (2.0 * wdt * tw) * tq[kPos][r]; }
          spmat J = spline_jac(o->s_force[ee], t, kPos);
          grad_add_rows(grad, varset_col0(o, TOWR_VAR_EE_FORCE, ee), &J, mf); sp_free(&J);
          if (tw != 0.0) { J = spline_jac(o->s_torque[ee], t, kPos); grad_add_rows(grad, varset_col0(o, TOWR_VAR_EE_TORQUE, ee), &J, mt); sp_free(&J); }
          int cs = varset_col0(o, TOWR_VAR_EE_SCHEDULE, ee);
          if (cs >= 0) {
            J = spline_jac_pos_wrt_durations(o->s_force[ee], t); grad_add_rows(grad, cs, &J, mf); sp_free(&J);
            if (tw != 0.0) { J = spline_jac_pos_wrt_durations(o->s_torque[ee], t); grad_add_rows(grad, cs, &J, mt); sp_free(&J); }
          }
        }
        cost += c->weight * inst * (c->dt > 0.0 ? c->dt : 1.0);
      }
      free(ts);
      break;
    }
    case TOWR_COST_ANG_MOMENTUM: {  /* angular_momentum_cost.cc:67-208 (SingleRigidBodyDynamics: true L) */
      if (c->weight <= 0.0) break;
      double* ts; int nt = cost_times(o, c->dt, &ts);
      double wdt = c->weight * (c->dt > 0.0 ? c->dt : 1.0);
      double Ib[3][3];
      { const double* I = o->d.robot.inertia;
        double m9[9] = {I[0], -I[3], -I[4], -I[3], I[1], -I[5], -I[4], -I[5], I[2]};
        memcpy(Ib, m9, sizeof Ib); }
      int col0 = varset_col0(o, TOWR_VAR_BASE_ANG, 0);
      for (int k = 0; k < nt; ++k) {
        double t = ts[k], R[3][3], w[3], RI[3][3], Iw[3][3], v[3];
        eu_R_t(&o->euler, t, R); eu_omega(&o->euler, t, w);
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) RI[i][j] = R[i][0] * Ib[0][j] + R[i][1] * Ib[1][j] + R[i][2] * Ib[2][j];
        for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Iw[i][j] = RI[i][0] * R[j][0] + RI[i][1] * R[j][1] + RI[i][2] * R[j][2];
        for (int i = 0; i < 3; ++i) v[i] = Iw[i][0] * w[0] + Iw[i][1] * w[1] + Iw[i][2] * w[2];
        cost += wdt * dot3(v, v);
        if (!grad || col0 < 0) continue;
        double m[3], u[3], v2[3];
        for (int r = 0; r < 3; ++r) m[r] = (2.0 * wdt) * v[r];
        for (int i = 0; i < 3; ++i) u[i] = R[0][i] * w[0] + R[1][i] * w[1] + R[2][i] * w[2];   /* R^T omega */
        for (int i = 0; i < 3; ++i) v2[i] = Ib[i][0] * u[0] + Ib[i][1] * u[1] + Ib[i][2] * u[2];
        spmat Jrv2 = eu_d_rotvec(&o->euler, t, v2, 0), Jrtw = eu_d_rotvec(&o->euler, t, w, 1), Jw = eu_d_angvel(&o->euler, t);
        int n = Jw.cols;
        double* ta = (double*)calloc((size_t)(3 * n), sizeof(double));
        double* tb = (double*)calloc((size_t)(3 * n), sizeof(double));
        for (int r = 0; r < 3; ++r) {
          for (int q = 0; q < Jrtw.r[r].n; ++q) ta[r * n + Jrtw.r[r].e[q].col] += Jrtw.r[r].e[q].val;
          for (int q = 0; q < Jw.r[r].n; ++q) tb[r * n + Jw.r[r].e[q].col] += Jw.r[r].e[q].val;
        }
        grad_add_rows(grad, col0, &Jrv2, m);
        for (int col = 0; col < n; ++col) {
          double tbc[3], tu[3], it[3], j2[3];
          for (int i = 0; i < 3; ++i) tbc[i] = R[0][i] * tb[0 * n + col] + R[1][i] * tb[1 * n + col] + R[2][i] * tb[2 * n + col];
          for (int i = 0; i < 3; ++i) tu[i] = ta[i * n + col] + tbc[i];
          for (int i = 0; i < 3; ++i) it[i] = Ib[i][0] * tu[0] + Ib[i][1] * tu[1] + Ib[i][2] * tu[2];
          for (int i = 0; i < 3; ++i) j2[i] = R[i][0] * it[0] + R[i][1] * it[1] + R[i][2] * it[2];
          double g2 = m[0] * j2[0] + m[1] * j2[1] + m[2] * j2[2];
          if (g2 != 0.0) grad[col0 + col] += g2;
        }
        free(ta); free(tb); sp_free(&Jrv2); sp_free(&Jrtw); sp_free(&Jw);
      }
      free(ts);
      break;
    }
    case TOWR_COST_EE_BASE_POS: {   /* ee_base_pos_cost.cc:57-162 */
      if (c->weight <= 0.0) break;
      double* ts; int nt = cost_times(o, c->dt, &ts);
      int ee = c->ee;
      for (int k = 0; k < nt; ++k) {
        double t = ts[k];
        if (pd_is_contact(o->pd[ee], t)) continue;   /* only during swing */
        double b[3][3], pe[3][3], R[3][3], rW[3], pB[3], e[3], m[3];
        spline_point(o->s_lin, t, b); spline_point(o->s_motion[ee], t, pe); eu_R_t(&o->euler, t, R);
        for (int q = 0; q < 3; ++q) rW[q] = pe[kPos][q] - b[kPos][q];
        for (int i = 0; i < 3; ++i) pB[i] = R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2];
        for (int i = 0; i < 3; ++i) e[i] = pB[i] - c->p[i];
        cost += c->weight * dot3(e, e);
        if (!grad) continue;
        for (int i = 0; i < 3; ++i) m[i] = (2.0 * c->weight) * e[i];
        double mW[3], mWn[3];
        for (int j = 0; j < 3; ++j) { mW[j] = m[0] * R[j][0] + m[1] * R[j][1] + m[2] * R[j][2]; }   /* m * b_R_w */
        for (int j = 0; j < 3; ++j) { double nm0 = -m[0], nm1 = -m[1], nm2 = -m[2]; mWn[j] = nm0 * R[j][0] + nm1 * R[j][1] + nm2 * R[j][2]; }
        spmat J = spline_jac(o->s_motion[ee], t, kPos); grad_add_rows(grad, varset_col0(o, TOWR_VAR_EE_MOTION, ee), &J, mW); sp_free(&J);
        J = spline_jac(o->s_lin, t, kPos); grad_add_rows(grad, varset_col0(o, TOWR_VAR_BASE_LIN, 0), &J, mWn); sp_free(&J);
        J = eu_d_rotvec(&o->euler, t, rW, 1); grad_add_rows(grad, varset_col0(o, TOWR_VAR_BASE_ANG, 0), &J, m); sp_free(&J);
        /* the schedule block is omitted by the reference (:150-154) */
      }
      free(ts);
      break;
    }
    case TOWR_COST_BASE_HEIGHT: {   /* base_height_cost.cc:55-142 (the fork's biped driver, test/biped_example.cc:199) */
      /* GetCost / FillJacobianBlock: t = 0, dt, ... (accumulated) while t <= T + 1e-9, T = base_linear_->GetTotalTime() */
      double* ts; int nt = cost_times(o, c->dt, &ts);
      const double dt = c->dt, w = c->weight, th = c->p[0];
      int col0 = varset_col0(o, TOWR_VAR_BASE_LIN, 0);
      for (int k = 0; k < nt; ++k) {
        const double t = ts[k];
        double b[3][3]; spline_point(o->s_lin, t, b);
        /* GetSupportPointAverageHeight (:100-125): mean z of the feet in contact, else the terrain
         * height under the base */
        double total = 0.0; int cnt = 0;
        for (int ee = 0; ee < o->n_ee; ++ee)
          if (pd_is_contact(o->pd[ee], t)) { double pe[3][3]; spline_point(o->s_motion[ee], t, pe); total += pe[kPos][Z]; cnt++; }
        const double avg = cnt == 0 ? ter_h(&o->terrain, b[kPos][X], b[kPos][Y]) : total / cnt;
        const double dev = b[kPos][Z] - (avg + th);   /* GetHeightDeviation (:88-98) */
        cost += w * dev * dev * dt;
        if (!grad || col0 < 0) continue;
        /* FillJacobianBlock (:70-86): base-lin only, 2 w dev dt * d p_z / d nodes; the dependence of the
         * target on the feet and the terrain is not differentiated (reference behaviour) */
        spmat J = spline_jac(o->s_lin, t, kPos);
        const double s2 = 2.0 * w * dev * dt;
        for (int q = 0; q < J.r[Z].n; ++q) grad[col0 + J.r[Z].e[q].col] += s2 * J.r[Z].e[q].val;
        sp_free(&J);
      }
      free(ts);
      break;
    }
    case TOWR_COST_SOFT: {          /* soft_constraint.cc:52-69: 0.5 (g-b)^T W (g-b), gradient J^T W (g-b), W = 1 */
      const Cons* w = &o->cons[c->ip[0]];
      const double* b = o->soft_b[ci];
      double* g = (double*)calloc((size_t)(w->rows > 0 ? w->rows : 1), sizeof(double));
      cons_values(o, w, g);
      for (int r = 0; r < w->rows; ++r) { g[r] -= b[r]; cost += (0.5 * g[r]) * g[r]; }
      if (grad)   /* constraint_->GetJacobian(): every variable set's block */
        for (int vi = 0; vi < o->n_vs; ++vi) {
          VarSet* v = &o->vs[vi];
          spmat jac = sp_zero(w->rows, v->n);
          cons_fill_jac(o, w, v, &jac);
          for (int r = 0; r < jac.rows; ++r)
            for (int q = 0; q < jac.r[r].n; ++q) grad[v->col0 + jac.r[r].e[q].col] += jac.r[r].e[q].val * g[r];
          sp_free(&jac);
        }
      free(g);
      break;
    }
  }
  return cost;
}

int oracle_eval_f(oracle_t* o, const double* x, double* f) {
  set_variables(o, x);
  double s = 0.0;
  for (int i = 0; i < o->d.n_costs; ++i) s += cost_term(o, i, NULL);
  *f = s;
  return 0;
}

int oracle_eval_grad_f(oracle_t* o, const double* x, double* grad) {
  set_variables(o, x);
  for (int j = 0; j < o->n; ++j) grad[j] = 0.0;
  for (int i = 0; i < o->d.n_costs; ++i) cost_term(o, i, grad);
  return 0;
}

/* SaveTrajectoryToCSV (save_data.cpp:9-130): rows at t = 0, dt, ... (accumulated) while t <= T + 1e-9,
 * 19 + 25 E columns (include/towr_gpu.h). Returns the sample count; out = NULL only counts. */
int oracle_sample_trajectory(oracle_t* o, const double* x, double dt, double* out) {
  if (!(dt > 0.0)) return -1;
  if (x) set_variables(o, x);
  double T = 0.0;
  for (int i = 0; i < o->s_lin->n_polys; ++i) T += o->s_lin->polys[i].T;
  const int E = o->n_ee, cols = 19 + 25 * E;
  int k = 0;
  for (double t = 0.0; t <= T + 1e-9; t += dt, ++k) {
    if (!out) continue;
    double* row = out + (size_t)k * cols, st[3][3];
    row[0] = t;
    const Spline* base[2] = {o->s_lin, o->s_ang};
    for (int s = 0; s < 2; ++s) {
      spline_point(base[s], t, st);
      for (int d = 0; d < 3; ++d) for (int e = 0; e < 3; ++e) row[1 + 9 * s + 3 * d + e] = st[d][e];
    }
    for (int ee = 0; ee < E; ++ee) {
      double* r = row + 19 + 25 * ee;
      spline_point(o->s_motion[ee], t, st);
      for (int d = 0; d < 3; ++d) for (int e = 0; e < 3; ++e) r[3 * d + e] = st[d][e];
      spline_point(o->s_ang_ee[ee], t, st);
      for (int d = 0; d < 3; ++d) for (int e = 0; e < 3; ++e) r[9 + 3 * d + e] = st[d][e];
      spline_point(o->s_force[ee], t, st);
      for (int e = 0; e < 3; ++e) r[18 + e] = st[kPos][e];
      spline_point(o->s_torque[ee], t, st);
      for (int e = 0; e < 3; ++e) r[21 + e] = st[kPos][e];
      r[24] = pd_is_contact(o->pd[ee], t) ? 1.0 : 0.0;
    }
  }
  return k;
}

int oracle_sizes(oracle_t* o, int* n, int* m) { *n = o->n; *m = o->m; return 0; }

/* ifopt Composite::GetValues over the variable sets */
int oracle_initial_x(oracle_t* o, double* x0) {
  for (int i = 0; i < o->n_vs; ++i) {
    VarSet* v = &o->vs[i];
    if (v->nv) nv_get_values(v->nv, x0 + v->col0);
    else for (int q = 0; q < v->pd->n - 1; ++q) x0[v->col0 + q] = v->pd->d[q];  /* phase_durations.cc:68-77 */
  }
  return 0;
}

int oracle_eval_g(oracle_t* o, const double* x, double* g) {
  set_variables(o, x);
  for (int i = 0; i < o->n_cons; ++i)
    if (o->cons[i].role != TOWR_ROLE_SOFT) cons_values(o, &o->cons[i], g + o->cons[i].row0);
  return g_segment_overflow ? 1 : 0;
}

long oracle_eval_jac(oracle_t* o, const double* x, long cap, int* rows, int* cols, double* vals) {
  set_variables(o, x);
  TripList all = {0, 0, 0};
  build_jacobian(o, &all);
  for (long i = 0; i < all.n && i < cap; ++i) { rows[i] = all.t[i].r; cols[i] = all.t[i].c; vals[i] = all.t[i].v; }
  long n = all.n;
  free(all.t);
  return n;
}

long oracle_eval_jac_values(oracle_t* o, const double* x, double* values) {
  set_variables(o, x);
  TripList all = {0, 0, 0};
  build_jacobian(o, &all);
  for (long i = 0; i < all.n; ++i) values[i] = all.t[i].v;   /* std::copy(valuePtr, ...) */
  long n = all.n;
  free(all.t);
  return n;
}

int oracle_constraint_rows(oracle_t* o, int i, int* row0, int* n_rows) {
  if (i < 0 || i >= o->n_cons) return -1;
  *row0 = o->cons[i].row0; *n_rows = o->cons[i].rows; return 0;
}
int oracle_varset_cols(oracle_t* o, int i, int* col0, int* n_cols) {
  if (i < 0 || i >= o->n_vs) return -1;
  *col0 = o->vs[i].col0; *n_cols = o->vs[i].n; return 0;
}

/* ------------------------------------------------------------------------ CPU baseline ---- */
typedef struct {
  const towr_problem_desc_t* d; int calls, nx; const double* X;
  pthread_barrier_t* start; long done; double* gbuf; double* vbuf;
} BenchArg;

static void* bench_thread(void* p) {
  BenchArg* a = (BenchArg*)p;
  char err[128];
  oracle_t* o = oracle_create(a->d, err, sizeof err);
  if (!o) { pthread_barrier_wait(a->start); pthread_barrier_wait(a->start); return NULL; }
  double* g = (double*)malloc(sizeof(double) * (size_t)o->m);
  long nnz = oracle_eval_jac(o, a->X, 0, NULL, NULL, NULL);
  double* v = (double*)malloc(sizeof(double) * (size_t)(nnz + 16));
  for (int w = 0; w < 2; ++w) { oracle_eval_g(o, a->X, g); oracle_eval_jac_values(o, a->X, v); }  /* warm-up */
  pthread_barrier_wait(a->start);
  for (int i = 0; i < a->calls; ++i) {
    const double* x = a->X + (size_t)(i % a->nx) * (size_t)o->n;
    oracle_eval_g(o, x, g);             /* IpoptAdapter::eval_g      */
    oracle_eval_jac_values(o, x, v);    /* IpoptAdapter::eval_jac_g  */
    a->done++;
  }
  pthread_barrier_wait(a->start);
  free(g); free(v);
  oracle_destroy(o);
  return NULL;
}

static double now_s(void) { struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec + 1e-9 * ts.tv_nsec; }

double oracle_bench(const towr_problem_desc_t* d, int threads, int calls_per_thread, int nx, const double* X, long* calls_done) {
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
  BenchArg* args = (BenchArg*)calloc((size_t)threads, sizeof(BenchArg));
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
  for (int i = 0; i < threads; ++i) {
    args[i].d = d; args[i].calls = calls_per_thread; args[i].nx = nx; args[i].X = X; args[i].start = &bar;
    pthread_create(&th[i], NULL, bench_thread, &args[i]);
  }
  pthread_barrier_wait(&bar);
  double t0 = now_s();
  pthread_barrier_wait(&bar);
  double t1 = now_s();
  long total = 0;
  for (int i = 0; i < threads; ++i) { pthread_join(th[i], NULL); total += args[i].done; }
  pthread_barrier_destroy(&bar);
  free(th); free(args);
  if (calls_done) *calls_done = total;
  return t1 - t0;
}

/* ------------------------------------------------------------- unit-level KAT entry points -- */
/* Hermite polynomial state at t and the 3x4 basis (d{pos,vel,acc}/d{n0.p,n0.v,n1.p,n1.v}),
 * via CubicHermitePolynomial::UpdateCoeff/GetPoint/GetDerivativeWrt{Start,End}Node.           */
void oracle_kat_hermite(double T, double t, const double n0[2], const double n1[2], double state[3], double basis[12]) {
  Poly p; memset(&p, 0, sizeof p);
  p.T = T;
  p.n0[kPos][0] = n0[0]; p.n0[kVel][0] = n0[1]; p.n1[kPos][0] = n1[0]; p.n1[kVel][0] = n1[1];
  poly_update_coeff(&p);
  double st[3][3]; poly_get_point(&p, t, st);
  for (int d = 0; d < 3; ++d) state[d] = st[d][0];
  for (int d = 0; d < 3; ++d) {
    basis[4 * d + 0] = poly_d_start(&p, d, kPos, t); basis[4 * d + 1] = poly_d_start(&p, d, kVel, t);
    basis[4 * d + 2] = poly_d_end(&p, d, kPos, t);   basis[4 * d + 3] = poly_d_end(&p, d, kVel, t);
  }
}
/* d pos / d T of the Hermite polynomial (GetDerivativeOfPosWrtDuration) */
double oracle_kat_hermite_dT(double T, double t, const double n0[2], const double n1[2]) {
  Poly p; memset(&p, 0, sizeof p);
  p.T = T;
  p.n0[kPos][0] = n0[0]; p.n0[kVel][0] = n0[1]; p.n1[kPos][0] = n1[0]; p.n1[kVel][0] = n1[1];
  poly_update_coeff(&p);
  double o[3]; poly_d_pos_wrt_duration(&p, t, o);
  return o[0];
}
/* Euler ZYX: R (row-major), omega = M thd, omega_dot = Mdot thd + M thdd */
void oracle_kat_euler(const double th[3], const double thd[3], const double thdd[3], double R[9], double w[3], double wd[3]) {
  double Rm[3][3]; euler_R(th, Rm); memcpy(R, Rm, sizeof Rm);
  spmat M = eu_M(th), Md = eu_Mdot(th, thd);
  double a[3], b[3];
  sp_mul_vec(&M, thd, w); sp_mul_vec(&Md, thd, a); sp_mul_vec(&M, thdd, b);
  for (int k = 0; k < 3; ++k) wd[k] = a[k] + b[k];
  sp_free(&M); sp_free(&Md);
}
/* RotVecConverter: R = Rodrigues(theta) (row-major), omega = J_L theta_dot, omega_dot = J_L_dot theta_dot + J_L theta_ddot */
void oracle_kat_rotvec(const double th[3], const double thd[3], const double thdd[3], double R[9], double w[3], double wd[3]) {
  double Rm[3][3], J[3][3], Jd[3][3], a[3], b[3];
  rv_rodrigues(th, Rm); memcpy(R, Rm, sizeof Rm);
  rv_left_jac(th, J); rv_left_jac_dot(th, thd, Jd);
  m3_vec(J, thd, w); m3_vec(Jd, thd, a); m3_vec(J, thdd, b);
  for (int k = 0; k < 3; ++k) wd[k] = a[k] + b[k];
}
/* SingleRigidBodyDynamics::GetDynamicViolation for n_ee contacts */
void oracle_kat_srbd(double m, double g, const double inertia[6], int n_ee, const double com[3], const double com_acc[3],
                     const double th[3], const double thd[3], const double thdd[3],
                     const double* f, const double* p, const double* tau, double out[6]) {
  Model M; memset(&M, 0, sizeof M);
  M.m = m; M.g = g; M.n_ee = n_ee;
  const double* I = inertia;
  double Ib[9] = {I[0], -I[3], -I[4], -I[3], I[1], -I[5], -I[4], -I[5], I[2]};
  M.I_b = sp_from_dense(3, 3, Ib, 0);
  memcpy(M.com_pos, com, sizeof(double[3])); memcpy(M.com_acc, com_acc, sizeof(double[3]));
  double R9[9], w[3], wd[3];
  oracle_kat_euler(th, thd, thdd, R9, w, wd);
  memcpy(M.R, R9, sizeof R9); memcpy(M.omega, w, sizeof w); memcpy(M.omega_dot, wd, sizeof wd);
  for (int e = 0; e < n_ee; ++e) for (int k = 0; k < 3; ++k) { M.f[e][k] = f[3 * e + k]; M.p[e][k] = p[3 * e + k]; M.tau[e][k] = tau[3 * e + k]; }
  model_violation(&M, out);
  sp_free(&M.I_b);
}
/* HeightMap: h, dh/dx, dh/dy, normalized basis (3x3, rows n t1 t2), d basis / d{x,y} (2x3x3) */
void oracle_kat_terrain(const towr_terrain_t* T, double x, double y, double out_h[3], double basis[9], double dbasis[18]) {
  out_h[0] = ter_h(T, x, y); out_h[1] = ter_dh(T, X, x, y); out_h[2] = ter_dh(T, Y, x, y);
  for (int b = 0; b < 3; ++b) ter_nbasis(T, b, x, y, basis + 3 * b);
  for (int d = 0; d < 2; ++d) for (int b = 0; b < 3; ++b) ter_d_nbasis(T, b, d, x, y, dbasis + 9 * d + 3 * b);
}
