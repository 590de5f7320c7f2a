// engine_math.h — per-work-item evaluation of towr's constraint values and Jacobian entries.
//
// Single source for two instantiations:
//   * device (towr_gpu.hip): the fused eval kernel, Emit = LDS accumulator indexed by slot table;
//   * host   (layout.hip):   the structure pass at the starting point x0, Emit = recorder of the
//                            (row, col) of every candidate entry (IPOPT's eval_jac_g(values=NULL)).
// The host instantiation's values are discarded; g/J values are only ever produced on the GPU.
//
// A "work item" is one (constraint set, instance, group) triple. Each item emits its g rows and an
// ordered list of Jacobian candidates (row, col, value, present). The ORDER of candidates is the
// contract between the two instantiations: candidate j of an item lands in slot_table[item.slot + j].
//
// Math follows the reference formulas (file:line cited per function); Jacobians are formed by the
// chain rule through the cubic-Hermite basis (polynomial.cc:135-214), which is exactly the
// structure the reference builds with NodeSpline::GetJacobianWrtNodes + Eigen sparse products.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/towr_gpu.h"

#define TG_HD __host__ __device__ __forceinline__

namespace tg {

enum { kPos = 0, kVel = 1, kAcc = 2 };

enum { X = 0, Y = 1, Z = 2 };
enum { AX = 0, AY = 1, AZ = 2, LX = 3, LY = 4, LZ = 5 };

// spline ids: 0 base-lin, 1 base-ang, 2 + 4*ee + {0 motion, 1 ang, 2 force, 3 torque}
enum { SP_BASE_LIN = 0, SP_BASE_ANG = 1 };
TG_HD int sp_motion(int ee) { return 2 + 4 * ee + 0; }
TG_HD int sp_force(int ee)  { return 2 + 4 * ee + 2; }
TG_HD int sp_torque(int ee) { return 2 + 4 * ee + 3; }
TG_HD int sp_ang(int ee)    { return 2 + 4 * ee + 1; }

// work item types
enum ItemType {
  IT_NONE = -1,  // padding lane of a tile
  IT_DYN = 0,    // DynamicConstraint instant; group 0: base-lin + g, 1: base-ang, 2+ee: ee blocks
  IT_ROM = 1,    // RangeOfMotionConstraint instant; group 0: base-lin + g, 1: base-ang, 2: motion
  IT_FDISC = 2,  // ForceConstraintDiscretized instant
  IT_FNODE = 3,  // ForceConstraint node
  IT_TERR = 4,   // TerrainConstraint node
  IT_BMOT = 5,   // BaseMotionConstraint instant
  IT_SACC = 6,   // SplineAccConstraint junction
  IT_BHGT = 7,   // BaseHeightConstraint node
  IT_SWING = 8,  // SwingConstraint node
  IT_TDUR = 9,   // TotalDurationConstraint (phase-duration optimisation)
  IT_TQDISC = 10,  // TorqueConstraintDiscretized instant
  IT_TQNODE = 11,  // TorqueConstraint node (a0 torque node, a1 motion node / a2 torque node at phase start)
  IT_THARD = 12,   // TerrainConstraintHard instant
  IT_EELIN = 13,   // EELinearConstraint instant (a0 = definition index)
  IT_LINEQ = 14,   // LinearEqualityConstraint row (a0 = first LinNz entry, a1 = entries)
  IT_COUNT = 15
};

struct SplineMeta {
  int32_t node_off;  // first node's index into nodecol (6 ints per node: [deriv][dim])
  int32_t n_polys;
  int32_t dur_off;   // first polynomial duration in the durations table
  // PhaseSpline (phase-duration optimisation, phase_spline.cc:35-93): durations come from the
  // ee's schedule variables and the Jacobian keeps the full pattern of every polynomial
  int32_t ee;        // endeffector of a PhaseSpline, else -1
  int32_t pinfo_off; // first PolyPhase of this spline
  int32_t pcol_off[3], pcol_n[3];   // PhaseCol entries of each dimension (the full pattern)
  int32_t pact_off;  // PhaseSpline: active PhaseCol range of each (dim, polynomial), see Ctx::pact
};

// phase of a polynomial (NodesVariablesPhaseBased::PolyInfo, nodes_variables_phase_based.cc:39-59)
struct PolyPhase { int16_t phase, poly_in_phase, n_in_phase, spl; };   // spl: the spline whose polynomial it is

// one column of a PhaseSpline's full Jacobian pattern in one dimension: the optimisation variable
// and the (1 or 2) node values it sets (a stance variable sets two nodes)
struct PhaseCol {
  int32_t col;
  int16_t id[2];
  int8_t deriv[2];
  int8_t n, reserved;
};

// PhaseDurations of one endeffector (phase_durations.cc:41-100): the first n_phases - 1 durations
// are the variables at col0.., the last is t_total minus their sum
struct SchedInfo { int32_t col0, n_phases; double t_total; };

// EELinearConstraint definition (ee_linear_constraint.cc:5-48): sum of coeff * (pos|vel)[dim] of the
// ee motion (target 0) or ee angle (target 1) splines; terms on one (ee, dim) are merged
struct EELinDef {
  int32_t target, deriv, n, reserved;
  int32_t code[6];   // ee * 3 + dim
  double coeff[6];
};

// LinearEqualityConstraint (linear_constraint.cc:35-80): the nonzeros of one row of M, by column
struct LinNz { int32_t col, reserved; double v; };

struct RobotC {
  double m, g;
  double Ib[9];      // BuildInertiaTensor (single_rigid_body_dynamics.cc:36-44), row-major
  int32_t n_ee, reserved;
};

// 64-byte work-item descriptor, shared by all problems of a batch
struct ItemDesc {
  int32_t type, group, ee, k;   // k: instance index inside the constraint set
  int32_t row0;                 // global row of the item's first row
  int32_t a0, a1;               // node ids (FNODE: force node, motion node at phase start; ...)
  int32_t slot;                 // candidate j of this item is slot_table[slot + j * stride]
  int32_t seg;                  // row of the segment table (time-discretised items), else -1
  int32_t ncand;                // number of candidates the item emits
  int32_t a2;                   // third node id (TorqueConstraint: torque node at phase start)
  int32_t rsel;                 // row select: 0 = the item emits all its rows' candidates, else it emits
                                // only rows row0 + rsel_first .. + rsel_count - 1 (phase-duration
                                // optimisation splits the heavy PhaseSpline items over lanes, see
                                // layout.h split_rows); encoding 1 + first + 16 count + 256 part
  double t;                     // time of the instant (time-discretised sets)
  double p0;                    // scalar parameter (safety distance, t_swing_avg, ...)
};

// Direct CSR positions of a lane's candidates (phase-duration optimisation, TileEmit DIRECT): for up
// to two variable-set column ranges [c0, c1) the lane's candidates sit at tile-relative position
// off + col (the row holds the set's columns contiguously: FDISC force and schedule blocks, RangeOfMotion
// motion and schedule blocks), so they need no slot-table load; other candidates use the slot table.
// [z0, z1): the tile-relative CSR range of the rows this lane owns whole (row-split FDISC / TQDISC
// lanes), which its wave zero-fills itself; else empty.
struct alignas(16) ItemDirect { int32_t c0[2], c1[2], off[2], z0, z1; };

// Spline::GetLocalTime result of one spline at one instant (precomputed on the host for fixed
// polynomial durations: the reference's scan, spline.cc:48-78, run once at setup)
struct SegRec {
  double tl, T;
  int32_t poly, reserved;
  double H[3][4];   // d{pos,vel,acc}(tl)/d{n0.p, n0.v, n1.p, n1.v}: batch-invariant Hermite basis
  int32_t col[4][3];   // x column of basis value b, dim e (device numbering: a constant node -> n, x[n] = 0)
};

// Slot table entry: 8 tile-relative LDS positions (uint16) of one lane's candidates 8g..8g+7, one
// 16-byte load per lane; group g of lane l of a tile sits at tile_base + g * block + l (a wave's
// load is one coalesced 1 KiB access). A present candidate's position is its CSR position minus
// the tile's first; an absent one's is the lane's dummy slot past the tile's values.
struct alignas(16) SlotGroup { uint32_t w[4]; };
constexpr int kSlotAbsent = 0xFFFF;
TG_HD int slot_pick(const SlotGroup& q, int k) {   // select chain: k may be a runtime value
  const uint32_t lo = (k & 2) ? q.w[1] : q.w[0], hi = (k & 2) ? q.w[3] : q.w[2];
  const uint32_t w = (k & 4) ? hi : lo;
  return (k & 1) ? (int)(w >> 16) : (int)(w & 0xFFFFu);
}

// No item emits the same column twice: contributions to one variable (the two nodes of a stance
// polynomial sharing one variable, the junction node of SplineAcc) are summed into one candidate
// before emission and the other candidate is marked absent (checked at build time), so every CSR
// position receives exactly one plain store.

// Device copy of the segment table in blocks of 32 rows (array of structures of arrays): for
// spline s and rows 32G..32G+31, one block of doubles [tl | T | H(d, b) x 12] and one block of
// ints [poly | col(b, e) x 12], each field 32 entries long. The lanes of a wave (consecutive
// instants) then read one field with one coalesced access, and every field of a row is an
// immediate offset (< 4 KiB) from the row's two base addresses.
constexpr int kSegGroup = 32;
constexpr int kSegDoubles = 14;   // tl, T, H[12]
constexpr int kSegInts = 13;      // poly, col[12]
struct SegSoA {
  const double* d;       // [(s * ng + G) * 14 * 32]
  const int32_t* i;      // [(s * ng + G) * 13 * 32]
  int32_t ng, reserved;  // 32-row groups
};

struct Ctx {
  const SegRec* seg;            // host: this item's segment row (one SegRec per spline), or nullptr
  SegSoA sg;                    // device: the segment table
  int32_t row;                  // device: this item's segment row, or -1
  const double* x;              // this problem's decision vector
  const int32_t* nodecol;       // node value -> global column of x, or -1 (constant 0)
  const SplineMeta* spl;
  const double* dur;            // polynomial durations
  const towr_terrain_t* ter;    // this problem's terrain
  RobotC rb;
  int32_t fdisc_motion;         // ForceConstraintDiscretized motion block enabled (terrain has d2h)
  bool gait;                    // phase-duration optimisation (a compile-time constant in kernels)
  bool rotvec;                  // Parameters::RotationVector base orientation (compile-time in kernels)
  double* dyn_scratch;          // device DYN tiles: per-instant endeffector terms (see dyn_g0_a), else nullptr
  const PolyPhase* pinfo;
  const PhaseCol* pcols;
  const int32_t* pact;          // PhaseSpline: [qa, qb] PhaseCol index range (within the dim's list) whose
                                // columns polynomial p touches, at pact[spl.pact_off + 2 (e n_polys + p)]
  const SchedInfo* sched;       // per endeffector
  const EELinDef* eelin;        // EELinearConstraint definitions
  const LinNz* lin;             // LinearEqualityConstraint rows (IT_LINEQ)
  const double* cq;             // cost kernel: CT_ENERGYQ Gram matrices (16 doubles each)
  // Device tile blocks under phase-duration optimisation: the x-dependent PhaseSpline timings,
  // computed once per block (gait_timings in towr_gpu.hip) with the same operations in the same order
  // as the per-call code below, so every lane reads bit-identical values: per PolyPhase entry the
  // polynomial duration (pdur) and the running sum of durations up to its end (pend); per endeffector
  // the running sum of phase durations up to each phase's end (phend, stride ph_stride).
  // nullptr: computed per call.
  const double* pdur = nullptr;
  const double* pend = nullptr;
  const double* phend = nullptr;
  int32_t ph_stride = 0;
};

// ----------------------------------------------------------------------------------------------
// cubic Hermite polynomial (towr/src/helpers/polynomial.cc)
// ----------------------------------------------------------------------------------------------
struct SplinePt {
  int poly;
  double T, tl;
  const double* H;   // device: basis of this instant, entry (d, b) at H[(4 * d + b) * hs]; else nullptr
  const int32_t* C;  // device: x columns of this instant, entry (b, e) at C[(3 * b + e) * kSegGroup]
  bool dyn;          // PhaseSpline: durations (hence polynomial, local time, basis) depend on x
  double p[3], v[3], a[3];
};

// Spline::GetSegmentID + GetLocalTime (spline.cc:48-78): eps = 1e-10, junction -> previous poly
TG_HD int seg_lookup(const double* d, int n, double tg, double* tl) {
  const double eps = 1e-10;
  double t = 0.0;
  int id = n - 1;   // the reference falls off an assert here; clamp to the last polynomial
  for (int i = 0; i < n; ++i) {
    t += d[i];
    if (t >= tg - eps) { id = i; break; }
  }
  double l = tg;
  for (int i = 0; i < id; ++i) l -= d[i];
  *tl = l;
  return id;
}

// x value of a node-value column; -1 = a constant node value (0). The device's staged x carries a
// zero at index n and its node tables point constant values there, so its loads need no branch.
TG_HD double xval(const Ctx& c, int col) {
#if defined(__HIP_DEVICE_COMPILE__)
  return c.x[col];
#else
  return col >= 0 ? c.x[col] : 0.0;
#endif
}
TG_HD int node_col(const Ctx& c, int s, int node, int deriv, int dim) {
  return c.nodecol[(c.spl[s].node_off + node) * 6 + deriv * 3 + dim];
}
// column of Hermite basis function b (0 n0.p, 1 n0.v, 2 n1.p, 3 n1.v) of polynomial `poly`, dim e
TG_HD int basis_col(const Ctx& c, int s, int poly, int b, int e) {
  return node_col(c, s, poly + (b >> 1), b & 1, e);
}

// x^k for small k, correctly rounded like the std::pow of the reference's host build: a double-double
// product on the device (the device pow is not correctly rounded). Used where the reference's
// formulas cancel (polynomial state, d pos / d duration), so that the engine reproduces them.
TG_HD double cpow(double x, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
  // no contraction: the double-double steps are exact only as written (p + e with p = hi * x contracted to
  // fma(hi, x, e) changes the result, and whether the compiler contracts it depended on the kernel cpow was inlined
  // into: the fused FDISC kernel and the record kernel gave force velocities 1 ulp apart)
#pragma clang fp contract(off)
  if (k == 0) return 1.0;
  double hi = x, lo = 0.0;
  for (int i = 1; i < k; ++i) {
    const double p = hi * x;
    double e = fma(hi, x, -p);
    e = fma(lo, x, e);
    hi = p + e;
    lo = e - (hi - p);
  }
  return hi;
#else
  return pow(x, k);
#endif
}

// GetDerivativeOf{Pos,Vel,Acc}Wrt{Start,End}Node (polynomial.cc:140-234); b = 0 n0.p, 1 n0.v, 2 n1.p, 3 n1.v.
// The reference's operations: std::pow powers (cpow), no contraction. At a polynomial's end a basis function
// vanishes only up to rounding, and the residue, times a large scale, is an entry the reference emits; the
// host precomputes the fixed-duration bases (SegRec) with these, so they are the reference's bit for bit.
TG_HD void hermite_dpos(double T, double t, double H[4]) {
#pragma clang fp contract(off)
  const double T2 = cpow(T, 2), T3 = cpow(T, 3), t2 = cpow(t, 2), t3 = cpow(t, 3);
  H[0] = (2 * t3) / T3 - (3 * t2) / T2 + 1;
  H[1] = t - (2 * t2) / T + t3 / T2;
  H[2] = (3 * t2) / T2 - (2 * t3) / T3;
  H[3] = t3 / T2 - t2 / T;
}
TG_HD void hermite_dvel(double T, double t, double H[4]) {
#pragma clang fp contract(off)
  const double T2 = cpow(T, 2), T3 = cpow(T, 3), t2 = cpow(t, 2);
  H[0] = (6 * t2) / T3 - (6 * t) / T2;
  H[1] = (3 * t2) / T2 - (4 * t) / T + 1;
  H[2] = (6 * t) / T2 - (6 * t2) / T3;
  H[3] = (3 * t2) / T2 - (2 * t) / T;
}
TG_HD void hermite_dacc(double T, double t, double H[4]) {
#pragma clang fp contract(off)
  const double T2 = cpow(T, 2), T3 = cpow(T, 3);
  H[0] = (12 * t) / T3 - 6 / T2;
  H[1] = (6 * t) / T2 - 4 / T;
  H[2] = 6 / T2 - (12 * t) / T3;
  H[3] = (6 * t) / T2 - 2 / T;
}

// one dimension of poly_state from the polynomial's node values (n0.p, n0.v, n1.p, n1.v)
TG_HD void poly_state_dim(double p0, double v0, double p1, double v1, double T, double tl, double& pp, double& vv, double& aa) {
#pragma clang fp contract(off)
  const double cf[4] = {p0, v0, -(3 * (p0 - p1) + T * (2 * v0 + v1)) / cpow(T, 2),
                        (2 * (p0 - p1) + T * (v0 + v1)) / cpow(T, 3)};
  pp = 0.0; vv = 0.0; aa = 0.0;
  for (int k = 0; k < 4; ++k) pp += cpow(tl, k) * cf[k];
  for (int k = 0; k < 4; ++k) vv += (k >= 1 ? k * cpow(tl, k - 1) : 0.0) * cf[k];
  for (int k = 0; k < 4; ++k) aa += (k >= 2 ? k * (k - 1) * cpow(tl, k - 2) : 0.0) * cf[k];
}
TG_HD void poly_state(const Ctx& c, int s, int poly, double T, double tl, SplinePt& o) {
  // The reference's own operation order (std::pow, sum over coefficients), on the host and the
  // device alike: data-dependent structure predicates (ForceConstraintDiscretized's `scale == 0.0`,
  // force_constraint_discretized.cc:58) must resolve floating-point ties as the source does, and
  // near-zero velocities of PhaseSplines enter the duration derivatives.
  for (int e = 0; e < 3; ++e) {
    const double p0 = xval(c, node_col(c, s, poly, kPos, e)), v0 = xval(c, node_col(c, s, poly, kVel, e));
    const double p1 = xval(c, node_col(c, s, poly + 1, kPos, e)), v1 = xval(c, node_col(c, s, poly + 1, kVel, e));
    poly_state_dim(p0, v0, p1, v1, T, tl, o.p[e], o.v[e], o.a[e]);
  }
}

// PhaseDurations::GetPhaseDurations after SetVariables (phase_durations.cc:79-100)
TG_HD double phase_duration(const Ctx& c, const SchedInfo& si, double last, int ph) {
  return ph < si.n_phases - 1 ? c.x[si.col0 + ph] : last;
}
TG_HD double last_phase_duration(const Ctx& c, const SchedInfo& si) {
  double sum = 0.0;
  for (int i = 0; i < si.n_phases - 1; ++i) sum += c.x[si.col0 + i];   // x.sum()
  return si.t_total - sum;
}
// polynomial duration of a PhaseSpline: phase duration / polynomials in the phase
// (ConvertPhaseToPolyDurations, nodes_variables_phase_based.cc:75-86)
TG_HD double phase_poly_duration(const Ctx& c, const SplineMeta& m, const SchedInfo& si, double last, int i) {
  const PolyPhase pp = c.pinfo[m.pinfo_off + i];
  return phase_duration(c, si, last, pp.phase) / pp.n_in_phase;
}
// The block-shared PhaseSpline timings of Ctx::pdur / pend / phend, by the per-call code's own
// operations: spline s's polynomial durations and their running sums (phase_spline_locate's scan),
// endeffector ee's running sums of phase durations (sched_jac's scan).
TG_HD void phase_spline_timings(const Ctx& c, int s, double* pdur, double* pend) {
  const SplineMeta m = c.spl[s];
  const SchedInfo si = c.sched[m.ee];
  const double last = last_phase_duration(c, si);
  double t = 0.0;
  for (int i = 0; i < m.n_polys; ++i) {
    const double d = phase_poly_duration(c, m, si, last, i);
    t += d;
    pdur[m.pinfo_off + i] = d;
    pend[m.pinfo_off + i] = t;
  }
}
TG_HD void phase_end_timings(const Ctx& c, int ee, double* phend) {
  const SchedInfo si = c.sched[ee];
  const double last = last_phase_duration(c, si);
  double acc = 0.0;
  for (int ph = 0; ph < si.n_phases; ++ph) {
    acc += phase_duration(c, si, last, ph);
    phend[ph] = acc;
  }
}
// Spline::GetSegmentID + GetLocalTime (spline.cc:48-78) over precomputed polynomial durations d[np] and their running
// sums e[np] (Ctx::pdur / pend): the first polynomial whose end is at or past tg - eps (else the last), and tg minus
// the durations before it, subtracted in order. The operands are loaded 8 at a time ahead of the comparisons / the
// dependent subtractions (one LDS round trip per 8 polynomials instead of one per polynomial).
TG_HD void locate_poly(const double* d, const double* e, int np, double tg, int& poly, double& tl, double& T) {
  const double eps = 1e-10, thr = tg - eps;
  int id = np - 1;
  for (int i0 = 0; i0 < np; i0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i0 + k < np ? e[i0 + k] : 0.0;
    int f = -1;
#pragma unroll
    for (int k = 7; k >= 0; --k)
      if (i0 + k < np && v[k] >= thr) f = k;   // the first entry of the group at or past tg - eps
    if (f >= 0) { id = i0 + f; break; }
  }
  double l = tg;
  for (int i0 = 0; i0 < id; i0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i0 + k < id ? d[i0 + k] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i0 + k < id) l -= v[k];
  }
  poly = id;
  tl = l;
  T = d[id];
}
// PhaseDurations' GetSegmentID over the running sums of phase durations pe[n] (Ctx::phend): the first phase whose end
// is at or past t - eps, else the last (loaded 8 at a time, as locate_poly)
TG_HD int phase_cur(const double* pe, int n, double t) {
  const double eps = 1e-10, thr = t - eps;
  for (int p0 = 0; p0 < n; p0 += 8) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = p0 + k < n ? pe[p0 + k] : 0.0;
    int f = -1;
#pragma unroll
    for (int k = 7; k >= 0; --k)
      if (p0 + k < n && v[k] >= thr) f = k;
    if (f >= 0) return p0 + f;
  }
  return n - 1;
}

// Spline::GetLocalTime (spline.cc:48-78) over the x-dependent durations of a PhaseSpline
TG_HD void phase_spline_locate(const Ctx& c, int s, double tg, SplinePt& o) {
  if (c.pdur) {   // the block's precomputed durations and running sums (see Ctx::pdur)
    const int off = c.spl[s].pinfo_off;
    locate_poly(c.pdur + off, c.pend + off, c.spl[s].n_polys, tg, o.poly, o.tl, o.T);
    return;
  }
  const SplineMeta m = c.spl[s];
  const SchedInfo si = c.sched[m.ee];
  const double last = last_phase_duration(c, si), eps = 1e-10;
  double t = 0.0;
  int id = m.n_polys - 1;
  for (int i = 0; i < m.n_polys; ++i) {
    t += phase_poly_duration(c, m, si, last, i);
    if (t >= tg - eps) { id = i; break; }
  }
  double l = tg;
  for (int i = 0; i < id; ++i) l -= phase_poly_duration(c, m, si, last, i);
  o.poly = id;
  o.tl = l;
  o.T = phase_poly_duration(c, m, si, last, id);
}

TG_HD void spline_eval(const Ctx& c, int s, double t, SplinePt& o) {
  o.dyn = false;
  if (c.gait && c.spl[s].ee >= 0) {
    o.dyn = true;
    o.H = nullptr;
    phase_spline_locate(c, s, t, o);
    poly_state(c, s, o.poly, o.T, o.tl, o);
    return;
  }
#if defined(__HIP_DEVICE_COMPILE__)
  const size_t blk = (size_t)s * c.sg.ng + (c.row >> 5);
  const double* D = c.sg.d + blk * (kSegDoubles * kSegGroup) + (c.row & 31);
  const int32_t* I = c.sg.i + blk * (kSegInts * kSegGroup) + (c.row & 31);
  o.poly = I[0]; o.tl = D[0]; o.T = D[kSegGroup];
  o.H = D + 2 * kSegGroup;
  o.C = I + kSegGroup;
  const double* H = o.H;
  const int32_t* C = o.C;
  constexpr int G = kSegGroup;
  for (int e = 0; e < 3; ++e) {
    const double u0 = c.x[C[(0 + e) * G]], u1 = c.x[C[(3 + e) * G]], u2 = c.x[C[(6 + e) * G]], u3 = c.x[C[(9 + e) * G]];
    o.p[e] = H[0 * G] * u0 + H[1 * G] * u1 + H[2 * G] * u2 + H[3 * G] * u3;
    o.v[e] = H[4 * G] * u0 + H[5 * G] * u1 + H[6 * G] * u2 + H[7 * G] * u3;
    o.a[e] = H[8 * G] * u0 + H[9 * G] * u1 + H[10 * G] * u2 + H[11 * G] * u3;
  }
#else
  o.H = nullptr;
  if (c.seg) {
    const SegRec& r = c.seg[s];
    o.poly = r.poly; o.tl = r.tl; o.T = r.T;
  } else {
    const SplineMeta m = c.spl[s];
    o.poly = seg_lookup(c.dur + m.dur_off, m.n_polys, t, &o.tl);
    o.T = c.dur[m.dur_off + o.poly];
  }
  poly_state(c, s, o.poly, o.T, o.tl, o);
#endif
}

// Hermite basis of a spline point for derivative d (precomputed on the device, evaluated on the host)
TG_HD void spline_basis(const SplinePt& o, int d, double H[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (!o.dyn) {
    for (int b = 0; b < 4; ++b) H[b] = o.H[(4 * d + b) * kSegGroup];
    return;
  }
#endif
  if (d == kPos) hermite_dpos(o.T, o.tl, H);
  else if (d == kVel) hermite_dvel(o.T, o.tl, H);
  else hermite_dacc(o.T, o.tl, H);
}

// Emitters that write into zero-filled outputs declare `static constexpr bool kSparse = true` and
// `skip(k)` (advance past k candidates whose value is 0); emit_dim then emits only the nonzero window
// of a PhaseSpline's full pattern. The structure pass and the test emulation emit every candidate.
template <class E, class = void> struct emit_sparse { static constexpr bool value = false; };
template <class E> struct emit_sparse<E, decltype((void)E::kSparse)> { static constexpr bool value = E::kSparse; };

TG_HD int rsel_first(int rsel) { return (rsel - 1) & 15; }
TG_HD int rsel_count(int rsel) { return ((rsel - 1) >> 4) & 15; }
TG_HD int rsel_part(int rsel) { return (rsel - 1) >> 8; }
// rows of part `part` of an item's `rows` rows split over `parts` lanes: part 0 takes the first
// rows - parts + 1 rows, every other part one row
TG_HD void split_part_rows(int rows, int parts, int part, int& first, int& count) {
  const int lead = rows - parts + 1;
  first = part == 0 ? 0 : lead + part - 1;
  count = part == 0 ? lead : 1;
}

// Emitters that evaluate only some rows of an item (row-split items, ItemDesc::rsel) declare
// `static constexpr bool kFilter = true` and `want(row)`; their operator() drops the other rows'
// candidates itself, and emit_dim skips such rows' full-pattern work before it starts.
template <class E, class = void> struct emit_filter { static constexpr bool value = false; };
template <class E> struct emit_filter<E, decltype((void)E::kFilter)> { static constexpr bool value = E::kFilter; };

// Emitters that evaluate only part of Dynamic's groups declare `static constexpr int kDynGroups`:
// 1 = every group but the base-angular block (group 1), 2 = group 1 only (eval_dyn returns early for
// the others, so the kernel instantiating it carries only those groups' registers).
template <class E, class = void> struct emit_dyn_groups { static constexpr int value = 0; };
template <class E> struct emit_dyn_groups<E, decltype((void)E::kDynGroups)> { static constexpr int value = E::kDynGroups; };

template <class E> TG_HD bool em_wants(const E& em, int row) {
  if constexpr (emit_filter<E>::value) return em.want(row);
  else return true;
}

// scale * d{P's derivative}(spline s)/dx restricted to dimension e, into `row`, given the basis H:
//   NodeSpline: the 4 basis columns of the active polynomial (node_spline.cc:62-112);
//   PhaseSpline: every column of the set in dimension e (the full pattern, phase_spline.cc:45-51,
//   kept through Eigen's products), non-zero only at the active polynomial's two nodes.
template <class Emit>
TG_HD void emit_dim(const Ctx& c, Emit& em, int row, int s, const SplinePt& P, const double H[4], int e, double scale,
                    bool pres = true) {
  if constexpr (emit_filter<Emit>::value)
    if (!em.want(row)) return;
  if (!P.dyn) {
    int col[4];
    for (int bb = 0; bb < 4; ++bb) col[bb] = basis_col(c, s, P.poly, bb, e);
    // a stance polynomial whose two nodes share one position variable (NodesVariablesPhaseBased,
    // nodes_variables_phase_based.cc:215-258): coeffRef sums both contributions into one entry
#if defined(__HIP_DEVICE_COMPILE__)
    const bool shared = P.C[e * kSegGroup] == P.C[(2 * 3 + e) * kSegGroup];   // both constant -> both absent anyway
#else
    const bool shared = col[0] >= 0 && col[0] == col[2];
#endif
    em(row, col[0], scale * (shared ? H[0] + H[2] : H[0]), pres && col[0] >= 0);
    em(row, col[1], scale * H[1], pres && col[1] >= 0);
    em(row, col[2], scale * H[2], pres && col[2] >= 0 && !shared);
    em(row, col[3], scale * H[3], pres && col[3] >= 0);
    return;
  }
  const SplineMeta m = c.spl[s];
  const PhaseCol* pc = c.pcols + m.pcol_off[e];
  const int n = m.pcol_n[e];
  // the basis as opaque registers: the compiler otherwise turns the selects below into a load
  // H[runtime index], which keeps H in scratch memory on the device
  double h0 = H[0], h1 = H[1], h2 = H[2], h3 = H[3];
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
#endif
  if constexpr (emit_sparse<Emit>::value) {
    // An emitter over a zero-filled output (the device tiles, the gradient) only needs the columns
    // the active polynomial touches: every other column of the full pattern is exactly 0.
    const int32_t* r = c.pact + m.pact_off + 2 * (e * m.n_polys + P.poly);
    const int qa = r[0], qb = r[1];
    em.skip(qa);
    for (int q = qa; q <= qb; ++q) {
      const PhaseCol pq = pc[q];
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < 2; ++k) {   // constant indices: a runtime-indexed pq.id / deriv would go to scratch
        if (k >= pq.n) break;
        if (pq.id[k] == P.poly) v += pq.deriv[k] ? h1 : h0;
        else if (pq.id[k] == P.poly + 1) v += pq.deriv[k] ? h3 : h2;
      }
      em(row, pq.col, scale * v, pres);
    }
    em.skip(n - 1 - (qb >= qa ? qb : qa - 1));
    return;
  }
  for (int q = 0; q < n; ++q) {
    const PhaseCol pq = pc[q];
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // coeffRef += per node value the variable sets
      if (k >= pq.n) break;
      if (pq.id[k] == P.poly) v += pq.deriv[k] ? h1 : h0;
      else if (pq.id[k] == P.poly + 1) v += pq.deriv[k] ? h3 : h2;
    }
    em(row, pq.col, scale * v, pres);
  }
}

// d pos(t) / d schedule of a PhaseSpline: PhaseSpline::GetJacobianOfPosWrtDurations
// (phase_spline.cc:67-93) with PhaseDurations::GetJacobianOfPos (phase_durations.cc:126-154).
// J[k][col] over the endeffector's n_phases - 1 schedule variables is dense (sparseView(1, -1)).
struct SchedJac { int cur, n, col0; double dx[3], v[3]; };
// one dimension of J.dx: CubicHermitePolynomial::GetDerivativeOfPosWrtDuration (polynomial.cc:236-257) of the polynomial
// with node values x0, v0, x1, v1, duration T, local time tl, minus the polynomial's share of the velocity vk
// (phase_spline.cc:67-93: inner = 1 / polynomials in the phase, prev = the polynomial's index in the phase)
TG_HD double sched_dx_dim(double x0, double v0, double x1, double v1, double T, double tl, double vk, const PolyPhase& pp) {
#pragma clang fp contract(off)
  const double inner = 1. / pp.n_in_phase, prev = pp.poly_in_phase;
  const double t2 = cpow(tl, 2), t3 = cpow(tl, 3), T2 = cpow(T, 2), T3 = cpow(T, 3), T4 = cpow(T, 4);
  const double dxdT = (t3 * (v0 + v1)) / T3 - (t2 * (2 * v0 + v1)) / T2 - (3 * t3 * (2 * x0 - 2 * x1 + T * v0 + T * v1)) / T4 +
                      (2 * t2 * (3 * x0 - 3 * x1 + 2 * T * v0 + T * v1)) / T3;
  return inner * (dxdT - prev * vk);
}
TG_HD void sched_jac(const Ctx& c, int s, double t, const SplinePt& P, SchedJac& J) {
  const SplineMeta m = c.spl[s];
  const SchedInfo si = c.sched[m.ee];
  const PolyPhase pp = c.pinfo[m.pinfo_off + P.poly];
  for (int k = 0; k < 3; ++k) {
    const double x0 = xval(c, node_col(c, s, P.poly, kPos, k)), v0 = xval(c, node_col(c, s, P.poly, kVel, k));
    const double x1 = xval(c, node_col(c, s, P.poly + 1, kPos, k)), v1 = xval(c, node_col(c, s, P.poly + 1, kVel, k));
    J.dx[k] = sched_dx_dim(x0, v0, x1, v1, P.T, P.tl, P.v[k], pp);
    J.v[k] = P.v[k];
  }
  const double eps = 1e-10;   // GetSegmentID over the phases
  J.cur = si.n_phases - 1;
  if (c.phend) {   // the block's running sums
    J.cur = phase_cur(c.phend + m.ee * c.ph_stride, si.n_phases, t);
  } else {
    const double last = last_phase_duration(c, si);
    double acc = 0.0;
    for (int ph = 0; ph < si.n_phases; ++ph) {
      acc += phase_duration(c, si, last, ph);
      if (acc >= t - eps) { J.cur = ph; break; }
    }
  }
  J.n = si.n_phases;
  J.col0 = si.col0;
}
TG_HD double sched_val(const SchedJac& J, int k, int col) {
  const bool last = J.cur == J.n - 1;
  if (col == J.cur && !last) return J.dx[k];
  if (col < J.cur) return last ? -J.v[k] - J.dx[k] : -J.v[k];
  return 0.0;
}

// ----------------------------------------------------------------------------------------------
// Euler ZYX (towr/src/helpers/euler_converter.cc)
// ----------------------------------------------------------------------------------------------
struct Trig { double sx, cx, sy, cy, sz, cz; };
TG_HD Trig trig(const double a[3]) {
  Trig r;
#if defined(__HIP_DEVICE_COMPILE__)
  sincos(a[0], &r.sx, &r.cx);   // one shared argument reduction per angle
  sincos(a[1], &r.sy, &r.cy);
  sincos(a[2], &r.sz, &r.cz);
#else
  r.sx = sin(a[0]); r.cx = cos(a[0]);
  r.sy = sin(a[1]); r.cy = cos(a[1]);
  r.sz = sin(a[2]); r.cz = cos(a[2]);
#endif
  return r;
}
// GetRotationMatrixBaseToWorld (:207-221)
TG_HD void euler_R(const Trig& q, double R[3][3]) {
  R[0][0] = q.cy * q.cz; R[0][1] = q.cz * q.sx * q.sy - q.cx * q.sz; R[0][2] = q.sx * q.sz + q.cx * q.cz * q.sy;
  R[1][0] = q.cy * q.sz; R[1][1] = q.cx * q.cz + q.sx * q.sy * q.sz; R[1][2] = q.cx * q.sy * q.sz - q.cz * q.sx;
  R[2][0] = -q.sy;       R[2][1] = q.cy * q.sx;                       R[2][2] = q.cx * q.cy;
}
// dR[i][j] = d R[i][j] / d theta_e for one Euler axis e (GetDerivativeOfRotationMatrixWrtNodes :241-268)
TG_HD void euler_dR_axis(const Trig& q, int e, double dR[3][3]) {
  const double sx = q.sx, cx = q.cx, sy = q.sy, cy = q.cy, sz = q.sz, cz = q.cz;
  if (e == 0) {
    dR[0][0] = 0.0; dR[0][1] = sx * sz + cx * cz * sy; dR[0][2] = cx * sz - cz * sx * sy;
    dR[1][0] = 0.0; dR[1][1] = cx * sy * sz - cz * sx; dR[1][2] = -cx * cz - sx * sy * sz;
    dR[2][0] = 0.0; dR[2][1] = cx * cy;                dR[2][2] = -cy * sx;
  } else if (e == 1) {
    dR[0][0] = -cz * sy; dR[0][1] = cy * cz * sx; dR[0][2] = cx * cy * cz;
    dR[1][0] = -sy * sz; dR[1][1] = cy * sx * sz; dR[1][2] = cx * cy * sz;
    dR[2][0] = -cy;      dR[2][1] = -sx * sy;     dR[2][2] = -cx * sy;
  } else {
    dR[0][0] = -cy * sz; dR[0][1] = -cx * cz - sx * sy * sz; dR[0][2] = cz * sx - cx * sy * sz;
    dR[1][0] = cy * cz;  dR[1][1] = cz * sx * sy - cx * sz;  dR[1][2] = sx * sz + cx * cz * sy;
    dR[2][0] = 0.0;      dR[2][1] = 0.0;                     dR[2][2] = 0.0;
  }
}

// omega = M thd, omega_dot = Mdot thd + M thdd (GetAngularVelocityInWorld / ...AccelerationInWorld,
// euler_converter.cc:58-83 with GetM :133-148, GetMdot :150-166)
TG_HD void euler_w_wd(const Trig& q, const double thd[3], const double thdd[3], double w[3], double wd[3]) {
  const double sy = q.sy, cy = q.cy, sz = q.sz, cz = q.cz, xd = thd[0], yd = thd[1], zd = thd[2];
  const double M0[3] = {cy * cz, cy * sz, -sy}, M1[3] = {-sz, cz, 0.0};
  const double Md0[3] = {-cz * sy * yd - cy * sz * zd, cy * cz * zd - sy * sz * yd, -cy * yd};
  const double Md1[3] = {-cz * zd, -sz * zd, 0.0};
  for (int i = 0; i < 3; ++i) {
    const double M2i = i == 2 ? 1.0 : 0.0;
    w[i] = M0[i] * xd + M1[i] * yd + M2i * zd;
    wd[i] = (Md0[i] * xd + Md1[i] * yd) + (M0[i] * thdd[0] + M1[i] * thdd[1] + M2i * thdd[2]);
  }
}

TG_HD void cross3(const double a[3], const double b[3], double o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
}
// Cross(in)[r][e]: in x v = Cross(in) v  (single_rigid_body_dynamics.cc:47-57)
TG_HD double cross_el(const double in[3], int r, int e) {
  const int d = (e - r + 3) % 3;     // 0 diag, 1 (r, r+1), 2 (r, r+2)
  if (d == 0) return 0.0;
  const int o = 3 - r - e;           // the remaining index
  return d == 1 ? -in[o] : in[o];
}
TG_HD void mat3_vec(const double A[3][3], const double v[3], double o[3]) {
  for (int i = 0; i < 3; ++i) o[i] = A[i][0] * v[0] + A[i][1] * v[1] + A[i][2] * v[2];
}

// ----------------------------------------------------------------------------------------------
// RotVecConverter (towr/src/helpers/rotvec_converter.cc): theta = rotation vector, R = exp([theta]x),
// omega = J_L theta_dot, omega_dot = J_L_dot theta_dot + J_L theta_ddot.
// Every Jacobian w.r.t. the base-angular nodes is returned in coefficient form: the entry at the
// basis column (b, axis l) is P[r][l] Hp[b] + V[r][l] Hv[b] + A[r][l] Ha[b], because each spline
// Jacobian row l of the reference (GetJacobianWrtNodes(t, kPos|kVel|kAcc).row(l)) is the basis of
// axis l. The reference's skip rules (|.| > 1e-15) and its small-angle branches are kept.
// ----------------------------------------------------------------------------------------------
constexpr double kRvEps = 1e-10;   // kEps, rotvec_converter.cc:10
struct RvCoeffs { double alpha, beta, gamma, dalpha, dbeta, dgamma, st, ct; };   // st, ct: sin, cos (theta >= eps)
TG_HD double rv_norm(const double v[3]) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
// ComputeCoeffs (:30-59)
TG_HD RvCoeffs rv_coeffs(double theta) {
  RvCoeffs c;
  const double t2 = theta * theta;
  if (theta < kRvEps) {
    c.alpha = 1.0 - t2 / 6.0; c.beta = 1.0 / 6.0 - t2 / 120.0; c.gamma = 0.5 - t2 / 24.0;
    c.dalpha = -theta / 3.0; c.dbeta = -theta / 60.0; c.dgamma = -theta / 12.0;
    c.st = c.ct = 0.0;
  } else {
    const double st = sin(theta), ct = cos(theta), t3 = t2 * theta, t4 = t3 * theta;
    c.st = st; c.ct = ct;
    c.alpha = st / theta; c.beta = (theta - st) / t3; c.gamma = (1.0 - ct) / t2;
    c.dalpha = (theta * ct - st) / t2;
    c.dbeta = (-2.0 * theta - theta * ct + 3.0 * st) / t4;
    c.dgamma = (theta * st - 2.0 + 2.0 * ct) / t3;
  }
  return c;
}
TG_HD void rv_skew(const double v[3], double S[3][3]) {   // Skew (:20-28)
  S[0][0] = 0.0;   S[0][1] = -v[2]; S[0][2] = v[1];
  S[1][0] = v[2];  S[1][1] = 0.0;   S[1][2] = -v[0];
  S[2][0] = -v[1]; S[2][1] = v[0];  S[2][2] = 0.0;
}
TG_HD void m3_mul(const double A[3][3], const double B[3][3], double C[3][3]) {   // C may not alias
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) C[i][j] = A[i][0] * B[0][j] + A[i][1] * B[1][j] + A[i][2] * B[2][j];
}
// Rodrigues (:61-72); the _c variants take theta = |rv| and rv_coeffs(theta) from the caller, so a
// lane evaluating several converter quantities at one instant forms the trigonometry once
// (sin(theta) / theta and (1 - cos(theta)) / theta^2 are ComputeCoeffs' alpha and gamma)
TG_HD void rv_rodrigues_c(const double rv[3], double theta, const RvCoeffs& c, double R[3][3]) {
  double K[3][3]; rv_skew(rv, K);
  if (theta < kRvEps) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) R[i][j] = (i == j ? 1.0 : 0.0) + K[i][j];
    return;
  }
  const double sn = c.alpha, h = c.gamma;
  double KK[3][3]; m3_mul(K, K, KK);
  for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) R[i][j] = ((i == j ? 1.0 : 0.0) + sn * K[i][j]) + h * KK[i][j];
}
TG_HD void rv_rodrigues(const double rv[3], double R[3][3]) {
  const double theta = rv_norm(rv);
  rv_rodrigues_c(rv, theta, rv_coeffs(theta), R);
}
// LeftJacobian (:74-85)
TG_HD void rv_left_jac_c(const double rv[3], double theta, const RvCoeffs& c, double J[3][3]) {
  double S[3][3]; rv_skew(rv, S);
  if (theta < kRvEps) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) J[i][j] = (i == j ? 1.0 : 0.0) + 0.5 * S[i][j];
    return;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) J[i][j] = (c.alpha * (i == j ? 1.0 : 0.0) + c.beta * (rv[i] * rv[j])) + c.gamma * S[i][j];
}
TG_HD void rv_left_jac(const double rv[3], double J[3][3]) {
  const double theta = rv_norm(rv);
  rv_left_jac_c(rv, theta, rv_coeffs(theta), J);
}
// LeftJacobianDot (:87-107)
TG_HD void rv_left_jac_dot_c(const double rv[3], const double rvd[3], double theta, const RvCoeffs& c, double J[3][3]) {
  double S[3][3], Sd[3][3]; rv_skew(rv, S); rv_skew(rvd, Sd);
  if (theta < kRvEps) {
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) J[i][j] = 0.5 * Sd[i][j];
    return;
  }
  const double td = (rv[0] * rvd[0] + rv[1] * rvd[1] + rv[2] * rvd[2]) / theta;
  const double ad = c.dalpha * td, bd = c.dbeta * td, gd = c.dgamma * td;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      J[i][j] = (((ad * (i == j ? 1.0 : 0.0) + bd * (rv[i] * rv[j])) + c.beta * (rvd[i] * rv[j] + rv[i] * rvd[j])) + gd * S[i][j]) + c.gamma * Sd[i][j];
}
TG_HD void rv_left_jac_dot(const double rv[3], const double rvd[3], double J[3][3]) {
  const double theta = rv_norm(rv);
  rv_left_jac_dot_c(rv, rvd, theta, rv_coeffs(theta), J);
}
TG_HD double rv_sign(int dim, int j) { return ((j - dim + 3) % 3 == 1) ? -1.0 : 1.0; }   // [theta]x_{dim,j} = sign theta_k

// GetDerivJLwrtNodes (:235-325) for all three rows dim: P[dim][j][l] = d J_L[dim][j] / d theta_l
TG_HD void rv_dJL(const double rv[3], double P[3][3][3]) {
  const double theta = rv_norm(rv);
  const RvCoeffs c = rv_coeffs(theta);
  double nh[3] = {0.0, 0.0, 0.0};   // theta^T jac_pos / theta, components with |theta_l| > 1e-15
  if (theta >= kRvEps) {
    const double inv = 1.0 / theta;
    for (int l = 0; l < 3; ++l) nh[l] = fabs(rv[l]) > 1e-15 ? rv[l] * inv : 0.0;
  }
  double Sk[3][3]; rv_skew(rv, Sk);
  for (int dim = 0; dim < 3; ++dim)
    for (int j = 0; j < 3; ++j) {
      double* p = P[dim][j];
      p[0] = p[1] = p[2] = 0.0;
      if (dim == j) for (int l = 0; l < 3; ++l) p[l] += c.dalpha * nh[l];
      const double rvdj = rv[dim] * rv[j];
      if (fabs(rvdj) > 1e-15) for (int l = 0; l < 3; ++l) p[l] += rvdj * (c.dbeta * nh[l]);
      if (fabs(c.beta) > 1e-15) {
        if (fabs(rv[j]) > 1e-15) p[dim] += c.beta * rv[j];
        if (fabs(rv[dim]) > 1e-15) p[j] += c.beta * rv[dim];
      }
      const double sk = Sk[dim][j];
      if (fabs(sk) > 1e-15) for (int l = 0; l < 3; ++l) p[l] += sk * (c.dgamma * nh[l]);
      if (fabs(c.gamma) > 1e-15 && dim != j) p[3 - dim - j] += c.gamma * rv_sign(dim, j);
    }
}

// Column l of rv_dJL: Pc[dim][j] = d J_L[dim][j] / d theta_l, the same operations in the same order
// restricted to one l (the device's RotVec Dynamic evaluates its base-angular block one column at a time)
TG_HD void rv_dJL_col(const double rv[3], const RvCoeffs& c, const double nh[3], int l, double Pc[3][3]) {
  for (int dim = 0; dim < 3; ++dim)
    for (int j = 0; j < 3; ++j) {
      double p = 0.0;
      if (dim == j) p += c.dalpha * nh[l];
      const double rvdj = rv[dim] * rv[j];
      if (fabs(rvdj) > 1e-15) p += rvdj * (c.dbeta * nh[l]);
      if (fabs(c.beta) > 1e-15) {
        if (fabs(rv[j]) > 1e-15 && l == dim) p += c.beta * rv[j];
        if (fabs(rv[dim]) > 1e-15 && l == j) p += c.beta * rv[dim];
      }
      const double sk = dim == j ? 0.0 : rv_sign(dim, j) * rv[3 - dim - j];   // Skew(rv)[dim][j]
      if (fabs(sk) > 1e-15) p += sk * (c.dgamma * nh[l]);
      if (fabs(c.gamma) > 1e-15 && dim != j && l == 3 - dim - j) p += c.gamma * rv_sign(dim, j);
      Pc[dim][j] = p;
    }
}
// n_hat of rv_dJL (theta^T jac_pos / theta, components with |theta_l| > 1e-15)
TG_HD void rv_dJL_nh(const double rv[3], double theta, double nh[3]) {
  nh[0] = nh[1] = nh[2] = 0.0;
  if (theta >= kRvEps) {
    const double inv = 1.0 / theta;
    for (int l = 0; l < 3; ++l) nh[l] = fabs(rv[l]) > 1e-15 ? rv[l] * inv : 0.0;
  }
}
// Column l of rv_angacc_jac's Pa and Va (Aa = J_L): the same operations restricted to one l
TG_HD void rv_angacc_col(const double rv[3], const double rvd[3], const double rva[3], int l, double theta, const RvCoeffs& c,
                         const double JLd[3][3], const double nhd[3], double pa_l[3], double va_l[3]) {
  double td = 0.0;
  if (theta > kRvEps) td = (rv[0] * rvd[0] + rv[1] * rvd[1] + rv[2] * rvd[2]) / theta;
  const double beta_dot = c.dbeta * td, gamma_dot = c.dgamma * td;
  double nh = 0.0, dap = 0.0, dav = 0.0, dbp = 0.0, dbv = 0.0, dgp = 0.0, dgv = 0.0, nh_l[3] = {0.0, 0.0, 0.0};
  if (theta > kRvEps) {
    const double inv = 1.0 / theta, t2 = theta * theta, st = c.st, ct = c.ct;
    nh = rv[l] * inv;
    for (int k = 0; k < 3; ++k) nh_l[k] = rv[k] * inv;
    const double dtp = rvd[l] * inv - (td * inv) * nh, dtv = rv[l] * inv;
    const double alpha_pp = (-theta * st - 2.0 * (theta * ct - st) / theta) / t2;
    double beta_pp, gamma_pp;
    { const double num = -2.0 * theta - theta * ct + 3.0 * st, dnum = -2.0 - ct + theta * st + 3.0 * ct;
      beta_pp = (dnum - 4.0 * num / theta) / (t2 * t2); }
    { const double num = theta * st - 2.0 + 2.0 * ct, dnum = st + theta * ct - 2.0 * st;
      gamma_pp = (dnum - 3.0 * num / theta) / (t2 * theta); }
    dap = (alpha_pp * td) * nh + c.dalpha * dtp; dav = c.dalpha * dtv;
    dbp = (beta_pp * td) * nh + c.dbeta * dtp;   dbv = c.dbeta * dtv;
    dgp = (gamma_pp * td) * nh + c.dgamma * dtp; dgv = c.dgamma * dtv;
  }
  double P1[3][3]; rv_dJL_col(rv, c, nhd, l, P1);   // acc * dJL_du, column l
  for (int dim = 0; dim < 3; ++dim) {
    double pa = 0.0, va = 0.0;
    for (int j = 0; j < 3; ++j) {
      double p = 0.0, v = 0.0;   // d J_L_dot[dim][j] / d (theta_l, theta_dot_l)
      if (dim == j) { p += dap; v += dav; }
      const double rv_dj = rv[dim] * rv[j];
      if (fabs(rv_dj) > 1e-15) { p += rv_dj * dbp; v += rv_dj * dbv; }
      if (fabs(beta_dot) > 1e-15) {
        if (fabs(rv[j]) > 1e-15 && l == dim) p += beta_dot * rv[j];
        if (fabs(rv[dim]) > 1e-15 && l == j) p += beta_dot * rv[dim];
      }
      const double td_dj = rvd[dim] * rv[j] + rv[dim] * rvd[j];
      if (fabs(td_dj) > 1e-15 && fabs(c.beta) > 1e-15 && theta > kRvEps) p += (c.dbeta * td_dj) * nh_l[l];
      if (fabs(c.beta) > 1e-15) {
        if (fabs(rv[j]) > 1e-15 && l == dim) v += c.beta * rv[j];
        if (fabs(rvd[dim]) > 1e-15 && l == j) p += c.beta * rvd[dim];
        if (fabs(rvd[j]) > 1e-15 && l == dim) p += c.beta * rvd[j];
        if (fabs(rv[dim]) > 1e-15 && l == j) v += c.beta * rv[dim];
      }
      const double sk = dim == j ? 0.0 : rv_sign(dim, j) * rv[3 - dim - j];
      if (fabs(sk) > 1e-15) { p += sk * dgp; v += sk * dgv; }
      if (fabs(gamma_dot) > 1e-15 && dim != j && l == 3 - dim - j) p += gamma_dot * rv_sign(dim, j);
      const double skd = dim == j ? 0.0 : rv_sign(dim, j) * rvd[3 - dim - j];
      if (fabs(skd) > 1e-15 && fabs(c.gamma) > 1e-15 && theta > kRvEps) p += (c.dgamma * skd) * nh_l[l];
      if (fabs(c.gamma) > 1e-15 && dim != j && l == 3 - dim - j) v += c.gamma * rv_sign(dim, j);
      pa += rvd[j] * p; va += rvd[j] * v;
    }
    pa_l[dim] = pa + (rva[0] * P1[dim][0] + rva[1] * P1[dim][1] + rva[2] * P1[dim][2]);
    va_l[dim] = va + JLd[dim][l];
  }
}

// d omega / d nodes (GetDerivOfAngVelWrtNodes, :508-528): Pw (theta), Vw (theta_dot)
TG_HD void rv_angvel_jac(const double rv[3], const double rvd[3], double Pw[3][3], double Vw[3][3]) {
  double P[3][3][3]; rv_dJL(rv, P);
  rv_left_jac(rv, Vw);
  for (int dim = 0; dim < 3; ++dim)
    for (int l = 0; l < 3; ++l) Pw[dim][l] = rvd[0] * P[dim][0][l] + rvd[1] * P[dim][1][l] + rvd[2] * P[dim][2][l];
}

// d omega_dot / d nodes (GetDerivOfAngAccWrtNodes :530-561 with GetDerivJLdotwrtNodes :327-506):
// Pa (theta), Va (theta_dot), Aa (theta_ddot)
TG_HD void rv_angacc_jac(const double rv[3], const double rvd[3], const double rva[3], double Pa[3][3], double Va[3][3],
                         double Aa[3][3]) {
  const double theta = rv_norm(rv);
  const RvCoeffs c = rv_coeffs(theta);
  double td = 0.0;
  if (theta > kRvEps) td = (rv[0] * rvd[0] + rv[1] * rvd[1] + rv[2] * rvd[2]) / theta;
  const double beta_dot = c.dbeta * td, gamma_dot = c.dgamma * td;
  // d(alpha_dot), d(beta_dot), d(gamma_dot) / d nodes: (theta part, theta_dot part); n_hat
  double nh[3] = {0.0, 0.0, 0.0}, dap[3] = {0, 0, 0}, dav[3] = {0, 0, 0}, dbp[3] = {0, 0, 0}, dbv[3] = {0, 0, 0},
         dgp[3] = {0, 0, 0}, dgv[3] = {0, 0, 0};
  if (theta > kRvEps) {
    const double inv = 1.0 / theta, t2 = theta * theta, st = sin(theta), ct = cos(theta);
    double dtp[3], dtv[3];   // d theta_dot_angle / d (theta, theta_dot)
    for (int l = 0; l < 3; ++l) { nh[l] = rv[l] * inv; dtp[l] = rvd[l] * inv - (td * inv) * nh[l]; dtv[l] = rv[l] * inv; }
    const double alpha_pp = (-theta * st - 2.0 * (theta * ct - st) / theta) / t2;
    double beta_pp, gamma_pp;
    { const double num = -2.0 * theta - theta * ct + 3.0 * st, dnum = -2.0 - ct + theta * st + 3.0 * ct;
      beta_pp = (dnum - 4.0 * num / theta) / (t2 * t2); }
    { const double num = theta * st - 2.0 + 2.0 * ct, dnum = st + theta * ct - 2.0 * st;
      gamma_pp = (dnum - 3.0 * num / theta) / (t2 * theta); }
    for (int l = 0; l < 3; ++l) {
      dap[l] = (alpha_pp * td) * nh[l] + c.dalpha * dtp[l]; dav[l] = c.dalpha * dtv[l];
      dbp[l] = (beta_pp * td) * nh[l] + c.dbeta * dtp[l];   dbv[l] = c.dbeta * dtv[l];
      dgp[l] = (gamma_pp * td) * nh[l] + c.dgamma * dtp[l]; dgv[l] = c.dgamma * dtv[l];
    }
  }
  double Sk[3][3], Skd[3][3]; rv_skew(rv, Sk); rv_skew(rvd, Skd);
  double JLd[3][3]; rv_left_jac_dot(rv, rvd, JLd);
  double P1[3][3][3]; rv_dJL(rv, P1);   // acc * dJL_du
  rv_left_jac(rv, Aa);
  for (int dim = 0; dim < 3; ++dim) {
    double pa[3] = {0, 0, 0}, va[3] = {0, 0, 0};
    for (int j = 0; j < 3; ++j) {
      double p[3] = {0, 0, 0}, v[3] = {0, 0, 0};   // d J_L_dot[dim][j] / d (theta, theta_dot)
      if (dim == j) for (int l = 0; l < 3; ++l) { p[l] += dap[l]; v[l] += dav[l]; }
      const double rv_dj = rv[dim] * rv[j];
      if (fabs(rv_dj) > 1e-15) for (int l = 0; l < 3; ++l) { p[l] += rv_dj * dbp[l]; v[l] += rv_dj * dbv[l]; }
      if (fabs(beta_dot) > 1e-15) {
        if (fabs(rv[j]) > 1e-15) p[dim] += beta_dot * rv[j];
        if (fabs(rv[dim]) > 1e-15) p[j] += beta_dot * rv[dim];
      }
      const double td_dj = rvd[dim] * rv[j] + rv[dim] * rvd[j];
      if (fabs(td_dj) > 1e-15 && fabs(c.beta) > 1e-15 && theta > kRvEps) for (int l = 0; l < 3; ++l) p[l] += (c.dbeta * td_dj) * nh[l];
      if (fabs(c.beta) > 1e-15) {
        if (fabs(rv[j]) > 1e-15) v[dim] += c.beta * rv[j];
        if (fabs(rvd[dim]) > 1e-15) p[j] += c.beta * rvd[dim];
        if (fabs(rvd[j]) > 1e-15) p[dim] += c.beta * rvd[j];
        if (fabs(rv[dim]) > 1e-15) v[j] += c.beta * rv[dim];
      }
      const double sk = Sk[dim][j];
      if (fabs(sk) > 1e-15) for (int l = 0; l < 3; ++l) { p[l] += sk * dgp[l]; v[l] += sk * dgv[l]; }
      if (fabs(gamma_dot) > 1e-15 && dim != j) p[3 - dim - j] += gamma_dot * rv_sign(dim, j);
      const double skd = Skd[dim][j];
      if (fabs(skd) > 1e-15 && fabs(c.gamma) > 1e-15 && theta > kRvEps) for (int l = 0; l < 3; ++l) p[l] += (c.dgamma * skd) * nh[l];
      if (fabs(c.gamma) > 1e-15 && dim != j) v[3 - dim - j] += c.gamma * rv_sign(dim, j);
      for (int l = 0; l < 3; ++l) { pa[l] += rvd[j] * p[l]; va[l] += rvd[j] * v[l]; }
    }
    for (int l = 0; l < 3; ++l) {
      Pa[dim][l] = pa[l] + (rva[0] * P1[dim][0][l] + rva[1] * P1[dim][1][l] + rva[2] * P1[dim][2][l]);
      Va[dim][l] = va[l] + JLd[dim][l];
    }
  }
}

// DerivOfRotVecMult (:210-233) coefficient matrix: d(R v)/dtheta = -[R v]x J_L (forward),
// d(R^T v)/dtheta = R^T [v]x J_L (inverse)
TG_HD void rv_rotvec_mult(const double R[3][3], const double JL[3][3], const double v[3], bool inverse, double A[3][3]) {
  double S[3][3], T[3][3];
  if (inverse) {
    double Rt[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Rt[i][j] = R[j][i];
    rv_skew(v, S); m3_mul(Rt, S, T); m3_mul(T, JL, A);
  } else {
    double Rv[3]; mat3_vec(R, v, Rv);
    rv_skew(Rv, S);
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) S[i][j] = -S[i][j];
    m3_mul(S, JL, A);
  }
}

// column e of rv_rotvec_mult's coefficient matrix (its element expressions, one column)
TG_HD void rv_rotvec_mult_col(const double R[3][3], const double JL[3][3], const double v[3], bool inverse, int e, double a[3]) {
  double S[3][3];
  if (inverse) {
    double Sv[3][3], T[3][3], Rt[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) Rt[i][j] = R[j][i];
    rv_skew(v, Sv); m3_mul(Rt, Sv, T);
    for (int i = 0; i < 3; ++i) a[i] = T[i][0] * JL[0][e] + T[i][1] * JL[1][e] + T[i][2] * JL[2][e];
  } else {
    double Rv[3]; mat3_vec(R, v, Rv);
    rv_skew(Rv, S);
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) S[i][j] = -S[i][j];
    for (int i = 0; i < 3; ++i) a[i] = S[i][0] * JL[0][e] + S[i][1] * JL[1][e] + S[i][2] * JL[2][e];
  }
}

// RotVec R, omega, omega_dot (GetRotationMatrixBaseToWorld / GetAngularVelocityInWorld /
// GetAngularAccelerationInWorld, :118-138)
TG_HD void rv_state(const SplinePt& A, double R[3][3], double w[3], double wd[3]) {
  double JL[3][3], JLd[3][3], a[3], b[3];
  const double theta = rv_norm(A.p);
  const RvCoeffs cf = rv_coeffs(theta);   // the trigonometry once for the three converter quantities
  rv_rodrigues_c(A.p, theta, cf, R);
  rv_left_jac_c(A.p, theta, cf, JL);
  rv_left_jac_dot_c(A.p, A.v, theta, cf, JLd);
  mat3_vec(JL, A.v, w);
  mat3_vec(JLd, A.v, a); mat3_vec(JL, A.a, b);
  for (int k = 0; k < 3; ++k) wd[k] = a[k] + b[k];
}

// base orientation at a spline point: R (base to world)
TG_HD void base_rot(const Ctx& c, const SplinePt& A, double R[3][3]) {
  if (c.rotvec) rv_rodrigues(A.p, R);
  else euler_R(trig(A.p), R);
}

// ----------------------------------------------------------------------------------------------
// terrain (towr/src/terrain/height_map.cc, height_map_examples.cc)
// ----------------------------------------------------------------------------------------------
TG_HD double ter_h(const towr_terrain_t& T, double x, double y) {
#pragma clang fp contract(off)
  const double* p = T.p;
  switch (T.id) {
    case TOWR_TERRAIN_FLAT: return p[0];
    case TOWR_TERRAIN_BLOCK: {
      double bs = p[0], len = p[1], hh = p[2], eps = p[3], h = 0.0;
      if (bs <= x && x <= bs + eps) h = hh / eps * (x - bs);
      if (bs + eps <= x && x <= bs + len) h = hh;
      return h;
    }
    case TOWR_TERRAIN_STAIRS: {
      double h = 0.0;
      if (x >= p[0]) h = p[2];
      if (x >= p[0] + p[1]) h = p[3];
      if (x >= p[0] + p[1] + p[4]) h = 0.0;
      return h;
    }
    case TOWR_TERRAIN_GAP: {
      double gs = p[0], w = p[1], hh = p[2], xc = gs + w / 2.0, ge = gs + w;
      double a = (4 * hh) / (w * w), b = -(8 * hh * xc) / (w * w), cc = -(hh * (w - 2 * xc) * (w + 2 * xc)) / (w * w);
      return (gs <= x && x <= ge) ? a * x * x + b * x + cc : 0.0;
    }
    case TOWR_TERRAIN_SLOPE: {
      double ss = p[0], xd = ss + p[1], xf = xd + p[2], hc = p[3], sl = hc / p[1], z = 0.0;
      if (x >= ss) z = sl * (x - ss);
      if (x >= xd) z = hc - sl * (x - xd);
      if (x >= xf) z = 0.0;
      return z;
    }
    case TOWR_TERRAIN_CHIMNEY: return (p[0] <= x && x <= p[0] + p[1]) ? p[3] * (y - p[2]) : 0.0;
    case TOWR_TERRAIN_CHIMNEY_LR: {
      double z = 0.0, e1 = p[0] + p[1], e2 = p[0] + 2 * p[1];
      if (p[0] <= x && x <= e1) z = p[3] * (y - p[2]);
      if (e1 <= x && x <= e2) z = -p[3] * (y + p[2]);
      return z;
    }
    case TOWR_TERRAIN_STEPS: {
      if (x < p[0]) return 0.0;
      int step = (int)((x - p[0]) / p[1]);
      return step >= (int)p[3] ? p[3] * p[2] : (step + 1) * p[2];
    }
  }
  return 0.0;
}
TG_HD double ter_dh(const towr_terrain_t& T, int dim, double x, double y) {
#pragma clang fp contract(off)   // the reference's operations: curved-terrain predicates depend on exact zeros
  const double* p = T.p;
  if (dim == X) {
    switch (T.id) {
      case TOWR_TERRAIN_BLOCK: return (p[0] <= x && x <= p[0] + p[3]) ? p[2] / p[3] : 0.0;
      case TOWR_TERRAIN_GAP: {
        double gs = p[0], w = p[1], hh = p[2], xc = gs + w / 2.0;
        double a = (4 * hh) / (w * w), b = -(8 * hh * xc) / (w * w);
        return (gs <= x && x <= gs + w) ? 2 * a * x + b : 0.0;
      }
      case TOWR_TERRAIN_SLOPE: {
        double ss = p[0], xd = ss + p[1], xf = xd + p[2], sl = p[3] / p[1], d = 0.0;
        if (x >= ss) d = sl;
        if (x >= xd) d = -sl;
        if (x >= xf) d = 0.0;
        return d;
      }
    }
    return 0.0;
  }
  switch (T.id) {
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
// GetSecondDerivativeOfHeightWrt (:150-163): only Gap has a nonzero (XX) second derivative
TG_HD double ter_d2h(const towr_terrain_t& T, int d1, int d2, double x, double y) {
  if (T.id == TOWR_TERRAIN_GAP && d1 == X && d2 == X) {
    double gs = T.p[0], w = T.p[1], hh = T.p[2];
    return (gs <= x && x <= gs + w) ? 2 * ((4 * hh) / (w * w)) : 0.0;
  }
  return 0.0;
}
TG_HD bool ter_has_curvature(int id) { return id == TOWR_TERRAIN_GAP; }

// GetBasis (:68-139); deriv < 0: the basis itself
TG_HD void ter_basis(const towr_terrain_t& T, int basis, double x, double y, int deriv, double v[3]) {
  const bool req = deriv < 0;
  if (basis == 0) {
    for (int d = 0; d < 2; ++d) v[d] = req ? -ter_dh(T, d, x, y) : -ter_d2h(T, d, deriv, x, y);
    v[2] = req ? 1.0 : 0.0;
  } else if (basis == 1) {
    v[0] = req ? 1.0 : 0.0; v[1] = 0.0;
    v[2] = req ? ter_dh(T, X, x, y) : ter_d2h(T, X, deriv, x, y);
  } else {
    v[0] = 0.0; v[1] = req ? 1.0 : 0.0;
    v[2] = req ? ter_dh(T, Y, x, y) : ter_d2h(T, Y, deriv, x, y);
  }
}
// Eigen normalized(): v / sqrt(|v|^2) if |v|^2 > 0. REF: the reference's own operations on the device too
// (three divisions, no FMA contraction), for predicates that must resolve exactly as the source does
template <bool REF = false>
TG_HD void normalize3(const double v[3], double o[3]) {
#pragma clang fp contract(off)
  const double z = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (!REF) {
    const double s = z > 0 ? 1.0 / sqrt(z) : 1.0;   // one division instead of three
    o[0] = v[0] * s; o[1] = v[1] * s; o[2] = v[2] * s;
    return;
  }
#endif
  if (z > 0) { const double s = sqrt(z); o[0] = v[0] / s; o[1] = v[1] / s; o[2] = v[2] / s; }
  else { o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; }
}
// GetNormalizedBasis (:62-66)
TG_HD void ter_nbasis(const towr_terrain_t& T, int basis, double x, double y, double o[3]) {
  double v[3]; ter_basis(T, basis, x, y, -1, v); normalize3(v, o);
}
// GetDerivativeOfNormalizedBasisWrt (:80-91, 141-148)
template <bool REF = false>
TG_HD void ter_d_nbasis(const towr_terrain_t& T, int basis, int dim, double x, double y, double o[3]) {
#pragma clang fp contract(off)
  double dv[3], v[3], vn[3];
  ter_basis(T, basis, x, y, dim, dv);
  ter_basis(T, basis, x, y, -1, v);
  const double sq = v[0] * v[0] + v[1] * v[1] + v[2] * v[2], nrm = sqrt(sq);
  normalize3<REF>(v, vn);
  for (int k = 0; k < 3; ++k) o[k] = (1 / sq * ((k == dim ? nrm : 0.0) - v[dim] * vn[k])) * dv[k];
}
// friction-pyramid directions b0..b4 = n, t1-mu n, t1+mu n, t2-mu n, t2+mu n
TG_HD void pyramid(const double n[3], const double t1[3], const double t2[3], double mu, double b[5][3]) {
  for (int q = 0; q < 3; ++q) {
    b[0][q] = n[q];
    b[1][q] = t1[q] - mu * n[q]; b[2][q] = t1[q] + mu * n[q];
    b[3][q] = t2[q] - mu * n[q]; b[4][q] = t2[q] + mu * n[q];
  }
}
TG_HD double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ----------------------------------------------------------------------------------------------
// work items
// ----------------------------------------------------------------------------------------------

// DynamicConstraint instant (dynamic_constraint.cc:63-148, single_rigid_body_dynamics.cc:76-204)
// Group 0 of a DynamicConstraint instant (g: GetDynamicViolation :76-102; d/d base-lin:
// GetJacobianWrtBaseLin :104-122) in two phases. Phase A needs no endeffector sum; phase B takes
// sum_ee (f x (c - p) + tau) and sum_ee f. On the device the endeffector lanes of the same instant
// deposit their terms in LDS (Ctx::dyn_scratch) and phase B runs after a block barrier, so the
// group-0 lane no longer evaluates 3 E splines in a latency-bound loop; the host sums inline in the
// same order.
struct DynG0 { double ab[3], La[3], Lp[3], Hp[4], Ha[4]; int poly; };
constexpr int kDynG0PhaseA = 12;   // candidates of dyn_g0_a (base-linear acceleration block)
constexpr int kDynG0Cand = 36;     // + dyn_g0_b's 24 (the base-linear block of the angular rows)
// I_w wd + w x (I_w w), I_w = R I_b R^T (the angular rows' base terms)
TG_HD void dyn_base_ab(const RobotC& rb, const double R[3][3], const double w[3], const double wd[3], double ab[3]) {
  double RI[3][3], Iw[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) RI[i][j] = R[i][0] * rb.Ib[0 * 3 + j] + R[i][1] * rb.Ib[1 * 3 + j] + R[i][2] * rb.Ib[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iw[i][j] = RI[i][0] * R[j][0] + RI[i][1] * R[j][1] + RI[i][2] * R[j][2];
  double a[3], Iww[3], b[3];
  mat3_vec(Iw, wd, a); mat3_vec(Iw, w, Iww); cross3(w, Iww, b);
  for (int e = 0; e < 3; ++e) ab[e] = a[e] + b[e];
}
// PRE (fixed gait, RotVec, device): the base terms ab come from the coefficient pre-pass (tiles.hip
// towr_rv_coef_kernel, fields kRvAb.. of the instant it.a0, field stride `stride`), so the lane forms no
// converter state
template <bool PRE = false, class Emit>
TG_HD void dyn_g0_a(const Ctx& c, const ItemDesc& it, Emit& em, DynG0& st, const double* pre = nullptr, int64_t stride = 0) {
  const double t = it.t;
  const int r0 = it.row0;
  SplinePt L; spline_eval(c, SP_BASE_LIN, t, L);
  if constexpr (PRE) {
    for (int e = 0; e < 3; ++e) st.ab[e] = pre[e * stride];
  } else {
    SplinePt A; spline_eval(c, SP_BASE_ANG, t, A);
    double R[3][3], w[3], wd[3];
    if (c.rotvec) rv_state(A, R, w, wd);
    else {
      const Trig q = trig(A.p);
      euler_R(q, R);
      euler_w_wd(q, A.v, A.a, w, wd);
    }
    dyn_base_ab(c.rb, R, w, wd, st.ab);
  }
  for (int e = 0; e < 3; ++e) { st.La[e] = L.a[e]; st.Lp[e] = L.p[e]; }
  st.poly = L.poly;
  spline_basis(L, kPos, st.Hp); spline_basis(L, kAcc, st.Ha);
  for (int e = 0; e < 3; ++e)
    for (int bb = 0; bb < 4; ++bb) em(r0 + LX + e, basis_col(c, SP_BASE_LIN, L.poly, bb, e), c.rb.m * st.Ha[bb], true);
}
// one endeffector's terms of the sums at an instant: ts = f x (c - p) + tau, fs = f
TG_HD void dyn_ee_terms(const double Lp[3], const SplinePt& F, const SplinePt& Tq, const SplinePt& P, double out[6]) {
  const double rr[3] = {Lp[0] - P.p[0], Lp[1] - P.p[1], Lp[2] - P.p[2]};
  double cr[3]; cross3(F.p, rr, cr);
  for (int e = 0; e < 3; ++e) { out[e] = cr[e] + Tq.p[e]; out[3 + e] = F.p[e]; }
}
template <class Emit>
TG_HD void dyn_g0_b(const Ctx& c, const ItemDesc& it, Emit& em, const DynG0& st, const double fs[3], const double ts[3]) {
  const int r0 = it.row0;
  for (int e = 0; e < 3; ++e) em.g(r0 + AX + e, st.ab[e] - ts[e]);
  const double grav[3] = {0.0, 0.0, -c.rb.m * c.rb.g};
  for (int e = 0; e < 3; ++e) em.g(r0 + LX + e, c.rb.m * st.La[e] - fs[e] - grav[e]);
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int d = 1; d <= 2; ++d) {
      const int e = (r + d) % 3;
      const double sc = -cross_el(fs, r, e);  // -(sum_ee Cross(f_ee))[r][e]
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) em(r0 + AX + r, basis_col(c, SP_BASE_LIN, st.poly, bb, e), sc * st.Hp[bb], true);
    }
}

// Dynamic's base-angular block (group 1: GetJacobianWrtBaseAng :124-166) in coefficient form: the
// entry at basis column (b, axis e) of angular row r is Ap[r] Hp[b] + Av[r] Hv[b] + Aa[r] Ha[b], with
// (Ap, Av, Aa) the derivatives w.r.t. (theta_e, theta_dot_e, theta_ddot_e) and H the base-angular
// spline's position / velocity / acceleration basis. The state shared by the axes of one instant is
// formed once (dyn_*_state); each axis / component then costs its own chain (dyn_euler_axis,
// dyn_rv_column). Used by eval_dyn (tile path, host structure pass) and by the gait Dynamic record
// kernel (gstream.hip), which stores the coefficients for the composer.
struct DynEulerState {
  SplinePt A;
  Trig q;
  double R[3][3], M0[3], M1[3], Md0[3], Md1[3], w[3], wd[3], RI[3][3], Iw[3][3], Iww[3];
};
// Euler ZYX: A(.) = I_w wd + w x (I_w w);  I_w = R I_b R^T,  w = M thd,  wd = Mdot thd + M thdd
TG_HD void dyn_euler_state(const Ctx& c, double t, DynEulerState& S) {
  spline_eval(c, SP_BASE_ANG, t, S.A);
  const SplinePt& A = S.A;
  S.q = trig(A.p);
  const double sy = S.q.sy, cy = S.q.cy, sz = S.q.sz, cz = S.q.cz;
  const double xd = A.v[0], yd = A.v[1], zd = A.v[2];
  euler_R(S.q, S.R);
  // M columns (GetM :133-148) and Mdot columns (GetMdot :150-166)
  S.M0[0] = cy * cz; S.M0[1] = cy * sz; S.M0[2] = -sy;
  S.M1[0] = -sz; S.M1[1] = cz; S.M1[2] = 0.0;
  S.Md0[0] = -cz * sy * yd - cy * sz * zd; S.Md0[1] = cy * cz * zd - sy * sz * yd; S.Md0[2] = -cy * yd;
  S.Md1[0] = -cz * zd; S.Md1[1] = -sz * zd; S.Md1[2] = 0.0;
  for (int i = 0; i < 3; ++i) {
    const double M2i = i == 2 ? 1.0 : 0.0;
    S.w[i] = S.M0[i] * xd + S.M1[i] * yd + M2i * zd;
    S.wd[i] = (S.Md0[i] * xd + S.Md1[i] * yd) + (S.M0[i] * A.a[0] + S.M1[i] * A.a[1] + M2i * A.a[2]);
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) S.RI[i][j] = S.R[i][0] * c.rb.Ib[0 * 3 + j] + S.R[i][1] * c.rb.Ib[1 * 3 + j] + S.R[i][2] * c.rb.Ib[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) S.Iw[i][j] = S.RI[i][0] * S.R[j][0] + S.RI[i][1] * S.R[j][1] + S.RI[i][2] * S.R[j][2];
  mat3_vec(S.Iw, S.w, S.Iww);
}
// one Euler axis e: the chain rule through (theta_e, theta_dot_e, theta_ddot_e)
TG_HD void dyn_euler_axis(const Ctx& c, const DynEulerState& S, const int e, double Ap[3], double Av[3], double Aa[3]) {
  const double sy = S.q.sy, cy = S.q.cy, sz = S.q.sz, cz = S.q.cz;
  const double xd = S.A.v[0], yd = S.A.v[1], zd = S.A.v[2];
  const double(&R)[3][3] = S.R;
  const double(&RI)[3][3] = S.RI;
  const double(&Iw)[3][3] = S.Iw;
  const double *w = S.w, *wd = S.wd;
  double dR[3][3]; euler_dR_axis(S.q, e, dR);
  // dw = dM_e thd; dwd = dMdot_e thd + dM_e thdd (GetDerivMwrtNodes :168-198, GetDerivMdotwrtNodes :270-304)
  double dw[3] = {0.0, 0.0, 0.0}, dwd[3] = {0.0, 0.0, 0.0};
  if (e == 1) {
    const double dM0[3] = {-sy * cz, -sy * sz, -cy};
    const double dMd0[3] = {-cy * cz * yd + sy * sz * zd, -cy * sz * yd - sy * cz * zd, sy * yd};
    for (int i = 0; i < 3; ++i) { dw[i] = dM0[i] * xd; dwd[i] = dMd0[i] * xd + dM0[i] * S.A.a[0]; }
  } else if (e == 2) {
    const double dM0[3] = {-cy * sz, cy * cz, 0.0}, dM1[3] = {-cz, -sz, 0.0};
    const double dMd0[3] = {sy * sz * yd - cy * cz * zd, -sy * cz * yd - cy * sz * zd, 0.0};
    const double dMd1[3] = {sz * zd, -cz * zd, 0.0};
    for (int i = 0; i < 3; ++i) {
      dw[i] = dM0[i] * xd + dM1[i] * yd;
      dwd[i] = (dMd0[i] * xd + dMd1[i] * yd) + (dM0[i] * S.A.a[0] + dM1[i] * S.A.a[1]);
    }
  }
  // dI_w/dtheta_e = dR I_b R^T + R I_b dR^T, applied to wd and w
  double dRI[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dRI[i][j] = dR[i][0] * c.rb.Ib[0 * 3 + j] + dR[i][1] * c.rb.Ib[1 * 3 + j] + dR[i][2] * c.rb.Ib[2 * 3 + j];
  double dIwd[3], dIw_w[3];
  {
    double u[3], v[3];   // R^T wd, dR^T wd (and the same for w)
    for (int j = 0; j < 3; ++j) { u[j] = R[0][j] * wd[0] + R[1][j] * wd[1] + R[2][j] * wd[2]; v[j] = dR[0][j] * wd[0] + dR[1][j] * wd[1] + dR[2][j] * wd[2]; }
    for (int i = 0; i < 3; ++i) dIwd[i] = (dRI[i][0] * u[0] + dRI[i][1] * u[1] + dRI[i][2] * u[2]) + (RI[i][0] * v[0] + RI[i][1] * v[1] + RI[i][2] * v[2]);
    for (int j = 0; j < 3; ++j) { u[j] = R[0][j] * w[0] + R[1][j] * w[1] + R[2][j] * w[2]; v[j] = dR[0][j] * w[0] + dR[1][j] * w[1] + dR[2][j] * w[2]; }
    for (int i = 0; i < 3; ++i) dIw_w[i] = (dRI[i][0] * u[0] + dRI[i][1] * u[1] + dRI[i][2] * u[2]) + (RI[i][0] * v[0] + RI[i][1] * v[1] + RI[i][2] * v[2]);
  }
  double t1[3], t2[3], t3[3];
  // theta_e: dI_w wd + I_w dwd + dw x (I_w w) + w x (dI_w w + I_w dw)
  mat3_vec(Iw, dwd, t1); cross3(dw, S.Iww, t2); mat3_vec(Iw, dw, t3);
  for (int i = 0; i < 3; ++i) t3[i] += dIw_w[i];
  double t4[3]; cross3(w, t3, t4);
  for (int i = 0; i < 3; ++i) Ap[i] = dIwd[i] + t1[i] + t2[i] + t4[i];
  // theta_dot_e: dw = M[:,e], dwd = dM_e thd + Mdot[:,e]
  const double Me[3] = {e == 0 ? S.M0[0] : e == 1 ? S.M1[0] : 0.0, e == 0 ? S.M0[1] : e == 1 ? S.M1[1] : 0.0,
                        e == 0 ? S.M0[2] : e == 1 ? S.M1[2] : 1.0};
  double dwv[3];
  for (int i = 0; i < 3; ++i) dwv[i] = dw[i] + (e == 0 ? S.Md0[i] : e == 1 ? S.Md1[i] : 0.0);
  mat3_vec(Iw, dwv, t1); cross3(Me, S.Iww, t2); mat3_vec(Iw, Me, t3); cross3(w, t3, t4);
  for (int i = 0; i < 3; ++i) { Av[i] = t1[i] + t2[i] + t4[i]; Aa[i] = t3[i]; }   // theta_ddot_e: I_w M[:,e]
}

// RotVecConverter (GetJacobianWrtBaseAng :124-166 with the converter's DerivOfRotVecMult /
// GetDerivOfAngVelWrtNodes / GetDerivOfAngAccWrtNodes), coefficient form:
//   jac1 = d(R v11)/. + R I_b d(R^T wd)/. + I_w d wd/.
//   jac2 = [w]x (d(R v21)/. + R I_b d(R^T w)/. + I_w d w/.) - [I_w w]x d w/.
// One rotation-vector component e (a column of every coefficient matrix) at a time, each column by the
// full-matrix code's element expressions: the whole matrices at once needed ~400 live doubles and
// spilled 884 bytes per lane to scratch.
struct DynRvState {
  SplinePt A;
  double theta;
  RvCoeffs cf;   // the instant's converter coefficients, formed once
  double R[3][3], w[3], wd[3], JL[3][3], JLd[3][3], RI[3][3], Iw[3][3], v11[3], v21[3], Iww[3], nhd[3];
};
TG_HD void dyn_rv_state(const Ctx& c, double t, DynRvState& S) {
  spline_eval(c, SP_BASE_ANG, t, S.A);
  const SplinePt& A = S.A;
  S.theta = rv_norm(A.p);
  S.cf = rv_coeffs(S.theta);
  rv_rodrigues_c(A.p, S.theta, S.cf, S.R);
  rv_left_jac_c(A.p, S.theta, S.cf, S.JL);
  rv_left_jac_dot_c(A.p, A.v, S.theta, S.cf, S.JLd);
  {   // rv_state
    double a[3], b[3];
    mat3_vec(S.JL, A.v, S.w);
    mat3_vec(S.JLd, A.v, a); mat3_vec(S.JL, A.a, b);
    for (int k = 0; k < 3; ++k) S.wd[k] = a[k] + b[k];
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) S.RI[i][j] = S.R[i][0] * c.rb.Ib[0 * 3 + j] + S.R[i][1] * c.rb.Ib[1 * 3 + j] + S.R[i][2] * c.rb.Ib[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) S.Iw[i][j] = S.RI[i][0] * S.R[j][0] + S.RI[i][1] * S.R[j][1] + S.RI[i][2] * S.R[j][2];
  double u[3];
  for (int j = 0; j < 3; ++j) u[j] = S.R[0][j] * S.wd[0] + S.R[1][j] * S.wd[1] + S.R[2][j] * S.wd[2];
  for (int i = 0; i < 3; ++i) S.v11[i] = c.rb.Ib[i * 3 + 0] * u[0] + c.rb.Ib[i * 3 + 1] * u[1] + c.rb.Ib[i * 3 + 2] * u[2];
  for (int j = 0; j < 3; ++j) u[j] = S.R[0][j] * S.w[0] + S.R[1][j] * S.w[1] + S.R[2][j] * S.w[2];
  for (int i = 0; i < 3; ++i) S.v21[i] = c.rb.Ib[i * 3 + 0] * u[0] + c.rb.Ib[i * 3 + 1] * u[1] + c.rb.Ib[i * 3 + 2] * u[2];
  mat3_vec(S.Iw, S.w, S.Iww);
  rv_dJL_nh(A.p, S.theta, S.nhd);
}
// component E (compile-time: a runtime index puts the 3x3 arrays in scratch) of every coefficient matrix
template <int E>
TG_HD void dyn_rv_column(const DynRvState& S, double Mp[3], double Mv[3], double Ma[3]) {
  constexpr int e = E;
  const SplinePt& A = S.A;
  const double(&R)[3][3] = S.R;
  const double(&JL)[3][3] = S.JL;
  const double(&RI)[3][3] = S.RI;
  const double(&Iw)[3][3] = S.Iw;
  double m1[3], t1[3], pa[3], va[3], pw[3];
  {
    double Pc[3][3]; rv_dJL_col(A.p, S.cf, S.nhd, e, Pc);   // Pw[:, e] (rv_angvel_jac)
    for (int d = 0; d < 3; ++d) pw[d] = A.v[0] * Pc[d][0] + A.v[1] * Pc[d][1] + A.v[2] * Pc[d][2];
  }
  rv_angacc_col(A.p, A.v, A.a, e, S.theta, S.cf, S.JLd, S.nhd, pa, va);   // Pa[:, e], Va[:, e]
  rv_rotvec_mult_col(R, JL, S.v11, false, e, m1);
  rv_rotvec_mult_col(R, JL, S.wd, true, e, t1);
  double mp[3], sc[3];
  for (int i = 0; i < 3; ++i)
    mp[i] = (m1[i] + (RI[i][0] * t1[0] + RI[i][1] * t1[1] + RI[i][2] * t1[2])) + (Iw[i][0] * pa[0] + Iw[i][1] * pa[1] + Iw[i][2] * pa[2]);
  rv_rotvec_mult_col(R, JL, S.v21, false, e, m1);
  rv_rotvec_mult_col(R, JL, S.w, true, e, t1);
  for (int i = 0; i < 3; ++i)
    sc[i] = (m1[i] + (RI[i][0] * t1[0] + RI[i][1] * t1[1] + RI[i][2] * t1[2])) + (Iw[i][0] * pw[0] + Iw[i][1] * pw[1] + Iw[i][2] * pw[2]);
  for (int r = 0; r < 3; ++r) {
    double a = 0.0, b = 0.0, av = 0.0, bv = 0.0;
    for (int k = 0; k < 3; ++k) {
      const double cw = cross_el(S.w, r, k), ci = cross_el(S.Iww, r, k);
      a += cw * sc[k]; b += ci * pw[k];
      double iv = Iw[k][0] * JL[0][e] + Iw[k][1] * JL[1][e] + Iw[k][2] * JL[2][e];
      av += cw * iv; bv += ci * JL[k][e];
    }
    Mp[r] = mp[r] + (a - b);
    Mv[r] = (Iw[r][0] * va[0] + Iw[r][1] * va[1] + Iw[r][2] * va[2]) + (av - bv);
    Ma[r] = Iw[r][0] * JL[0][e] + Iw[r][1] * JL[1][e] + Iw[r][2] * JL[2][e];
  }
}

// The base-angular entries of a RotVec group-1 item from the instant's formed state: one column per
// call (a RotVec g1 item carries its component in a1 = 1 + e, layout.hip; the device evaluates exactly
// that column, a loop over three columns spilled to scratch), the host structure pass and emulation take
// every column of an unsplit item in order. The fixed-gait device tile forms S once per instant in LDS
// (tiles.hip tile_body) and calls this from each component lane.
template <class Emit>
TG_HD void dyn_rv_emit(const Ctx& c, const ItemDesc& it, const DynRvState& S, Emit& em) {
  const int r0 = it.row0;
  double Hp[4], Hv[4], Ha[4];
  spline_basis(S.A, kPos, Hp); spline_basis(S.A, kVel, Hv); spline_basis(S.A, kAcc, Ha);
  auto column = [&](auto ec) {   // ec: std::integral_constant (the device instantiates each column)
    constexpr int e = decltype(ec)::value;
    double Mp[3], Mv[3], Ma[3];
    dyn_rv_column<e>(S, Mp, Mv, Ma);
    for (int r = 0; r < 3; ++r)
      for (int bb = 0; bb < 4; ++bb)
        em(r0 + AX + r, basis_col(c, SP_BASE_ANG, S.A.poly, bb, e), Mp[r] * Hp[bb] + Mv[r] * Hv[bb] + Ma[r] * Ha[bb], true);
  };
  const int e_lo = it.a1 > 0 ? it.a1 - 1 : 0, e_hi = it.a1 > 0 ? it.a1 : 3;
  if (e_lo <= 0 && 0 < e_hi) column(std::integral_constant<int, 0>{});
  if (e_lo <= 1 && 1 < e_hi) column(std::integral_constant<int, 1>{});
  if (e_lo <= 2 && 2 < e_hi) column(std::integral_constant<int, 2>{});
}

// The same entries from precomputed coefficients (the device's RotVec pre-pass, tiles.hip towr_rv_coef_kernel):
// coef[(9 e + f) stride] = field f (Mp[3] | Mv[3] | Ma[3]) of the item's component e = a1 - 1
template <class Emit>
TG_HD void dyn_rv_emit_pre(const Ctx& c, const ItemDesc& it, const double* coef, int64_t stride, Emit& em) {
  const int r0 = it.row0, e = it.a1 - 1;
  SplinePt A;
  spline_eval(c, SP_BASE_ANG, it.t, A);
  double Hp[4], Hv[4], Ha[4];
  spline_basis(A, kPos, Hp); spline_basis(A, kVel, Hv); spline_basis(A, kAcc, Ha);
  double M[9];
  for (int f = 0; f < 9; ++f) M[f] = coef[(9 * e + f) * stride];
  for (int r = 0; r < 3; ++r)
    for (int bb = 0; bb < 4; ++bb)
      em(r0 + AX + r, basis_col(c, SP_BASE_ANG, A.poly, bb, e), M[r] * Hp[bb] + M[3 + r] * Hv[bb] + M[6 + r] * Ha[bb], true);
}

template <class Emit>
TG_HD void eval_dyn(const Ctx& c, const ItemDesc& it, Emit& em) {
  if constexpr (emit_dyn_groups<Emit>::value == 1) { if (it.group == 1) return; }
  if constexpr (emit_dyn_groups<Emit>::value == 2) { if (it.group != 1) return; }
  const double t = it.t;
  const int r0 = it.row0, E = c.rb.n_ee;
  if (it.group == 0) {   // both phases inline (host structure pass; see dyn_g0_a)
    DynG0 st;
    dyn_g0_a(c, it, em, st);
    double fs[3] = {0, 0, 0}, ts[3] = {0, 0, 0};
    for (int ee = 0; ee < E; ++ee) {
      SplinePt F, Tq, P;
      spline_eval(c, sp_force(ee), t, F);
      spline_eval(c, sp_torque(ee), t, Tq);
      spline_eval(c, sp_motion(ee), t, P);
      double v[6]; dyn_ee_terms(st.Lp, F, Tq, P, v);
      for (int e = 0; e < 3; ++e) { ts[e] += v[e]; fs[e] += v[3 + e]; }
    }
    dyn_g0_b(c, it, em, st, fs, ts);
    return;
  }
  if (it.group == 1 && c.rotvec) {
    DynRvState S;
    dyn_rv_state(c, t, S);
    dyn_rv_emit(c, it, S, em);
    return;
  }
  if (it.group == 1) {
    DynEulerState S;
    dyn_euler_state(c, t, S);
    double Hp[4], Hv[4], Ha[4];
    spline_basis(S.A, kPos, Hp); spline_basis(S.A, kVel, Hv); spline_basis(S.A, kAcc, Ha);
    // all three axes in one lane (236 VGPRs on the fixed-gait device tile); the host (structure pass,
    // emulation) takes the axes of an unsplit item (a1 = 0) in order
    auto axis = [&](const int e) {
      double Ap[3], Av[3], Aa[3];
      dyn_euler_axis(c, S, e, Ap, Av, Aa);
      for (int r = 0; r < 3; ++r)
        for (int bb = 0; bb < 4; ++bb)
          em(r0 + AX + r, basis_col(c, SP_BASE_ANG, S.A.poly, bb, e), Ap[r] * Hp[bb] + Av[r] * Hv[bb] + Aa[r] * Ha[bb], true);
    };
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int e = 0; e < 3; ++e) axis(e);
#else
    for (int e = 0; e < 3; ++e)
      if (it.a1 == 0 || it.a1 == 1 + e) axis(e);
#endif
    return;
  }
  // group 2 + ee: force (GetJacobianWrtForce :168-180), torque (:182-191), motion (:193-204)
  const int ee = it.group - 2;
  // A row-split lane (gait, ItemDesc::rsel) whose rows are all linear (LX..LZ) needs only the force
  // spline and its schedule Jacobian: the base, torque and motion terms enter the angular rows only.
  // Emission order is unchanged (a filtered row's candidates are neither emitted nor counted).
  bool ang = true;
  if constexpr (emit_filter<Emit>::value) ang = em_wants(em, r0 + AX) || em_wants(em, r0 + AY) || em_wants(em, r0 + AZ);
  SplinePt L, F, Tq, P;
  spline_eval(c, sp_force(ee), t, F);
  double rv[3] = {0.0, 0.0, 0.0};
  if (ang) {
    spline_eval(c, SP_BASE_LIN, t, L);
    spline_eval(c, sp_torque(ee), t, Tq);
    spline_eval(c, sp_motion(ee), t, P);
    if (c.dyn_scratch) {   // this endeffector's terms of the group-0 sums (it.a2 = instant within the tile)
      double v[6]; dyn_ee_terms(L.p, F, Tq, P, v);
      double* d = c.dyn_scratch + (it.a2 * E + ee) * 6;
      for (int q = 0; q < 6; ++q) d[q] = v[q];
    }
    for (int k = 0; k < 3; ++k) rv[k] = L.p[k] - P.p[k];
  }
  double H[4];
  spline_basis(F, kPos, H);
  if (ang) {
    #pragma unroll
    for (int r = 0; r < 3; ++r)
      #pragma unroll
      for (int d = 1; d <= 2; ++d) {
        const int e = (r + d) % 3;
        emit_dim(c, em, r0 + AX + r, sp_force(ee), F, H, e, cross_el(rv, r, e));
      }
  }
  #pragma unroll
  for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + LX + e, sp_force(ee), F, H, e, -1.0);
  if (ang) {
    spline_basis(Tq, kPos, H);
    #pragma unroll
    for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + AX + e, sp_torque(ee), Tq, H, e, -1.0);
    spline_basis(P, kPos, H);
    #pragma unroll
    for (int r = 0; r < 3; ++r)
      #pragma unroll
      for (int d = 1; d <= 2; ++d) {
        const int e = (r + d) % 3;
        emit_dim(c, em, r0 + AX + r, sp_motion(ee), P, H, e, cross_el(F.p, r, e));
      }
  }
  if (c.gait) {
    // d/d ee schedule (dynamic_constraint.cc:116-122): force and ee-position terms; the reference
    // omits the torque term here and so does this engine
    SchedJac Jf;
    sched_jac(c, sp_force(ee), t, F, Jf);
    if (ang) {
      SchedJac Jx;
      sched_jac(c, sp_motion(ee), t, P, Jx);
      #pragma unroll
      for (int r = 0; r < 3; ++r) {
        if (!em_wants(em, r0 + AX + r)) continue;
        const int e1 = (r + 1) % 3, e2 = (r + 2) % 3;
        for (int col = 0; col < Jf.n - 1; ++col) {
          const double a = cross_el(rv, r, e1) * sched_val(Jf, e1, col) + cross_el(rv, r, e2) * sched_val(Jf, e2, col);
          const double b = cross_el(F.p, r, e1) * sched_val(Jx, e1, col) + cross_el(F.p, r, e2) * sched_val(Jx, e2, col);
          em(r0 + AX + r, Jf.col0 + col, a + b, true);
        }
      }
    }
    #pragma unroll
    for (int e = 0; e < 3; ++e)
      if (em_wants(em, r0 + LX + e))
        for (int col = 0; col < Jf.n - 1; ++col) em(r0 + LX + e, Jf.col0 + col, -sched_val(Jf, e, col), true);
  }
}


// RangeOfMotionConstraint instant (range_of_motion_constraint.cc:72-131)
template <class Emit>
TG_HD void eval_rom(const Ctx& c, const ItemDesc& it, Emit& em) {
  const double t = it.t;
  const int r0 = it.row0, ee = it.ee;
  SplinePt L, A, P;
  spline_eval(c, SP_BASE_LIN, t, L);
  spline_eval(c, SP_BASE_ANG, t, A);
  spline_eval(c, sp_motion(ee), t, P);
  double R[3][3];
  Trig q{};
  double th = 0.0;
  RvCoeffs cf{};
  if (c.rotvec) { th = rv_norm(A.p); cf = rv_coeffs(th); rv_rodrigues_c(A.p, th, cf, R); }
  else { q = trig(A.p); euler_R(q, R); }
  const double rW[3] = {P.p[0] - L.p[0], P.p[1] - L.p[1], P.p[2] - L.p[2]};
  double H[4];
  if (it.group == 1 && c.rotvec) {
    // DerivOfRotVecMult(t, r_W, inverse = true) of the RotVecConverter: R^T [r_W]x J_L, full pattern (the
    // trigonometry shared with R; unrolled like the Euler branch below, so the slot-group loads are hoisted)
    double JL[3][3], Am[3][3];
    rv_left_jac_c(A.p, th, cf, JL);
    rv_rotvec_mult(R, JL, rW, true, Am);
    spline_basis(A, kPos, H);
#pragma unroll
    for (int e = 0; e < 3; ++e)
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) em(r0 + r, basis_col(c, SP_BASE_ANG, A.poly, bb, e), Am[r][e] * H[bb], true);
    return;
  }
  if (it.group == 0) {
    for (int i = 0; i < 3; ++i) em.g(r0 + i, R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2]);
    spline_basis(L, kPos, H);
    for (int r = 0; r < 3; ++r)
      for (int e = 0; e < 3; ++e)
        for (int bb = 0; bb < 4; ++bb) em(r0 + r, basis_col(c, SP_BASE_LIN, L.poly, bb, e), -R[e][r] * H[bb], true);
  } else if (it.group == 1) {
    // DerivOfRotVecMult(t, r_W, inverse=true): row r = sum_c rW[c] dR[c][r]; row X has no roll terms.
    // Fully unrolled: the 33 candidates then have compile-time emission indices, so the slot-group
    // loads are hoisted instead of waited for one group at a time.
    spline_basis(A, kPos, H);
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      double dR[3][3]; euler_dR_axis(q, e, dR);
#pragma unroll
      for (int r = (e == 0 ? 1 : 0); r < 3; ++r) {
        const double s = rW[0] * dR[0][r] + rW[1] * dR[1][r] + rW[2] * dR[2][r];
        for (int bb = 0; bb < 4; ++bb) em(r0 + r, basis_col(c, SP_BASE_ANG, A.poly, bb, e), s * H[bb], true);
      }
    }
  } else {
    spline_basis(P, kPos, H);
    #pragma unroll
    for (int r = 0; r < 3; ++r)
      #pragma unroll
      for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + r, sp_motion(ee), P, H, e, R[e][r]);
    if (c.gait) {   // b_R_w * d pos / d schedule (range_of_motion_constraint.cc:123-130)
      SchedJac Jx;
      sched_jac(c, sp_motion(ee), t, P, Jx);
      #pragma unroll
      for (int r = 0; r < 3; ++r)
        if (em_wants(em, r0 + r))
          for (int col = 0; col < Jx.n - 1; ++col)
            em(r0 + r, Jx.col0 + col, R[0][r] * sched_val(Jx, 0, col) + R[1][r] * sched_val(Jx, 1, col) + R[2][r] * sched_val(Jx, 2, col), true);
    }
  }
}

// The motion-block scales of a ForceConstraintDiscretized instant on curved terrain: row i, position
// dimension dim gets F . d(pyramid row i)/d p_dim (force_constraint_discretized.cc:125-155), added through
// AccumulateScaledRowJacobian, which skips the whole block when the scale is exactly 0.0 (:58): the
// Jacobian pattern then depends on x. Shared by eval_fdisc and the pattern watch (towr_gpu_pattern_outside).
// Evaluated with the reference's operations on the device too (ter_d_nbasis<true>, no contraction): whether
// a scale is exactly 0.0 decides the pattern.
TG_HD void fdisc_motion_scales(const towr_terrain_t& T, double mu, const double p[3], const double f[3], double sc[2][5]) {
#pragma clang fp contract(off)
  for (int dim = 0; dim < 2; ++dim) {
    double dn[3], dt1[3], dt2[3], db[5][3];
    ter_d_nbasis<true>(T, 0, dim, p[0], p[1], dn);
    ter_d_nbasis<true>(T, 1, dim, p[0], p[1], dt1);
    ter_d_nbasis<true>(T, 2, dim, p[0], p[1], dt2);
    for (int q = 0; q < 3; ++q) {   // pyramid
      db[0][q] = dn[q];
      db[1][q] = dt1[q] - mu * dn[q]; db[2][q] = dt1[q] + mu * dn[q];
      db[3][q] = dt2[q] - mu * dn[q]; db[4][q] = dt2[q] + mu * dn[q];
    }
    for (int i = 0; i < 5; ++i) sc[dim][i] = f[0] * db[i][0] + f[1] * db[i][1] + f[2] * db[i][2];
  }
}
// The same for a TorqueConstraintDiscretized instant (torque_constraint_discretized.cc:175-198): rows
// tau . d t1, tau . d t2, +-(tau . d n) - k mu f . d n
TG_HD void tqdisc_motion_scales(const towr_terrain_t& T, double mu, double kf, const double p[3], const double f[3], const double tq[3],
                                double sc[2][4]) {
#pragma clang fp contract(off)
  auto dot = [](const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
  for (int dim = 0; dim < 2; ++dim) {
    double dn[3], dt1[3], dt2[3];
    ter_d_nbasis<true>(T, 0, dim, p[0], p[1], dn);
    ter_d_nbasis<true>(T, 1, dim, p[0], p[1], dt1);
    ter_d_nbasis<true>(T, 2, dim, p[0], p[1], dt2);
    const double s_tau_n = dot(tq, dn), s_lim = kf * mu * dot(f, dn);
    sc[dim][0] = dot(tq, dt1);
    sc[dim][1] = dot(tq, dt2);
    sc[dim][2] = s_tau_n - s_lim;
    sc[dim][3] = -s_tau_n - s_lim;
  }
}

// ForceConstraintDiscretized instant (force_constraint_discretized.cc:97-221)
template <class Emit>
TG_HD void eval_fdisc(const Ctx& c, const ItemDesc& it, Emit& em) {
  const double t = it.t, mu = c.ter->friction_coeff;
  const int r0 = it.row0, ee = it.ee;
  SplinePt P, F;
  spline_eval(c, sp_motion(ee), t, P);
  spline_eval(c, sp_force(ee), t, F);
  double n[3], t1[3], t2[3], b[5][3];
  ter_nbasis(*c.ter, 0, P.p[0], P.p[1], n);
  ter_nbasis(*c.ter, 1, P.p[0], P.p[1], t1);
  ter_nbasis(*c.ter, 2, P.p[0], P.p[1], t2);
  pyramid(n, t1, t2, mu, b);
  for (int i = 0; i < 5; ++i) em.g(r0 + i, dot3(F.p, b[i]));
  double H[4];
  spline_basis(F, kPos, H);
  #pragma unroll
  for (int i = 0; i < 5; ++i)
    #pragma unroll
    for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + i, sp_force(ee), F, H, e, b[i][e]);
  double sc[2][5] = {{0, 0, 0, 0, 0}, {0, 0, 0, 0, 0}};   // F . d(pyramid)/d p_dim
  if (c.fdisc_motion) {   // AccumulateScaledRowJacobian: skipped when scale == 0.0 (:58)
    spline_basis(P, kPos, H);
    fdisc_motion_scales(*c.ter, mu, P.p, F.p, sc);
    #pragma unroll
    for (int dim = 0; dim < 2; ++dim)
      #pragma unroll
      for (int i = 0; i < 5; ++i) emit_dim(c, em, r0 + i, sp_motion(ee), P, H, dim, sc[dim][i], sc[dim][i] != 0.0);
  }
  if (c.gait) {   // schedule (force_constraint_discretized.cc:158-190): force linear form + motion scaled rows
    SchedJac Jf, Jx;
    sched_jac(c, sp_force(ee), t, F, Jf);
    sched_jac(c, sp_motion(ee), t, P, Jx);
    #pragma unroll
    for (int i = 0; i < 5; ++i)
      if (em_wants(em, r0 + i))
        for (int col = 0; col < Jf.n - 1; ++col) {
        double v = b[i][0] * sched_val(Jf, 0, col) + b[i][1] * sched_val(Jf, 1, col) + b[i][2] * sched_val(Jf, 2, col);
        if (sc[0][i] != 0.0) v += sc[0][i] * sched_val(Jx, 0, col);
        if (sc[1][i] != 0.0) v += sc[1][i] * sched_val(Jx, 1, col);
        em(r0 + i, Jf.col0 + col, v, true);
      }
  }
}

// ForceConstraintDiscretized under phase-duration optimisation on a terrain without curvature
// (no motion block, fdisc_motion == 0), split for the streaming composer (towr_gpu.hip
// fdisc_stream_body): fdisc_instant computes once per instant what eval_fdisc computes per lane
// (force_constraint_discretized.cc:71-221), and every Jacobian entry of the instant's 5 rows is
// then a function of it and the entry's column: a force column is b[i][e] times the Hermite basis
// of the active force polynomial at the column's node values (phase_basis_sum, emit_dim's
// full-pattern arithmetic), a schedule column a combination of the force spline's d pos / d schedule
// (fdisc_sched_value, eval_fdisc's arithmetic). The operations are eval_fdisc's, in its order.
struct FdiscInstant {
  int poly;          // active polynomial of the force PhaseSpline
  double H[4];       // its position basis at the instant
  double nb[3][3];   // the normalized terrain basis n, t1, t2 at the foot
  double b[5][3];    // the 5 pyramid rows (normal, friction +- mu normal) of the terrain basis
  SchedJac Jf;       // d force(t) / d schedule
  double g[5];
};
TG_HD void fdisc_instant(const Ctx& c, int ee, double t, FdiscInstant& o) {
  const double mu = c.ter->friction_coeff;
  SplinePt P, F;
  spline_eval(c, sp_motion(ee), t, P);
  spline_eval(c, sp_force(ee), t, F);
  ter_nbasis(*c.ter, 0, P.p[0], P.p[1], o.nb[0]);
  ter_nbasis(*c.ter, 1, P.p[0], P.p[1], o.nb[1]);
  ter_nbasis(*c.ter, 2, P.p[0], P.p[1], o.nb[2]);
  pyramid(o.nb[0], o.nb[1], o.nb[2], mu, o.b);
  for (int i = 0; i < 5; ++i) o.g[i] = dot3(F.p, o.b[i]);
  spline_basis(F, kPos, o.H);
  o.poly = F.poly;
  sched_jac(c, sp_force(ee), t, F, o.Jf);
}
// emit_dim's full-pattern basis sum of PhaseSpline column pq at polynomial `poly` (the entry is then
// scale * sum, scale = b[i][e]); 0.0 off the active polynomial
TG_HD double phase_basis_sum(const PhaseCol& pq, int poly, double h0, double h1, double h2, double h3) {
  double v = 0.0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {   // constant indices: a runtime-indexed pq.id / deriv goes to scratch
    if (k >= pq.n) break;
    if (pq.id[k] == poly) v += pq.deriv[k] ? h1 : h0;
    else if (pq.id[k] == poly + 1) v += pq.deriv[k] ? h3 : h2;
  }
  return v;
}
TG_HD double fdisc_sched_value(const double bi[3], const SchedJac& Jf, int col) {
  return bi[0] * sched_val(Jf, 0, col) + bi[1] * sched_val(Jf, 1, col) + bi[2] * sched_val(Jf, 2, col);
}

// ForceConstraint node (force_constraint.cc:62-171); a0 = force node, a1 = motion node at phase start
template <class Emit>
TG_HD void eval_fnode(const Ctx& c, const ItemDesc& it, Emit& em) {
  const double mu = c.ter->friction_coeff;
  const int r0 = it.row0, ee = it.ee, fs = sp_force(ee), ms = sp_motion(ee);
  double p[3], f[3];
  for (int e = 0; e < 3; ++e) { p[e] = xval(c, node_col(c, ms, it.a1, kPos, e)); f[e] = xval(c, node_col(c, fs, it.a0, kPos, e)); }
  double n[3], t1[3], t2[3], b[5][3];
  ter_nbasis(*c.ter, 0, p[0], p[1], n);
  ter_nbasis(*c.ter, 1, p[0], p[1], t1);
  ter_nbasis(*c.ter, 2, p[0], p[1], t2);
  pyramid(n, t1, t2, mu, b);
  for (int i = 0; i < 5; ++i) em.g(r0 + i, dot3(f, b[i]));
  for (int e = 0; e < 3; ++e) {
    const int col = node_col(c, fs, it.a0, kPos, e);
    for (int i = 0; i < 5; ++i) em(r0 + i, col, b[i][e], true);
  }
  for (int dim = 0; dim < 2; ++dim) {
    double dn[3], dt1[3], dt2[3], db[5][3];
    ter_d_nbasis(*c.ter, 0, dim, p[0], p[1], dn);
    ter_d_nbasis(*c.ter, 1, dim, p[0], p[1], dt1);
    ter_d_nbasis(*c.ter, 2, dim, p[0], p[1], dt2);
    pyramid(dn, dt1, dt2, mu, db);
    const int col = node_col(c, ms, it.a1, kPos, dim);
    for (int i = 0; i < 5; ++i) em(r0 + i, col, dot3(f, db[i]), true);
  }
}

// TerrainConstraint node (terrain_constraint.cc:61-111); BaseHeightConstraint node (:58-110)
template <class Emit>
TG_HD void eval_height(const Ctx& c, const ItemDesc& it, int s, double offset, Emit& em) {
  double p[3];
  for (int e = 0; e < 3; ++e) p[e] = xval(c, node_col(c, s, it.a0, kPos, e));
  em.g(it.row0, p[2] - ter_h(*c.ter, p[0], p[1]) - offset);
  em(it.row0, node_col(c, s, it.a0, kPos, Z), 1.0, true);
  for (int dim = 0; dim < 2; ++dim)
    em(it.row0, node_col(c, s, it.a0, kPos, dim), -ter_dh(*c.ter, dim, p[0], p[1]), true);
}

// BaseMotionConstraint instant (base_motion_constraint.cc:60-85)
template <class Emit>
TG_HD void eval_bmot(const Ctx& c, const ItemDesc& it, Emit& em) {
  SplinePt L, A;
  spline_eval(c, SP_BASE_LIN, it.t, L);
  spline_eval(c, SP_BASE_ANG, it.t, A);
  for (int e = 0; e < 3; ++e) { em.g(it.row0 + LX + e, L.p[e]); em.g(it.row0 + AX + e, A.p[e]); }
  double H[4];
  spline_basis(A, kPos, H);
  for (int e = 0; e < 3; ++e)
    for (int bb = 0; bb < 4; ++bb) em(it.row0 + AX + e, basis_col(c, SP_BASE_ANG, A.poly, bb, e), H[bb], true);
  spline_basis(L, kPos, H);
  for (int e = 0; e < 3; ++e)
    for (int bb = 0; bb < 4; ++bb) em(it.row0 + LX + e, basis_col(c, SP_BASE_LIN, L.poly, bb, e), H[bb], true);
}

// SplineAccConstraint junction j = it.k (spline_acc_constraint.cc:48-80); it.ee = spline id
template <class Emit>
TG_HD void eval_sacc(const Ctx& c, const ItemDesc& it, Emit& em) {
  const int s = it.ee, j = it.k;
  const SplineMeta m = c.spl[s];
  const double Tp = c.dur[m.dur_off + j], Tn = c.dur[m.dur_off + j + 1];
  SplinePt a, b;
  poly_state(c, s, j, Tp, Tp, a);
  poly_state(c, s, j + 1, Tn, 0.0, b);
  for (int e = 0; e < 3; ++e) em.g(it.row0 + e, a.a[e] - b.a[e]);
  double Hp[4], Hn[4];
  hermite_dacc(Tp, Tp, Hp); hermite_dacc(Tn, 0.0, Hn);
  // acc_prev - acc_next; node j+1 belongs to both polynomials (a base spline: its values are their
  // own variables), so its two contributions are summed into one candidate each for p and v
  for (int e = 0; e < 3; ++e) {
    em(it.row0 + e, basis_col(c, s, j, 0, e), Hp[0], true);
    em(it.row0 + e, basis_col(c, s, j, 1, e), Hp[1], true);
    em(it.row0 + e, basis_col(c, s, j, 2, e), Hp[2] - Hn[0], true);
    em(it.row0 + e, basis_col(c, s, j, 3, e), Hp[3] - Hn[1], true);
    em(it.row0 + e, basis_col(c, s, j + 1, 2, e), -Hn[2], true);
    em(it.row0 + e, basis_col(c, s, j + 1, 3, e), -Hn[3], true);
  }
}

// SwingConstraint node (swing_constraint.cc:54-108); it.p0 = t_swing_avg
template <class Emit>
TG_HD void eval_swing(const Ctx& c, const ItemDesc& it, Emit& em) {
  const int s = sp_motion(it.ee), id = it.a0;
  const double tsw = it.p0;
  int row = it.row0;
  for (int dim = 0; dim < 2; ++dim) {
    const double prev = xval(c, node_col(c, s, id - 1, kPos, dim)), next = xval(c, node_col(c, s, id + 1, kPos, dim));
    const double dist = next - prev, center = prev + 0.5 * dist, vdes = dist / tsw;
    em.g(row, xval(c, node_col(c, s, id, kPos, dim)) - center);
    em(row, node_col(c, s, id, kPos, dim), 1.0, true);
    em(row, node_col(c, s, id + 1, kPos, dim), -0.5, true);
    em(row, node_col(c, s, id - 1, kPos, dim), -0.5, true);
    ++row;
    em.g(row, xval(c, node_col(c, s, id, kVel, dim)) - vdes);
    em(row, node_col(c, s, id, kVel, dim), 1.0, true);
    em(row, node_col(c, s, id + 1, kPos, dim), -1.0 / tsw, true);
    em(row, node_col(c, s, id - 1, kPos, dim), +1.0 / tsw, true);
    ++row;
  }
}

// TorqueConstraintDiscretized instant (torque_constraint_discretized.cc:101-235); it.p0 = k_friction
template <class Emit>
TG_HD void eval_tqdisc(const Ctx& c, const ItemDesc& it, Emit& em) {
  const double t = it.t, mu = c.ter->friction_coeff, kf = it.p0;
  const int r0 = it.row0, ee = it.ee;
  SplinePt P, F, Tq;
  spline_eval(c, sp_motion(ee), t, P);
  spline_eval(c, sp_force(ee), t, F);
  spline_eval(c, sp_torque(ee), t, Tq);
  double n[3], t1[3], t2[3];
  ter_nbasis(*c.ter, 0, P.p[0], P.p[1], n);
  ter_nbasis(*c.ter, 1, P.p[0], P.p[1], t1);
  ter_nbasis(*c.ter, 2, P.p[0], P.p[1], t2);
  const double tau_n = dot3(Tq.p, n), tz_lim = kf * mu * dot3(F.p, n);
  em.g(r0 + 0, dot3(Tq.p, t1));
  em.g(r0 + 1, dot3(Tq.p, t2));
  em.g(r0 + 2, tau_n - tz_lim);
  em.g(r0 + 3, -tau_n - tz_lim);
  const double mn[3] = {-n[0], -n[1], -n[2]}, b[3] = {-kf * mu * n[0], -kf * mu * n[1], -kf * mu * n[2]};
  const double* tb[4] = {t1, t2, n, mn};
  double H[4];
  spline_basis(Tq, kPos, H);   // AccumulateLinearFormJacobian of the torque spline
  #pragma unroll
  for (int r = 0; r < 4; ++r)
    #pragma unroll
    for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + r, sp_torque(ee), Tq, H, e, tb[r][e]);
  spline_basis(F, kPos, H);    // ... of the force spline into the two normal-torque rows
  #pragma unroll
  for (int r = 2; r < 4; ++r)
    #pragma unroll
    for (int e = 0; e < 3; ++e) emit_dim(c, em, r0 + r, sp_force(ee), F, H, e, b[e]);
  double sc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};   // d rows / d p_dim through the terrain basis
  if (c.fdisc_motion) {   // AccumulateScaledRowJacobian: skipped when scale == 0.0 (:58)
    spline_basis(P, kPos, H);
    tqdisc_motion_scales(*c.ter, mu, kf, P.p, F.p, Tq.p, sc);
    #pragma unroll
    for (int dim = 0; dim < 2; ++dim)
      #pragma unroll
      for (int r = 0; r < 4; ++r) emit_dim(c, em, r0 + r, sp_motion(ee), P, H, dim, sc[dim][r], sc[dim][r] != 0.0);
  }
  if (c.gait) {   // schedule (:210-234): torque and force linear forms, motion scaled rows
    SchedJac Jt, Jf, Jx;
    sched_jac(c, sp_torque(ee), t, Tq, Jt);
    sched_jac(c, sp_force(ee), t, F, Jf);
    sched_jac(c, sp_motion(ee), t, P, Jx);
    #pragma unroll
    for (int r = 0; r < 4; ++r)
      if (em_wants(em, r0 + r))
        for (int col = 0; col < Jt.n - 1; ++col) {
        double v = tb[r][0] * sched_val(Jt, 0, col) + tb[r][1] * sched_val(Jt, 1, col) + tb[r][2] * sched_val(Jt, 2, col);
        if (r >= 2) v += b[0] * sched_val(Jf, 0, col) + b[1] * sched_val(Jf, 1, col) + b[2] * sched_val(Jf, 2, col);
        if (sc[0][r] != 0.0) v += sc[0][r] * sched_val(Jx, 0, col);
        if (sc[1][r] != 0.0) v += sc[1][r] * sched_val(Jx, 1, col);
        em(r0 + r, Jt.col0 + col, v, true);
      }
  }
}

// TorqueConstraint node (torque_constraint.cc:68-193): a0 = torque node, a1 = motion node and
// a2 = torque node at the start of its phase. The motion Jacobian uses the torque at the start of
// the phase, not the node's own torque (torque_constraint.cc:166), as the reference does.
template <class Emit>
TG_HD void eval_tqnode(const Ctx& c, const ItemDesc& it, Emit& em) {
  const int r0 = it.row0, ee = it.ee, ts = sp_torque(ee), ms = sp_motion(ee);
  double p[3], tau[3], tau0[3];
  for (int e = 0; e < 3; ++e) {
    p[e] = xval(c, node_col(c, ms, it.a1, kPos, e));
    tau[e] = xval(c, node_col(c, ts, it.a0, kPos, e));
    tau0[e] = xval(c, node_col(c, ts, it.a2, kPos, e));
  }
  double n[3], t1[3], t2[3];
  ter_nbasis(*c.ter, 0, p[0], p[1], n);
  ter_nbasis(*c.ter, 1, p[0], p[1], t1);
  ter_nbasis(*c.ter, 2, p[0], p[1], t2);
  em.g(r0 + 0, dot3(tau, t1));
  em.g(r0 + 1, dot3(tau, t2));
  em.g(r0 + 2, dot3(tau, n));
  for (int dim = 0; dim < 3; ++dim) {
    const int col = node_col(c, ts, it.a0, kPos, dim);
    em(r0 + 0, col, t1[dim], true);
    em(r0 + 1, col, t2[dim], true);
    em(r0 + 2, col, n[dim], true);
  }
  for (int dim = 0; dim < 2; ++dim) {
    double dn[3], dt1[3], dt2[3];
    ter_d_nbasis(*c.ter, 1, dim, p[0], p[1], dt1);
    ter_d_nbasis(*c.ter, 2, dim, p[0], p[1], dt2);
    ter_d_nbasis(*c.ter, 0, dim, p[0], p[1], dn);
    const int col = node_col(c, ms, it.a1, kPos, dim);
    em(r0 + 0, col, dot3(tau0, dt1), true);
    em(r0 + 1, col, dot3(tau0, dt2), true);
    em(r0 + 2, col, dot3(tau0, dn), true);
  }
}

// TerrainConstraintHard instant (terrain_constraint_hard.cc:50-132). The value caps the clearance
// term at k_coeff_ = 0.02 while the Jacobian's velocity term switches off at 0.05 (SURVEY A22 iii),
// as in the reference. Position and velocity rows of one dimension share their columns.
template <class Emit>
TG_HD void eval_thard(const Ctx& c, const ItemDesc& it, Emit& em) {
  const int ms = sp_motion(it.ee);
  SplinePt P;
  spline_eval(c, ms, it.t, P);
  double n[3], t1[3], t2[3];
  ter_nbasis(*c.ter, 0, P.p[0], P.p[1], n);
  ter_nbasis(*c.ter, 1, P.p[0], P.p[1], t1);
  ter_nbasis(*c.ter, 2, P.p[0], P.p[1], t2);
  const double vt1 = dot3(P.v, t1), vt2 = dot3(P.v, t2), vtm = sqrt(vt1 * vt1 + vt2 * vt2), kc = 0.02;
  const double a = kc * vtm;
  em.g(it.row0, (P.p[2] - ter_h(*c.ter, P.p[0], P.p[1])) - (kc < a ? kc : a));
  const bool vel = vtm > 1e-6 && a < 0.05 - 1e-6;
  double Hp[4], Hv[4];
  spline_basis(P, kPos, Hp);
  spline_basis(P, kVel, Hv);
  for (int k = 0; k < 3; ++k) {
    const int dim = k == 0 ? Z : k - 1;   // jac_pos.row(Z), then -= dh/d(x|y) * jac_pos.row(x|y)
    const double cp = dim == Z ? 1.0 : -ter_dh(*c.ter, dim, P.p[0], P.p[1]);
    const double cv = vel ? -(kc * ((vt1 * t1[dim] + vt2 * t2[dim]) / vtm)) : 0.0;
    double Heff[4];
    for (int bb = 0; bb < 4; ++bb) Heff[bb] = cp * Hp[bb] + cv * Hv[bb];
    emit_dim(c, em, it.row0, ms, P, Heff, dim, 1.0);
  }
}

// EELinearConstraint instant (ee_linear_constraint.cc:19-48); it.a0 = definition
template <class Emit>
TG_HD void eval_eelin(const Ctx& c, const ItemDesc& it, Emit& em) {
  const EELinDef& d = c.eelin[it.a0];
  double val = 0.0;
  for (int q = 0; q < d.n; ++q) {
    const int ee = d.code[q] / 3, dim = d.code[q] % 3, s = d.target == 0 ? sp_motion(ee) : sp_ang(ee);
    SplinePt P;
    spline_eval(c, s, it.t, P);
    // select chains, not a runtime index or pointer (either keeps P in scratch on the device)
    const double pd = dim == 0 ? P.p[0] : dim == 1 ? P.p[1] : P.p[2];
    const double vd = dim == 0 ? P.v[0] : dim == 1 ? P.v[1] : P.v[2];
    val += d.coeff[q] * (d.deriv == 0 ? pd : vd);
    double H[4];
    spline_basis(P, d.deriv == 0 ? kPos : kVel, H);
    emit_dim(c, em, it.row0, s, P, H, dim, d.coeff[q]);
  }
  em.g(it.row0, val);
}

// LinearEqualityConstraint row (linear_constraint.cc:47-76): g = M x_set, Jacobian = M.sparseView().
// The reference's dense product also adds the zero entries' 0 * x_j, which changes no finite sum.
template <class Emit>
TG_HD void eval_lineq(const Ctx& c, const ItemDesc& it, Emit& em) {
  double s = 0.0;
  for (int k = 0; k < it.a1; ++k) {
    const LinNz e = c.lin[it.a0 + k];
    s += e.v * xval(c, e.col);
    em(it.row0, e.col, e.v, true);
  }
  em.g(it.row0, s);
}

// TotalDurationConstraint (total_duration_constraint.cc:49-72): sum of the ee's optimised durations
template <class Emit>
TG_HD void eval_tdur(const Ctx& c, const ItemDesc& it, Emit& em) {
  const SchedInfo si = c.sched[it.ee];
  double sum = 0.0;
  for (int i = 0; i < si.n_phases - 1; ++i) sum += c.x[si.col0 + i];
  em.g(it.row0, sum);
  for (int i = 0; i < si.n_phases - 1; ++i) em(it.row0, si.col0 + i, 1.0, true);
}

// ----------------------------------------------------------------------------------------------
// cost terms (NlpFormulation::GetCosts, nlp_formulation.cc:604-680; towr/src/costs/)
//   eval_f = sum of every term's GetCost; eval_grad_f = the dense sum of their gradients.
// A cost work item is one (term, sample time[, endeffector]) of a time-sampled cost, or one whole
// NodeCost. It adds its value to em.f and its gradient entries with em(0, col, value, present):
// the same emitter interface as the constraint items, so the spline chain rules (emit_dim, the
// PhaseSpline full pattern, sched_jac) are shared with the constraints.
// ----------------------------------------------------------------------------------------------
// CT_ENERGYQ: EnergyCost of one polynomial of a force / torque spline with fixed durations (see
// cost_energy_q); CT_ENERGY: one (sample, ee) of EnergyCost under phase-duration optimisation
// CT_BHC: one sample of BaseHeightCost
enum CostType { CT_NODE = 0, CT_ENERGY = 1, CT_ANGMOM = 2, CT_EEBP = 3, CT_ENERGYQ = 4, CT_BHC = 5, CT_COUNT = 6 };

struct CostItem {
  int32_t type, ee, seg, s;        // seg: segment-table row of the sample time; s: spline (CT_NODE)
  int32_t deriv, dim;              // CT_NODE: node value penalised; CT_ENERGYQ: deriv = polynomial of spline s
  int32_t a0, a1;                  // CT_NODE: nodes [a0, a1); CT_EEBP: a0 = ee in contact at start (swing
                                   // test under gait optimisation); CT_ENERGYQ: a0 = Gram matrix index (Ctx::cq);
                                   // CT_BHC: a0 = contact-at-start bits, a1 = contact bits at t (fixed gait) or -1
  double t, w, wdt, tw;            // sample time, weight, weight * dt, EnergyCost torque weight
  double p[3];                     // CT_EEBP: reference ee position in base frame
  int32_t cslot, cn;               // gradient contribution slots [cslot, cslot + cn) (Layout::cost_nslot > 0)
};

// NodeCost (node_cost.cc:55-79): sum over nodes of w * value^2; d/dx_i = sum over the node values
// variable i sets of 2 w value (a stance position variable sets two nodes: counted twice)
template <class Emit>
TG_HD void cost_node(const Ctx& c, const CostItem& it, Emit& em) {
  for (int id = it.a0; id < it.a1; ++id) {   // one chunk of the spline's nodes (layout.hip build_costs)
    const int col = node_col(c, it.s, id, it.deriv, it.dim);
    const double v = xval(c, col);
    em.f += it.w * (v * v);
    em(0, col, it.w * 2.0 * v, col >= 0);
  }
}

// EnergyCost sample (energy_cost.cc:57-152) of one endeffector: w dt (|f|^2 + tw |tau|^2)
template <class Emit>
TG_HD void cost_energy(const Ctx& c, const CostItem& it, Emit& em) {
  const int ee = it.ee;
  SplinePt F, Tq;
  spline_eval(c, sp_force(ee), it.t, F);
  spline_eval(c, sp_torque(ee), it.t, Tq);
  em.f += it.wdt * (dot3(F.p, F.p) + it.tw * dot3(Tq.p, Tq.p));
  double mf[3], mt[3], H[4];
  for (int r = 0; r < 3; ++r) { mf[r] = (2.0 * it.wdt) * F.p[r]; mt[r] = (2.0 * it.wdt * it.tw) * Tq.p[r]; }
  spline_basis(F, kPos, H);
  for (int e = 0; e < 3; ++e) emit_dim(c, em, 0, sp_force(ee), F, H, e, mf[e]);
  if (it.tw != 0.0) {
    spline_basis(Tq, kPos, H);
    for (int e = 0; e < 3; ++e) emit_dim(c, em, 0, sp_torque(ee), Tq, H, e, mt[e]);
  }
  if (c.gait) {   // d pos / d schedule of both splines (energy_cost.cc:131-150)
    SchedJac Jf, Jt;
    sched_jac(c, sp_force(ee), it.t, F, Jf);
    if (it.tw != 0.0) sched_jac(c, sp_torque(ee), it.t, Tq, Jt);
    for (int col = 0; col < Jf.n - 1; ++col) {
      double v = mf[0] * sched_val(Jf, 0, col) + mf[1] * sched_val(Jf, 1, col) + mf[2] * sched_val(Jf, 2, col);
      if (it.tw != 0.0) v += mt[0] * sched_val(Jt, 0, col) + mt[1] * sched_val(Jt, 1, col) + mt[2] * sched_val(Jt, 2, col);
      em(0, Jf.col0 + col, v, true);
    }
  }
}

// EnergyCost (energy_cost.cc:57-152) over one polynomial of a force or torque spline whose durations
// are fixed. The polynomial's samples contribute sum_t w dt |F(t)|^2 with F_e(t) = H(t) . u_e (the
// Hermite position basis times the polynomial's four node values of dim e), i.e. sum_e u_e^T Q u_e
// with the batch-invariant Gram matrix Q = sum_t w dt H(t) H(t)^T (times the torque weight for a
// torque spline), built once on the host from the same sample times and basis (layout.hip
// build_costs). d/du_e = 2 Q u_e: one gradient entry per node value and polynomial instead of one
// per sample. Equal to the per-sample sums of the reference up to rounding (summation order).
template <class Emit>
TG_HD void cost_energy_q(const Ctx& c, const CostItem& it, Emit& em) {
  const double* Q = c.cq + 16 * (size_t)it.a0;
  for (int e = 0; e < 3; ++e) {
    int col[4];
    double u[4], Qu[4];
    for (int b = 0; b < 4; ++b) { col[b] = basis_col(c, it.s, it.deriv, b, e); u[b] = xval(c, col[b]); }
    for (int b = 0; b < 4; ++b) Qu[b] = Q[4 * b + 0] * u[0] + Q[4 * b + 1] * u[1] + Q[4 * b + 2] * u[2] + Q[4 * b + 3] * u[3];
    em.f += u[0] * Qu[0] + u[1] * Qu[1] + u[2] * Qu[2] + u[3] * Qu[3];
    for (int b = 0; b < 4; ++b) em(0, col[b], 2.0 * Qu[b], col[b] >= 0);   // a shared stance variable sums both
  }
}

// AngularMomentumCost sample with the RotVecConverter: dL = d(R v2)/. + R I_b (d(R^T w)/. + R^T dw/.)
// (angular_momentum_cost.cc:150-200), v2 = I_b R^T w
template <class Emit>
TG_HD void cost_angmom_rotvec(const Ctx& c, const CostItem& it, const SplinePt& A, Emit& em) {
  double R[3][3], JL[3][3], w[3];
  rv_rodrigues(A.p, R);
  rv_left_jac(A.p, JL);
  mat3_vec(JL, A.v, w);
  double RI[3][3], Iw[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) RI[i][j] = R[i][0] * c.rb.Ib[0 * 3 + j] + R[i][1] * c.rb.Ib[1 * 3 + j] + R[i][2] * c.rb.Ib[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iw[i][j] = RI[i][0] * R[j][0] + RI[i][1] * R[j][1] + RI[i][2] * R[j][2];
  double L[3]; mat3_vec(Iw, w, L);
  em.f += it.wdt * dot3(L, L);
  double m[3];
  for (int r = 0; r < 3; ++r) m[r] = (2.0 * it.wdt) * L[r];
  double u[3], v2[3];
  for (int j = 0; j < 3; ++j) u[j] = R[0][j] * w[0] + R[1][j] * w[1] + R[2][j] * w[2];
  for (int i = 0; i < 3; ++i) v2[i] = c.rb.Ib[i * 3 + 0] * u[0] + c.rb.Ib[i * 3 + 1] * u[1] + c.rb.Ib[i * 3 + 2] * u[2];
  double Pw[3][3], Vw[3][3], A1[3][3], A2[3][3];
  rv_angvel_jac(A.p, A.v, Pw, Vw);
  rv_rotvec_mult(R, JL, v2, false, A1);
  rv_rotvec_mult(R, JL, w, true, A2);
  double Hp[4], Hv[4];
  spline_basis(A, kPos, Hp);
  spline_basis(A, kVel, Hv);
  for (int e = 0; e < 3; ++e) {
    // m . (A1 + R I_b (A2 + R^T Pw)) [:, e] and m . (R I_b R^T Vw) [:, e]
    double sp = 0.0, sv = 0.0;
    for (int i = 0; i < 3; ++i) {
      double tu[3], tv[3];
      for (int k = 0; k < 3; ++k) {
        tu[k] = A2[k][e] + (R[0][k] * Pw[0][e] + R[1][k] * Pw[1][e] + R[2][k] * Pw[2][e]);
        tv[k] = R[0][k] * Vw[0][e] + R[1][k] * Vw[1][e] + R[2][k] * Vw[2][e];
      }
      sp += m[i] * (A1[i][e] + (RI[i][0] * tu[0] + RI[i][1] * tu[1] + RI[i][2] * tu[2]));
      sv += m[i] * (RI[i][0] * tv[0] + RI[i][1] * tv[1] + RI[i][2] * tv[2]);
    }
    for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_ANG, A.poly, bb, e), sp * Hp[bb] + sv * Hv[bb], true);
  }
}

// AngularMomentumCost sample (angular_momentum_cost.cc:67-208): w dt |L|^2, L = R I_b R^T omega,
// omega = M(theta) theta_dot. d L / d theta_e = dR I_b R^T w + R I_b dR^T w + I_w dM_e theta_dot;
// d L / d theta_dot_e = I_w M[:, e]; chained through the Euler spline's position / velocity basis.
template <class Emit>
TG_HD void cost_angmom(const Ctx& c, const CostItem& it, Emit& em) {
  SplinePt A;
  spline_eval(c, SP_BASE_ANG, it.t, A);
  if (c.rotvec) { cost_angmom_rotvec(c, it, A, em); return; }
  const Trig q = trig(A.p);
  const double sy = q.sy, cy = q.cy, sz = q.sz, cz = q.cz, xd = A.v[0], yd = A.v[1];
  double R[3][3]; euler_R(q, R);
  const double M0[3] = {cy * cz, cy * sz, -sy}, M1[3] = {-sz, cz, 0.0};
  double w[3];
  for (int i = 0; i < 3; ++i) w[i] = M0[i] * xd + M1[i] * yd + (i == 2 ? A.v[2] : 0.0);
  double RI[3][3], Iw[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) RI[i][j] = R[i][0] * c.rb.Ib[0 * 3 + j] + R[i][1] * c.rb.Ib[1 * 3 + j] + R[i][2] * c.rb.Ib[2 * 3 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iw[i][j] = RI[i][0] * R[j][0] + RI[i][1] * R[j][1] + RI[i][2] * R[j][2];
  double L[3]; mat3_vec(Iw, w, L);
  em.f += it.wdt * dot3(L, L);
  double m[3], u[3];
  for (int r = 0; r < 3; ++r) m[r] = (2.0 * it.wdt) * L[r];
  for (int j = 0; j < 3; ++j) u[j] = R[0][j] * w[0] + R[1][j] * w[1] + R[2][j] * w[2];   // R^T w
  double Hp[4], Hv[4];
  spline_basis(A, kPos, Hp);
  spline_basis(A, kVel, Hv);
#pragma unroll 1
  for (int e = 0; e < 3; ++e) {
    double dR[3][3]; euler_dR_axis(q, e, dR);
    double dw[3] = {0.0, 0.0, 0.0};   // dM_e theta_dot (GetDerivMwrtNodes, euler_converter.cc:168-198)
    if (e == 1) { dw[0] = -sy * cz * xd; dw[1] = -sy * sz * xd; dw[2] = -cy * xd; }
    else if (e == 2) { dw[0] = -cy * sz * xd - cz * yd; dw[1] = cy * cz * xd - sz * yd; }
    double v[3], dRI[3][3], t1[3], t2[3];
    for (int j = 0; j < 3; ++j) v[j] = dR[0][j] * w[0] + dR[1][j] * w[1] + dR[2][j] * w[2];   // dR^T w
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dRI[i][j] = dR[i][0] * c.rb.Ib[0 * 3 + j] + dR[i][1] * c.rb.Ib[1 * 3 + j] + dR[i][2] * c.rb.Ib[2 * 3 + j];
    mat3_vec(Iw, dw, t1);
    double sp = 0.0;
    for (int i = 0; i < 3; ++i)
      sp += m[i] * ((dRI[i][0] * u[0] + dRI[i][1] * u[1] + dRI[i][2] * u[2]) + (RI[i][0] * v[0] + RI[i][1] * v[1] + RI[i][2] * v[2]) + t1[i]);
    const double Me[3] = {e == 0 ? M0[0] : e == 1 ? M1[0] : 0.0, e == 0 ? M0[1] : e == 1 ? M1[1] : 0.0, e == 0 ? M0[2] : e == 1 ? M1[2] : 1.0};
    mat3_vec(Iw, Me, t2);
    const double sv = dot3(m, t2);
    for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_ANG, A.poly, bb, e), sp * Hp[bb] + sv * Hv[bb], true);
  }
}

// PhaseDurations::IsContactPhase (phase_durations.cc:120-124) over the optimised durations
TG_HD bool sched_is_contact(const Ctx& c, int ee, bool contact0, double t) {
  const SchedInfo si = c.sched[ee];
  const double last = last_phase_duration(c, si), eps = 1e-10;
  double acc = 0.0;
  int id = si.n_phases - 1;
  for (int ph = 0; ph < si.n_phases; ++ph) {
    acc += phase_duration(c, si, last, ph);
    if (acc >= t - eps) { id = ph; break; }
  }
  return (id % 2 == 0) ? contact0 : !contact0;
}

// EEBasePosCost sample (ee_base_pos_cost.cc:57-162), only while the foot swings: w |R^T (p_ee - p_b) - p_ref|^2.
// The reference adds no schedule block (:150-154); neither does this engine.
template <class Emit>
TG_HD void cost_eebp(const Ctx& c, const CostItem& it, Emit& em) {
  const int ee = it.ee;
  if (c.gait && sched_is_contact(c, ee, it.a0 != 0, it.t)) return;   // fixed gait: filtered at build
  SplinePt L, A, P;
  spline_eval(c, SP_BASE_LIN, it.t, L);
  spline_eval(c, SP_BASE_ANG, it.t, A);
  spline_eval(c, sp_motion(ee), it.t, P);
  double R[3][3]; base_rot(c, A, R);
  const double rW[3] = {P.p[0] - L.p[0], P.p[1] - L.p[1], P.p[2] - L.p[2]};
  double e3[3], m[3], mW[3];
  for (int i = 0; i < 3; ++i) e3[i] = (R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2]) - it.p[i];
  em.f += it.w * dot3(e3, e3);
  for (int i = 0; i < 3; ++i) m[i] = (2.0 * it.w) * e3[i];
  for (int j = 0; j < 3; ++j) mW[j] = m[0] * R[j][0] + m[1] * R[j][1] + m[2] * R[j][2];   // m b_R_w
  double H[4];
  spline_basis(P, kPos, H);
  for (int j = 0; j < 3; ++j) emit_dim(c, em, 0, sp_motion(ee), P, H, j, mW[j]);
  spline_basis(L, kPos, H);
  for (int j = 0; j < 3; ++j)
    for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_LIN, L.poly, bb, j), -mW[j] * H[bb], true);
  spline_basis(A, kPos, H);   // DerivOfRotVecMult(t, r_W, inverse = true)
  if (c.rotvec) {
    double JL[3][3], Am[3][3];
    rv_left_jac(A.p, JL);
    rv_rotvec_mult(R, JL, rW, true, Am);
    for (int e = 0; e < 3; ++e) {
      const double s = m[0] * Am[0][e] + m[1] * Am[1][e] + m[2] * Am[2][e];
      for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_ANG, A.poly, bb, e), s * H[bb], true);
    }
    return;
  }
  const Trig q = trig(A.p);
  for (int e = 0; e < 3; ++e) {
    double dR[3][3]; euler_dR_axis(q, e, dR);
    double s = 0.0;
    for (int r = 0; r < 3; ++r) s += m[r] * (rW[0] * dR[0][r] + rW[1] * dR[1][r] + rW[2] * dR[2][r]);
    for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_ANG, A.poly, bb, e), s * H[bb], true);
  }
}

// BaseHeightCost sample (base_height_cost.cc:55-142, the fork's biped driver): w dt dev^2 with
// dev = p_z(base) - (mean z of the feet in contact + target), or the terrain height under the base
// when no foot is in contact. Its gradient is the reference's: only the base-linear nodes, through
// d p_z / d nodes; the target's dependence on the feet and the terrain is not differentiated.
template <class Emit>
TG_HD void cost_bhc(const Ctx& c, const CostItem& it, Emit& em) {
  SplinePt L;
  spline_eval(c, SP_BASE_LIN, it.t, L);
  double total = 0.0;
  int cnt = 0;
  for (int ee = 0; ee < c.rb.n_ee; ++ee) {
    const bool contact = it.a1 >= 0 ? ((it.a1 >> ee) & 1) != 0 : sched_is_contact(c, ee, ((it.a0 >> ee) & 1) != 0, it.t);
    if (!contact) continue;
    SplinePt P;
    spline_eval(c, sp_motion(ee), it.t, P);
    total += P.p[2];
    ++cnt;
  }
  const double avg = cnt == 0 ? ter_h(*c.ter, L.p[0], L.p[1]) : total / cnt;
  const double dev = L.p[2] - (avg + it.p[0]);
  em.f += it.w * dev * dev * it.wdt;   // weight_ * deviation * deviation * dt_ (it.wdt = dt here)
  const double s = 2.0 * it.w * dev * it.wdt;
  double H[4];
  spline_basis(L, kPos, H);
  for (int bb = 0; bb < 4; ++bb) em(0, basis_col(c, SP_BASE_LIN, L.poly, bb, 2), s * H[bb], true);
}

template <class Emit>
TG_HD void eval_cost_item(const Ctx& c, const CostItem& it, Emit& em) {
  switch (it.type) {
    case CT_NODE: cost_node(c, it, em); break;
    case CT_ENERGY: cost_energy(c, it, em); break;
    case CT_ANGMOM: cost_angmom(c, it, em); break;
    case CT_EEBP: cost_eebp(c, it, em); break;
    case CT_ENERGYQ: cost_energy_q(c, it, em); break;
    case CT_BHC: cost_bhc(c, it, em); break;
  }
}

// Gradient emitters of the objective kernel (cost_traj.hip), single-source so that the host emulation
// (tests/host_emu) runs the kernel's exact accumulation. Both give the same bits on every call.
// CostSlotEmit (fixed phase durations): an item's present entries (a variable's column: not a constant
// node value, which is -1 on the host and the zero slot n on the device) go, in emission order, to the
// slots slot[0], slot[1], ... of its range of Layout::cost_cslot (layout.hip build_cost_slots enumerates the
// same entries).
struct CostSlotEmit {
  double* cs;
  const uint16_t* slot;
  int n;
  double f = 0.0;
  static constexpr bool kSparse = true;
  TG_HD void skip(int) {}
  TG_HD void operator()(int, int col, double v, bool pres) {
    if (pres && col >= 0 && col < n) cs[*slot++] = v;
  }
};
struct CostFEmit {   // f only
  double f = 0.0;
  static constexpr bool kSparse = true;
  TG_HD void skip(int) {}
  TG_HD void operator()(int, int, double, bool) {}
};
// CostLimbEmit (phase-duration optimisation): an entry v is added as the exact fixed-point integer
// v * 2^60 split into three signed 42-bit limbs, accumulator k of column j at acc[k * n_pad + j]
// (64-bit integer atomics on the device). Integer sums do not depend on the order of the additions.
// Entries below 2^-60 in magnitude are truncated (the parity floor is 1e-12); a NaN, an infinity or
// |v| >= 2^65 sets *bad (the kernel then returns a NaN gradient). Exact while a column has fewer than
// 2^11 entries (its limb sums stay below 2^53 and convert to double exactly).
constexpr unsigned long long kLimbMask = (1ull << 42) - 1;
TG_HD long long limb_of(unsigned long long m, int s) {   // bits [0, 42) of m * 2^s
  if (s >= 42 || s <= -64) return 0;
  return (long long)((s >= 0 ? (m << s) : (m >> -s)) & kLimbMask);
}
TG_HD double limb_value(long long l0, long long l1, long long l2) {
  return ((double)l2 * 0x1p24 + (double)l1 * 0x1p-18) + (double)l0 * 0x1p-60;
}
struct CostLimbEmit {
  unsigned long long* acc;
  int n_pad;
  int* bad;
  double f = 0.0;
  static constexpr bool kSparse = true;   // zero entries need no addition
  TG_HD void skip(int) {}
  TG_HD void operator()(int, int col, double v, bool pres) {
    if (!pres || v == 0.0 || col < 0) return;
    unsigned long long bits;
    __builtin_memcpy(&bits, &v, sizeof bits);
    const int ex = (int)((bits >> 52) & 0x7ff);
    if (ex == 0) return;                                        // subnormal: below the resolution
    const int sh = ex - 1075 + 60;                              // v * 2^60 = m * 2^sh
    if (ex == 0x7ff || sh > 126 - 53) { *bad = 1; return; }     // NaN / inf / |v| >= 2^65
    const unsigned long long m = (bits & ((1ull << 52) - 1)) | (1ull << 52);
    long long l0 = limb_of(m, sh), l1 = limb_of(m, sh - 42), l2 = limb_of(m, sh - 84);
    if (bits >> 63) { l0 = -l0; l1 = -l1; l2 = -l2; }
#if defined(__HIP_DEVICE_COMPILE__)
    if (l0) atomicAdd(acc + col, (unsigned long long)l0);
    if (l1) atomicAdd(acc + n_pad + col, (unsigned long long)l1);
    if (l2) atomicAdd(acc + 2 * n_pad + col, (unsigned long long)l2);
#else
    acc[col] += (unsigned long long)l0;
    acc[n_pad + col] += (unsigned long long)l1;
    acc[2 * n_pad + col] += (unsigned long long)l2;
#endif
  }
};

// ----------------------------------------------------------------------------------------------
// Trajectory export (SaveTrajectoryToCSV, towr/src/utils/save_data.cpp:9-130): one row per sample
// time, columns (traj_cols = 19 + 25 E):
//   time | base-lin p v a | base-ang p v a (the raw spline: Euler angles or rotation vector and their
//   time derivatives, as the reference writes them) | per ee: motion p v a | ee-ang p v a |
//   force p | torque p | is_contact (PhaseDurations::IsContactPhase, phase_durations.cc:120-124)
// ----------------------------------------------------------------------------------------------
TG_HD int traj_cols(int E) { return 19 + 25 * E; }
// fixed phase durations (no phase-duration optimisation): [ee * TOWR_MAX_PHASES + phase], counts,
// contact at start
struct TrajPhases { const double* d; const int32_t* n; const int32_t* c0; };

// Spline::GetPoint at an arbitrary time (spline.cc:80-93): the segment scan, then the polynomial
TG_HD void spline_eval_at(const Ctx& c, int s, double t, SplinePt& o) {
  o.H = nullptr;
  if (c.gait && c.spl[s].ee >= 0) {
    o.dyn = true;
    phase_spline_locate(c, s, t, o);
  } else {
    o.dyn = false;
    const SplineMeta m = c.spl[s];
    o.poly = seg_lookup(c.dur + m.dur_off, m.n_polys, t, &o.tl);
    o.T = c.dur[m.dur_off + o.poly];
  }
  poly_state(c, s, o.poly, o.T, o.tl, o);
}

TG_HD void traj_row(const Ctx& c, const TrajPhases& ph, double t, double* row, int stride) {
  const int E = c.rb.n_ee;
  row[0] = t;
  SplinePt P;
  for (int s = 0; s < 2; ++s) {   // base-lin, base-ang
    spline_eval_at(c, s, t, P);
    for (int e = 0; e < 3; ++e) {
      row[(1 + 9 * s + e) * stride] = P.p[e];
      row[(4 + 9 * s + e) * stride] = P.v[e];
      row[(7 + 9 * s + e) * stride] = P.a[e];
    }
  }
  for (int ee = 0; ee < E; ++ee) {
    const int b = 19 + 25 * ee;
    spline_eval_at(c, sp_motion(ee), t, P);
    for (int e = 0; e < 3; ++e) { row[(b + e) * stride] = P.p[e]; row[(b + 3 + e) * stride] = P.v[e]; row[(b + 6 + e) * stride] = P.a[e]; }
    spline_eval_at(c, sp_ang(ee), t, P);
    for (int e = 0; e < 3; ++e) { row[(b + 9 + e) * stride] = P.p[e]; row[(b + 12 + e) * stride] = P.v[e]; row[(b + 15 + e) * stride] = P.a[e]; }
    spline_eval_at(c, sp_force(ee), t, P);
    for (int e = 0; e < 3; ++e) row[(b + 18 + e) * stride] = P.p[e];
    spline_eval_at(c, sp_torque(ee), t, P);
    for (int e = 0; e < 3; ++e) row[(b + 21 + e) * stride] = P.p[e];
    bool contact;
    if (c.gait) contact = sched_is_contact(c, ee, ph.c0[ee] != 0, t);
    else {
      double tl;
      const int id = seg_lookup(ph.d + ee * TOWR_MAX_PHASES, ph.n[ee], t, &tl);
      contact = (id % 2 == 0) ? (ph.c0[ee] != 0) : (ph.c0[ee] == 0);
    }
    row[(b + 24) * stride] = contact ? 1.0 : 0.0;
  }
}

template <class Emit>
TG_HD void eval_item(const Ctx& c, const ItemDesc& it, Emit& em) {
  switch (it.type) {
    case IT_NONE: break;
    case IT_DYN: eval_dyn(c, it, em); break;
    case IT_ROM: eval_rom(c, it, em); break;
    case IT_FDISC: eval_fdisc(c, it, em); break;
    case IT_FNODE: eval_fnode(c, it, em); break;
    case IT_TERR: eval_height(c, it, sp_motion(it.ee), 0.0, em); break;
    case IT_BMOT: eval_bmot(c, it, em); break;
    case IT_SACC: eval_sacc(c, it, em); break;
    case IT_BHGT: eval_height(c, it, SP_BASE_LIN, it.p0, em); break;
    case IT_SWING: eval_swing(c, it, em); break;
    case IT_TDUR: eval_tdur(c, it, em); break;
    case IT_TQDISC: eval_tqdisc(c, it, em); break;
    case IT_TQNODE: eval_tqnode(c, it, em); break;
    case IT_THARD: eval_thard(c, it, em); break;
    case IT_EELIN: eval_eelin(c, it, em); break;
    case IT_LINEQ: eval_lineq(c, it, em); break;
  }
}

}  // namespace tg
