// gs_cls.h — the per-class arithmetic of the phase-duration path's composers (gstream.hip) as single-source
// __host__ __device__ code: the active-window basis sums, the record's view of an instant and each class's
// entry expression (RomCls / DynCls / TqCls::value), and the TorqueConstraintDiscretized record builder, so
// the test-only host emulation (tests/host_emu) runs exactly the composer's expressions on the CPU.
#pragma once

#include "engine_math.h"
#include "layout.h"

namespace tg {

// two int fields of a record in one double: lo is dword 2 j, hi dword 2 j + 1 of the record's int area (the composer
// reads them in place)
TG_HD double gs_int2(int lo, int hi) {
  return __builtin_bit_cast(double, (unsigned long long)(uint32_t)lo | ((unsigned long long)(uint32_t)hi << 32));
}

// The active-window basis sums of one PhaseSpline at one instant, from the block's PhaseSpline tables
// (Ctx: SplineMeta, pact, PhaseCol in LDS): sums[e][q] = emit_dim's basis sum of the dimension's PhaseCol
// qa[e] + q (phase_basis_sum), qa[e] = the polynomial's first active PhaseCol (1 << 24: none)
TG_HD void gs_window(const Ctx& c, int s, int poly, const double H[4], double sums[3][kGsAct], int qa[3]) {
  const SplineMeta& m = c.spl[s];
  double h0 = H[0], h1 = H[1], h2 = H[2], h3 = H[3];
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));   // opaque: no runtime-indexed H (scratch)
#endif
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int32_t* w = c.pact + m.pact_off + 2 * (e * m.n_polys + poly);
    const int a = w[0], z = w[1];
    qa[e] = z >= a ? a : (1 << 24);
#pragma unroll
    for (int q = 0; q < kGsAct; ++q) sums[e][q] = a + q <= z ? phase_basis_sum(c.pcols[m.pcol_off[e] + a + q], poly, h0, h1, h2, h3) : 0.0;
  }
}

// SchedJac's sched_val from a record in LDS (dx, v) with the instant's phase and the ee's phase count
TG_HD double gs_sched_val(const double* dx, const double* v, int cur, int n, int k, int col) {
  const bool last = cur == n - 1;
  if (col == cur && !last) return dx[k];
  if (col < cur) return last ? -v[k] - dx[k] : -v[k];
  return 0.0;
}
// Per-class pieces of the composer (gs_compose): an instant's record in LDS is its RS fields
// (stride RS | 1, layout.h record format); ci = its int fields, int j at ci[j] (gs_int2);
//   poly(): the active polynomial of a PhaseSpline segment's spline at the instant;
//   value(): value q of a segment at the instant (the tile path's expression for that entry).
struct RomCls {
  TG_HD static int poly(const int32_t* ci, int, int) { return ci[4]; }
  TG_HD static double value(const RobotC& rb, const int32_t* tmpl, const GsSeg& sg, int pos, const double* d, const int32_t* ci,
                                 const uint8_t* pcl, int nph) {
    const int r = sg.r;
    if (sg.type == 0) {   // base prefix (eval_rom groups 0 and 1)
      const int code = pcl[sg.toff + pos];
      const int e = (code >> 2) & 3, bb = code & 3;
      return (code >> 4) == 0 ? -d[3 * e + r] * d[9 + bb]     // -R[e][r] * HL[b]
                              : d[13 + 3 * e + r] * d[22 + bb];   // Ag[e][r] * HA[b]
    }
    const int32_t t = tmpl[sg.toff + pos];
    if (sg.type == 2) {   // R^T d pos / d schedule (:123-130)
      const int col = t & 0xFFFF, cur = ci[0];
      return d[r] * gs_sched_val(d + 26, d + 29, cur, nph, 0, col) + d[3 + r] * gs_sched_val(d + 26, d + 29, cur, nph, 1, col) +
             d[6 + r] * gs_sched_val(d + 26, d + 29, cur, nph, 2, col);
    }
    const int e = (t >> 22) & 3, q = t & 0x3FFFFF;   // motion PhaseCol: R[e][r] * basis sum (emit_dim)
    const unsigned rel = (unsigned)(q - ci[1 + e]);
    return rel < (unsigned)kGsAct ? d[3 * e + r] * d[32 + e * kGsAct + rel] : 0.0;
  }
};

struct DynCls {
  // an endeffector's ints (layout.h): curX | qaX[3] | polyX | - | curF | qaF | polyF | - | qaT | polyT
  TG_HD static int poly(const int32_t* ci, int kind, int ee) { return ci[2 * ee * kDynEeNI + (kind == 0 ? 4 : kind == 1 ? 8 : 11)]; }
  TG_HD static double value(const RobotC& rb, const int32_t* tmpl, const GsSeg& sg, int pos, const double* d, const int32_t* ci,
                                 const uint8_t* pcl, const int32_t* nph) {
    const int r = sg.r;
    if (sg.type == 0) {   // base prefix
      const int code = pcl[sg.toff + pos];
      const int e = (code >> 2) & 3, bb = code & 3;
      if ((code >> 4) == 0)   // base-linear: -Cross(sum f)[r][e] Hp (dyn_g0_b), m Ha (dyn_g0_a)
        return r < 3 ? -cross_el(d, r, e) * d[6 + bb] : rb.m * d[10 + bb];
      // base-angular: Ap[r] Hp + Av[r] Hv + Aa[r] Ha of axis e (eval_dyn group 1)
      return d[14 + 9 * e + r] * d[41 + bb] + d[14 + 9 * e + 3 + r] * d[45 + bb] + d[14 + 9 * e + 6 + r] * d[49 + bb];
    }
    const int32_t t = tmpl[sg.toff + pos];
    const int ee = sg.ee;
    const double* de = d + kDynBaseND + ee * kDynEeND;
    const int32_t* ii = ci + 2 * ee * kDynEeNI;
    if (sg.type == 2) {   // d/d ee schedule (eval_dyn, dynamic_constraint.cc:116-122)
      const int col = t & 0xFFFF, n = nph[ee];
      if (r >= 3) return -gs_sched_val(de + 6, de + 9, ii[6], n, r - 3, col);
      const int e1 = r == 2 ? 0 : r + 1, e2 = r == 0 ? 2 : r - 1;
      const double a = cross_el(de + 3, r, e1) * gs_sched_val(de + 6, de + 9, ii[6], n, e1, col) +
                       cross_el(de + 3, r, e2) * gs_sched_val(de + 6, de + 9, ii[6], n, e2, col);
      const double bq = cross_el(de, r, e1) * gs_sched_val(de + 12, de + 15, ii[0], n, e1, col) +
                        cross_el(de, r, e2) * gs_sched_val(de + 12, de + 15, ii[0], n, e2, col);
      return a + bq;
    }
    const int kind = sg.kind, e = (t >> 22) & 3, q = t & 0x3FFFFF;
    const unsigned rel = (unsigned)(q - ii[kind == 0 ? 1 + e : kind == 1 ? 7 : 10]);
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double v = de[dyn_sum_field(kind, e, rel)];
    // emit_dim scales: motion Cross(f)[r][e]; force Cross(rv)[r][e] (angular) or -1 (linear); torque -1
    const double sc = kind == 0 ? cross_el(de, r, e) : kind == 1 ? (r < 3 ? cross_el(de + 3, r, e) : -1.0) : -1.0;
    return sc * v;
  }
};

// TorqueConstraintDiscretized rows r = 0..3 scale the torque window by tb[r] = t1, t2, n, -n and (rows 2,
// 3) the force window by b = -k mu n; a schedule column is eval_tqdisc's sum of the two linear forms
struct TqCls {
  TG_HD static int poly(const int32_t* ci, int kind, int) { return ci[kind == 2 ? 3 : 4]; }   // cur | qaT | qaF | polyT | polyF
  TG_HD static double tb(const double* d, int r, int e) { return r == 3 ? -d[6 + e] : d[3 * r + e]; }
  TG_HD static double value(const RobotC& rb, const int32_t* tmpl, const GsSeg& sg, int pos, const double* d, const int32_t* ci,
                                 const uint8_t*, int nph) {
    (void)rb;
    const int r = sg.r;
    const int32_t t = tmpl[sg.toff + pos];
    if (sg.type == 2) {   // d / d schedule (torque_constraint_discretized.cc:210-234)
      const int col = t & 0xFFFF, cur = ci[0];
      double v = tb(d, r, 0) * gs_sched_val(d + 12, d + 15, cur, nph, 0, col) + tb(d, r, 1) * gs_sched_val(d + 12, d + 15, cur, nph, 1, col) +
                 tb(d, r, 2) * gs_sched_val(d + 12, d + 15, cur, nph, 2, col);
      if (r >= 2)
        v += d[9] * gs_sched_val(d + 18, d + 21, cur, nph, 0, col) + d[10] * gs_sched_val(d + 18, d + 21, cur, nph, 1, col) +
             d[11] * gs_sched_val(d + 18, d + 21, cur, nph, 2, col);
      return v;
    }
    const int kind = sg.kind, e = (t >> 22) & 3, q = t & 0x3FFFFF;   // torque (kind 2) or force (1) PhaseCol
    const unsigned rel = (unsigned)(q - ci[kind == 2 ? 1 : 2]);   // (one first PhaseCol for the three dimensions)
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double sum = d[(kind == 2 ? 24 : 28) + rel];   // (one set for the three dimensions, layout.h)
    return (kind == 2 ? tb(d, r, e) : d[9 + e]) * sum;   // emit_dim: scale * basis sum
  }
};

// One TorqueConstraintDiscretized instant's record (layout.h record format, GS_TQ) through put(field, value),
// and its 4 g rows: eval_tqdisc's quantities (torque_constraint_discretized.cc:101-235) in the composer's form,
// without the motion block (a terrain without curvature: every motion scale is exactly 0.0, skipped at :57)
template <class Put>
TG_HD void tq_record(const Ctx& c, const GsInst& gi, Put&& put, double g[4]) {
  const int ee = gi.ee;
  const double t = gi.t, kf = gi.p0, mu = c.ter->friction_coeff;
  SplinePt Pm, F, Tq;
  spline_eval(c, sp_motion(ee), t, Pm);
  spline_eval(c, sp_force(ee), t, F);
  spline_eval(c, sp_torque(ee), t, Tq);
  double n[3], t1[3], t2[3];
  ter_nbasis(*c.ter, 0, Pm.p[0], Pm.p[1], n);
  ter_nbasis(*c.ter, 1, Pm.p[0], Pm.p[1], t1);
  ter_nbasis(*c.ter, 2, Pm.p[0], Pm.p[1], t2);
  const double tau_n = dot3(Tq.p, n), tz_lim = kf * mu * dot3(F.p, n);   // g rows (:101-125)
  g[0] = dot3(Tq.p, t1);
  g[1] = dot3(Tq.p, t2);
  g[2] = tau_n - tz_lim;
  g[3] = -tau_n - tz_lim;
#pragma unroll
  for (int e = 0; e < 3; ++e) { put(e, t1[e]); put(3 + e, t2[e]); put(6 + e, n[e]); put(9 + e, -kf * mu * n[e]); }
  SchedJac Jt, Jf;   // the schedule rows (:210-234): torque and force linear forms (one endeffector: one phase index)
  sched_jac(c, sp_torque(ee), t, Tq, Jt);
  sched_jac(c, sp_force(ee), t, F, Jf);
#pragma unroll
  for (int e = 0; e < 3; ++e) { put(12 + e, Jt.dx[e]); put(15 + e, Jt.v[e]); put(18 + e, Jf.dx[e]); put(21 + e, Jf.v[e]); }
  double H[4], sums[3][kGsAct];
  int qa[3], qaT;
  // (the window sums of the three dimensions coincide: the layout checked the PhaseCols, spline_dims_coincide)
  spline_basis(Tq, kPos, H);   // AccumulateLinearFormJacobian of the torque spline (:147-155)
  gs_window(c, sp_torque(ee), Tq.poly, H, sums, qa);
  qaT = qa[0];
  put(kTqND, gs_int2(Jt.cur, qaT));
#pragma unroll
  for (int q = 0; q < kGsAct; ++q) put(24 + q, sums[0][q]);
  spline_basis(F, kPos, H);    // ... of the force spline into the normal-torque rows (:158-163)
  gs_window(c, sp_force(ee), F.poly, H, sums, qa);
#pragma unroll
  for (int q = 0; q < kGsAct; ++q) put(28 + q, sums[0][q]);
  put(kTqND + 1, gs_int2(qa[0], Tq.poly));
  put(kTqND + 2, gs_int2(F.poly, 0));
}

}  // namespace tg
