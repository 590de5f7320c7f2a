// gs_cls.h — the per-class arithmetic of the phase-duration path's composers (gstream.hip) as single-source
// __host__ __device__ code: the active-window basis sums, the record's view of an instant and each class's
// entry expression (RomCls / DynCls / TqCls::value), and the TorqueConstraintDiscretized record builder, so
// the test-only host emulation (tests/host_emu) runs exactly the composer's expressions on the CPU.
#pragma once

#include "engine_math.h"
#include "layout.h"

namespace tg {

// an int field of a record: its 64-bit integer bit pattern (the composer reads the low dword in place)
TG_HD double gs_int(int v) { return __builtin_bit_cast(double, (long long)v); }

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
// (stride RS | 1, layout.h record format); ci = its int fields, field j at ci[2 j] (gs_int);
//   poly(): the active polynomial of a PhaseSpline segment's spline at the instant;
//   value(): value q of a segment at the instant (the tile path's expression for that entry).
struct RomCls {
  TG_HD static int poly(const int32_t* ci, int, int) { return ci[8]; }
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
    const unsigned rel = (unsigned)(q - ci[2 + 2 * e]);
    return rel < (unsigned)kGsAct ? d[3 * e + r] * d[32 + e * kGsAct + rel] : 0.0;
  }
};

struct DynCls {
  TG_HD static int poly(const int32_t* ci, int kind, int ee) { return ci[2 * (ee * kDynEeNI + 11 + kind)]; }
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
      if (r >= 3) return -gs_sched_val(de + 6, de + 9, ii[0], n, r - 3, col);
      const int e1 = r == 2 ? 0 : r + 1, e2 = r == 0 ? 2 : r - 1;
      const double a = cross_el(de + 3, r, e1) * gs_sched_val(de + 6, de + 9, ii[0], n, e1, col) +
                       cross_el(de + 3, r, e2) * gs_sched_val(de + 6, de + 9, ii[0], n, e2, col);
      const double bq = cross_el(de, r, e1) * gs_sched_val(de + 12, de + 15, ii[2], n, e1, col) +
                        cross_el(de, r, e2) * gs_sched_val(de + 12, de + 15, ii[2], n, e2, col);
      return a + bq;
    }
    const int kind = sg.kind, e = (t >> 22) & 3, q = t & 0x3FFFFF;
    const unsigned rel = (unsigned)(q - ii[2 * (2 + 3 * kind + e)]);
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double v = de[18 + (kind * 3 + e) * kGsAct + rel];
    // emit_dim scales: motion Cross(f)[r][e]; force Cross(rv)[r][e] (angular) or -1 (linear); torque -1
    const double sc = kind == 0 ? cross_el(de, r, e) : kind == 1 ? (r < 3 ? cross_el(de + 3, r, e) : -1.0) : -1.0;
    return sc * v;
  }
};

// TorqueConstraintDiscretized rows r = 0..3 scale the torque window by tb[r] = t1, t2, n, -n and (rows 2,
// 3) the force window by b = -k mu n; a schedule column is eval_tqdisc's sum of the two linear forms
struct TqCls {
  TG_HD static int poly(const int32_t* ci, int kind, int) { return ci[2 * (kind == 2 ? 7 : 8)]; }
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
    const unsigned rel = (unsigned)(q - ci[2 * (kind == 2 ? 1 + e : 4 + e)]);
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double sum = d[(kind == 2 ? 24 : 36) + e * kGsAct + rel];
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
  put(kTqND, gs_int(Jt.cur));
  double H[4], sums[3][kGsAct];
  int qa[3];
  spline_basis(Tq, kPos, H);   // AccumulateLinearFormJacobian of the torque spline (:147-155)
  gs_window(c, sp_torque(ee), Tq.poly, H, sums, qa);
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    put(kTqND + 1 + e, gs_int(qa[e]));
#pragma unroll
    for (int q = 0; q < kGsAct; ++q) put(24 + e * kGsAct + q, sums[e][q]);
  }
  spline_basis(F, kPos, H);    // ... of the force spline into the normal-torque rows (:158-163)
  gs_window(c, sp_force(ee), F.poly, H, sums, qa);
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    put(kTqND + 4 + e, gs_int(qa[e]));
#pragma unroll
    for (int q = 0; q < kGsAct; ++q) put(36 + e * kGsAct + q, sums[e][q]);
  }
  put(kTqND + 7, gs_int(Tq.poly));
  put(kTqND + 8, gs_int(F.poly));
}

// ------------------------------------------------------------------------------------------------
// The fused ForceConstraintDiscretized kernel's stages (gstream.hip towr_fdisc_fused_kernel), single-source so that
// the host emulation (tests/host_emu emu_ff_check) runs exactly them. A view of one (problem, constraint): its blob
// (layout.h FfGeo), the local x (motion node values, force node values, schedule variables) and the timings.
// Every quantity is formed by the function the record kernel uses for it (fdisc_instant / fdisc_record), split
// over kFfLanes lanes per instant (sub).
// ------------------------------------------------------------------------------------------------
enum { kXfT = 0, kXfTl, kXfPoly, kXmT, kXmTl, kXmPoly, kXcur, kXws, kXwd, kXFp, kXFv = kXFp + 3, kXMp = kXFv + 3,
       kXH = kXMp + 2, kXb = kXH + 4, kFfEx = kXb + 16 };   // per-instant exchange slots (doubles) between the stages
TG_HD int gs_iget(double d) { return (int)__builtin_bit_cast(long long, d); }
struct FfView {
  FfGeo g;
  const int32_t* blob;
  const double* lx;          // local x: motion node values (node j at 6 j + 3 deriv + dim), force node values, schedule
  double *pdm, *pem, *pdf, *pef, *phe;   // polynomial durations and running sums (motion, force), phase ends
  const towr_terrain_t* ter;
  TG_HD const PolyPhase* pim() const { return reinterpret_cast<const PolyPhase*>(blob + g.o_pinfo); }
  TG_HD const PolyPhase* pif() const { return pim() + g.np_m; }
  TG_HD const double* sx() const { return lx + 6 * (g.nm + g.nf); }
  TG_HD const double* nvm() const { return lx; }
  TG_HD const double* nvf() const { return lx + 6 * g.nm; }
  // PhaseDurations (phase_durations.cc:79-100): the last phase is the total minus the others (last_phase_duration)
  TG_HD double last_phase() const {
    double sum = 0.0;
    for (int i = 0; i < g.n_ph - 1; ++i) sum += sx()[i];
    return g.t_total - sum;
  }
  TG_HD double phase_dur(int ph, double last) const { return ph < g.n_ph - 1 ? sx()[ph] : last; }
};
// timings, step 1: polynomial duration i of the motion (i < np_m) or force spline (phase_poly_duration)
TG_HD void ff_pdur(const FfView& v, int i) {
  const double last = v.last_phase();
  const bool f = i >= v.g.np_m;
  const PolyPhase pp = f ? v.pif()[i - v.g.np_m] : v.pim()[i];
  (f ? v.pdf[i - v.g.np_m] : v.pdm[i]) = v.phase_dur(pp.phase, last) / pp.n_in_phase;
}
// timings, step 2 (which 0: motion running sums, 1: force, 2: phase ends), in the reference's order
TG_HD void ff_sums(const FfView& v, int which) {
  if (which == 2) {
    const double last = v.last_phase();
    double acc = 0.0;
    for (int ph = 0; ph < v.g.n_ph; ++ph) { acc += v.phase_dur(ph, last); v.phe[ph] = acc; }
    return;
  }
  const double* d = which ? v.pdf : v.pdm;
  double* out = which ? v.pef : v.pem;
  const int n = which ? v.g.np_f : v.g.np_m;
  double acc = 0.0;
  for (int i0 = 0; i0 < n; i0 += 8) {   // (operands loaded 8 at a time ahead of the dependent additions)
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = i0 + k < n ? d[i0 + k] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (i0 + k < n) { acc += x[k]; out[i0 + k] = acc; }
  }
}
// stage 1 (sub 0: force, 1: motion, 2: phase): the active polynomials and phase at time t
TG_HD void ff_stage1(const FfView& v, double t, int sub, double* X) {
  if (sub < 2) {
    int poly; double tl, T;
    if (sub == 0) locate_poly(v.pdf, v.pef, v.g.np_f, t, poly, tl, T);
    else locate_poly(v.pdm, v.pem, v.g.np_m, t, poly, tl, T);
    const int o = sub == 0 ? kXfT : kXmT;
    X[o] = T; X[o + 1] = tl; X[o + 2] = gs_int(poly);
  } else if (sub == 2) {
    X[kXcur] = gs_int(phase_cur(v.phe, v.g.n_ph, t));
  }
}
// stage 2 (sub 0-2: force dimension, 3-4: motion x / y, 5: the force basis, 6: the window): poly_state_dim, hermite_dpos
TG_HD void ff_stage2(const FfView& v, int sub, double* X) {
  if (sub < 5) {
    const bool f = sub < 3;
    const int e = f ? sub : sub - 3, o = f ? kXfT : kXmT;
    const int poly = gs_iget(X[o + 2]);
    const double* nv = f ? v.nvf() : v.nvm();
    double pp, vv, aa;
    poly_state_dim(nv[6 * poly + e], nv[6 * poly + 3 + e], nv[6 * poly + 6 + e], nv[6 * poly + 9 + e], X[o], X[o + 1], pp, vv, aa);
    if (f) { X[kXFp + e] = pp; X[kXFv + e] = vv; }
    else X[kXMp + e] = pp;
  } else if (sub == 5) {
    double H[4];
    hermite_dpos(X[kXfT], X[kXfTl], H);
    for (int q = 0; q < 4; ++q) X[kXH + q] = H[q];
  } else if (sub == 6) {
    const int32_t* ws = v.blob + v.g.o_ws + 2 * gs_iget(X[kXfPoly]);
    X[kXws] = gs_int(ws[0]);
    X[kXwd] = gs_int(ws[1]);
  }
}
// stage 3 (sub 0-2: d force / d schedule dimension, 3: the pyramid rows, 4-15: window position sub - 4): the record
// fields (fdisc_record's layout: window sums | b | Jf.dx | Jf.v | ws, wd, cur); the rows b also to the exchange
TG_HD void ff_stage3(const FfView& v, int sub, double* X, double* R) {
  const int poly = gs_iget(X[kXfPoly]);
  if (sub < 3) {
    const int k = sub;
    const double* nv = v.nvf();
    R[kFsDx + k] = sched_dx_dim(nv[6 * poly + k], nv[6 * poly + 3 + k], nv[6 * poly + 6 + k], nv[6 * poly + 9 + k], X[kXfT], X[kXfTl],
                                X[kXFv + k], v.pif()[poly]);
    R[kFsV + k] = X[kXFv + k];
    if (k == 0) { R[kFsND] = X[kXws]; R[kFsND + 1] = X[kXwd]; R[kFsND + 2] = X[kXcur]; }
  } else if (sub == 3) {
    double nb[3][3], bb[5][3];
    ter_nbasis(*v.ter, 0, X[kXMp], X[kXMp + 1], nb[0]);
    ter_nbasis(*v.ter, 1, X[kXMp], X[kXMp + 1], nb[1]);
    ter_nbasis(*v.ter, 2, X[kXMp], X[kXMp + 1], nb[2]);
    pyramid(nb[0], nb[1], nb[2], v.ter->friction_coeff, bb);
    for (int i = 0; i < 5; ++i)
      for (int e = 0; e < 3; ++e) { R[kFsB + 3 * i + e] = bb[i][e]; X[kXb + 3 * i + e] = bb[i][e]; }
  } else if (sub < 4 + kFsWin) {   // emit_dim's basis sum of the template column at window position q (0 past the row)
    const int q = sub - 4, pos = gs_iget(X[kXws]) + q;
    const int32_t te = pos < v.g.L ? v.blob[v.g.o_tmpl + pos] : -1;
    double h0 = X[kXH], h1 = X[kXH + 1], h2 = X[kXH + 2], h3 = X[kXH + 3];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
#endif
    const PhaseCol* pc = reinterpret_cast<const PhaseCol*>(v.blob + v.g.o_pcols);
    R[q] = te >= 0 ? phase_basis_sum(pc[te & 0xFFFFFF], poly, h0, h1, h2, h3) : 0.0;
  }
}
// g row i of the instant (fdisc_instant: F . b_i)
TG_HD double ff_g(const double* X, int i) {
  const double Fp[3] = {X[kXFp], X[kXFp + 1], X[kXFp + 2]}, bi[3] = {X[kXb + 3 * i], X[kXb + 3 * i + 1], X[kXb + 3 * i + 2]};
  return dot3(Fp, bi);
}

}  // namespace tg
