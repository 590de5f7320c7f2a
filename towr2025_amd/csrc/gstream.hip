// gstream.hip — the streaming RangeOfMotion and Dynamic kernels under phase-duration optimisation
// (layout.h GsGeo, towr_gpu.hip launch_gstream). With OptimizePhaseDurations every endeffector spline is
// a PhaseSpline whose Jacobian keeps the full pattern of every polynomial (phase_spline.cc:45-51): ~90 %
// of a row's entries are exact zeros whose positions move with x. The tile path evaluated each instant
// once per row lane and scattered 8-byte value stores over a zero-filled range (RangeOfMotion wrote
// 2.66x, Dynamic 1.28x the algorithmic bytes: an isolated 8-byte store costs a 32-byte granule). Here:
//   record:  one block per problem stages x and the PhaseSpline tables once; each lane evaluates one
//            instant (Dynamic: one instant's base terms, one base-angular axis, or one endeffector)
//            with engine_math.h's item code and stores what the instant's Jacobian entries are built
//            from, field-major (a wave's stores coalesce);
//   compose: one block per (problem, GsBlock) reads its instants' records, forms the active-window
//            basis sums once per (instant, spline, dimension), then streams its whole CSR range with
//            16-byte non-temporal stores, each unit written once, zeros included.
// Every entry is the tile path's own expression (eval_rom / eval_dyn, cited per case), so parity is
// the tile path's parity.
#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"

namespace tg {
namespace {

constexpr int kGsRecBlock = 256;

// ------------------------------------------------------------------------------------------------
// records
// ------------------------------------------------------------------------------------------------
// RangeOfMotion (range_of_motion_constraint.cc:72-131, eval_rom): one lane per instant of every
// RangeOfMotion set; its 3 g rows go straight out.
template <bool ROTVEC>
__global__ void __launch_bounds__(kGsRecBlock, 2) towr_rom_rec_kernel(KParams P, double* rec, int64_t ldr, int32_t ni) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  Ctx c = gait_record_setup<kGsRecBlock>(P, b, smem);
  c.rotvec = ROTVEC;
  double* Rb = rec + (int64_t)b * ldr;
  double* Gb = P.G + (int64_t)b * P.ldg;
  for (int k = threadIdx.x; k < ni; k += kGsRecBlock) {
    const GsInst gi = P.gs_inst[k];
    c.row = gi.seg;
    const double t = gi.t;
    SplinePt L, A, M;
    spline_eval(c, SP_BASE_LIN, t, L);
    spline_eval(c, SP_BASE_ANG, t, A);
    spline_eval(c, sp_motion(gi.ee), t, M);
    double R[3][3];
    Trig q{};
    if constexpr (ROTVEC) rv_rodrigues(A.p, R);
    else { q = trig(A.p); euler_R(q, R); }
    const double rW[3] = {M.p[0] - L.p[0], M.p[1] - L.p[1], M.p[2] - L.p[2]};
    if (P.want_g)
      for (int i = 0; i < 3; ++i) __builtin_nontemporal_store(R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2], Gb + gi.row0 + i);
    double* r = Rb + k;
    auto put = [&](int f, double v) { r[(int64_t)f * ni] = v; };
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) put(3 * i + j, R[i][j]);
    double H[4];
    spline_basis(L, kPos, H);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) put(9 + bb, H[bb]);
    // base-angular coefficients Ag[e][r]: the entry at (axis e, basis b) of row r is Ag[e][r] HA[b]
    if constexpr (ROTVEC) {   // DerivOfRotVecMult(t, r_W, inverse = true): R^T [r_W]x J_L
      double JL[3][3], Am[3][3];
      rv_left_jac(A.p, JL);
      rv_rotvec_mult(R, JL, rW, true, Am);
#pragma unroll
      for (int e = 0; e < 3; ++e)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) put(13 + 3 * e + rr, Am[rr][e]);
    } else {                  // row r = sum_c rW[c] dR_e[c][r]
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        double dR[3][3]; euler_dR_axis(q, e, dR);
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) put(13 + 3 * e + rr, rW[0] * dR[0][rr] + rW[1] * dR[1][rr] + rW[2] * dR[2][rr]);
      }
    }
    spline_basis(A, kPos, H);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) put(22 + bb, H[bb]);
    put(26, (double)M.poly);
    spline_basis(M, kPos, H);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) put(27 + bb, H[bb]);
    SchedJac Jx;
    sched_jac(c, sp_motion(gi.ee), t, M, Jx);   // b_R_w * d pos / d schedule (:123-130)
#pragma unroll
    for (int e = 0; e < 3; ++e) { put(31 + e, Jx.dx[e]); put(34 + e, Jx.v[e]); }
    put(37, (double)Jx.cur);
  }
}

// Dynamic (dynamic_constraint.cc:63-148, single_rigid_body_dynamics.cc:76-204, eval_dyn). Lanes in
// ranges padded to whole waves, so a wave runs one path: per instant the base terms (dyn_g0_a's state),
// per (axis, instant) the base-angular coefficients (dyn_euler_axis / dyn_rv_column), per (endeffector,
// instant) the force / torque / motion PhaseSplines and their schedule Jacobians. The g rows need the
// endeffector sums and are written by the composer.
template <bool ROTVEC>
__global__ void __launch_bounds__(kGsRecBlock, 2) towr_dyn_rec_kernel(KParams P, double* rec, int64_t ldr, int32_t K) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  Ctx c = gait_record_setup<kGsRecBlock>(P, b, smem);
  c.rotvec = ROTVEC;
  const int E = P.rb.n_ee;
  double* Rb = rec + (int64_t)b * ldr;
  const int Kp = (K + 63) & ~63, EKp = (E * K + 63) & ~63;
  const int total = 4 * Kp + EKp;
  for (int i = threadIdx.x; i < total; i += kGsRecBlock) {
    if (i < Kp) {   // base terms of instant k
      const int k = i;
      if (k >= K) continue;
      const GsInst gi = P.gs_inst[k];
      c.row = gi.seg;
      ItemDesc it{};
      it.t = gi.t; it.row0 = gi.row0; it.seg = gi.seg;
      struct NoEmit {
        TG_HD void g(int, double) {}
        TG_HD void operator()(int, int, double, bool) {}
      } ne;
      DynG0 st;
      dyn_g0_a(c, it, ne, st);
      double* r = Rb + k;
      auto put = [&](int f, double v) { r[(int64_t)f * K] = v; };
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(e, st.ab[e]); put(3 + e, st.La[e]); put(6 + e, st.Lp[e]); }
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) { put(9 + bb, st.Hp[bb]); put(13 + bb, st.Ha[bb]); }
    } else if (i < 4 * Kp) {   // base-angular axis e of instant k
      const int e = (i - Kp) / Kp, k = (i - Kp) - e * Kp;
      if (k >= K) continue;
      const GsInst gi = P.gs_inst[k];
      c.row = gi.seg;
      double Ap[3], Av[3], Aa[3], Hp[4], Hv[4], Ha[4];
      if constexpr (ROTVEC) {
        DynRvState S;
        dyn_rv_state(c, gi.t, S);
        if (e == 0) dyn_rv_column<0>(S, Ap, Av, Aa);
        else if (e == 1) dyn_rv_column<1>(S, Ap, Av, Aa);
        else dyn_rv_column<2>(S, Ap, Av, Aa);
        if (e == 0) { spline_basis(S.A, kPos, Hp); spline_basis(S.A, kVel, Hv); spline_basis(S.A, kAcc, Ha); }
      } else {
        DynEulerState S;
        dyn_euler_state(c, gi.t, S);
        dyn_euler_axis(c, S, e, Ap, Av, Aa);
        if (e == 0) { spline_basis(S.A, kPos, Hp); spline_basis(S.A, kVel, Hv); spline_basis(S.A, kAcc, Ha); }
      }
      double* r = Rb + (int64_t)kDynBaseRec * K + e * K + k;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        r[(int64_t)(q) * 3 * K] = Ap[q];
        r[(int64_t)(3 + q) * 3 * K] = Av[q];
        r[(int64_t)(6 + q) * 3 * K] = Aa[q];
      }
      if (e == 0) {   // the base-angular basis of the instant, once
        double* h = Rb + (int64_t)(kDynBaseRec + 3 * kDynAxisRec) * K + k;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) { h[(int64_t)bb * K] = Hp[bb]; h[(int64_t)(4 + bb) * K] = Hv[bb]; h[(int64_t)(8 + bb) * K] = Ha[bb]; }
      }
    } else {   // endeffector ee of instant k
      const int idx = i - 4 * Kp;
      if (idx >= E * K) continue;
      const int ee = idx / K, k = idx - ee * K;
      const GsInst gi = P.gs_inst[k];
      c.row = gi.seg;
      const double t = gi.t;
      SplinePt F, Tq, M;
      spline_eval(c, sp_force(ee), t, F);
      spline_eval(c, sp_torque(ee), t, Tq);
      spline_eval(c, sp_motion(ee), t, M);
      double* r = Rb + (int64_t)(kDynBaseRec + 3 * kDynAxisRec + kDynHangRec) * K + idx;
      const int64_t st = (int64_t)E * K;
      auto put = [&](int f, double v) { r[f * st] = v; };
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(e, F.p[e]); put(3 + e, Tq.p[e]); put(6 + e, M.p[e]); }
      double H[4];
      put(9, (double)F.poly);
      spline_basis(F, kPos, H);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) put(10 + bb, H[bb]);
      put(14, (double)Tq.poly);
      spline_basis(Tq, kPos, H);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) put(15 + bb, H[bb]);
      put(19, (double)M.poly);
      spline_basis(M, kPos, H);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) put(20 + bb, H[bb]);
      SchedJac Jf, Jx;   // force and ee-position terms (dynamic_constraint.cc:116-122; no torque term)
      sched_jac(c, sp_force(ee), t, F, Jf);
      sched_jac(c, sp_motion(ee), t, M, Jx);
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(24 + e, Jf.dx[e]); put(27 + e, Jf.v[e]); put(31 + e, Jx.dx[e]); put(34 + e, Jx.v[e]); }
      put(30, (double)Jf.cur);
      put(37, (double)Jx.cur);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// composers
// ------------------------------------------------------------------------------------------------
// SchedJac's sched_val from a record in LDS (dx, v) with the instant's phase and the ee's phase count
__device__ __forceinline__ double gs_sched_val(const double* dx, const double* v, int cur, int n, int k, int col) {
  const bool last = cur == n - 1;
  if (col == cur && !last) return dx[k];
  if (col < cur) return last ? -v[k] - dx[k] : -v[k];
  return 0.0;
}
// The active-window basis sums of one PhaseSpline at one instant: sums[e][q] = emit_dim's basis sum of
// the dimension's PhaseCol qa[e] + q (phase_basis_sum), qa[e] = the polynomial's first active PhaseCol
__device__ __forceinline__ void gs_window(const KParams& P, int s, int poly, const double H[4], double* sums, int32_t* qa) {
  const SplineMeta m = P.spl[s];
  double h0 = H[0], h1 = H[1], h2 = H[2], h3 = H[3];
  asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
#pragma unroll
  for (int e = 0; e < 3; ++e) {
    const int32_t* w = P.pact + m.pact_off + 2 * (e * m.n_polys + poly);
    const int a = w[0], z = w[1];
    qa[e] = z >= a ? a : (1 << 24);
#pragma unroll
    for (int q = 0; q < kGsAct; ++q) sums[e * kGsAct + q] = a + q <= z ? phase_basis_sum(P.pcols[m.pcol_off[e] + a + q], poly, h0, h1, h2, h3) : 0.0;
  }
}

// block geometry in registers: row starts of an instant and the per-row-type prefix / template offsets
struct GsRows {
  int nrt, Li;
  int S[kGsRowTypes + 1], Pl[kGsRowTypes], To[kGsRowTypes], Po[kGsRowTypes];
  float invLi;
  __device__ __forceinline__ void load(const GsGeo& g, int t0) {
    nrt = g.nrt; Li = g.Li;
    S[0] = 0;
#pragma unroll
    for (int r = 0; r < kGsRowTypes; ++r) {
      S[r + 1] = S[r] + (r < g.nrt ? g.L[r] : 0);
      Pl[r] = g.P[r]; To[r] = g.T[r] - t0; Po[r] = g.poff[r];
    }
    invLi = 1.0f / (float)Li;
  }
  // entry e of the block (e < n_inst * Li) -> instant k, row type r, position j in the row
  __device__ __forceinline__ void locate(int e, int& k, int& r, int& j) {
    k = (int)(((float)e + 0.5f) * invLi);   // exact for block ranges < 2^20
    const int rr = e - k * Li;
    r = 0;
#pragma unroll
    for (int q = 1; q < kGsRowTypes; ++q) r += rr >= S[q] && q < nrt;
    int s = 0, p = 0, t = 0, o = 0;
#pragma unroll
    for (int q = 0; q < kGsRowTypes; ++q)
      if (q == r) { s = S[q]; p = Pl[q]; t = To[q]; o = Po[q]; }
    j = rr - s;
    pl_ = p; to_ = t; po_ = o;
  }
  int pl_, to_, po_;   // the located row's prefix length, template and prefix-code offsets
};

// Streams the block's CSR range [v0, v0 + nv): `entry(k, r, j, ...)` forms the value of position j of
// row type r of the block's instant k; kGsUnits 16-byte units per lane are composed into registers and
// then stored together (as the FDISC stream kernel).
constexpr int kGsUnits = 4;
template <class Entry>
__device__ __forceinline__ void gs_stream_out(double* out, int n, const GsRows& G, const Entry& entry) {
  auto value = [&](int e) -> double {
    int k, r, j;
    GsRows g = G;
    g.locate(e, k, r, j);
    return entry(k, r, j, g.pl_, g.to_, g.po_);
  };
  const int tid = threadIdx.x;
  const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
  if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
  const int m2 = (n - head) >> 1;
  dbl2_t* d2 = reinterpret_cast<dbl2_t*>(out + head);
  for (int u0 = tid; u0 < m2; u0 += kGsBlock * kGsUnits) {
    dbl2_t v[kGsUnits];
#pragma unroll
    for (int q = 0; q < kGsUnits; ++q) {
      const int u = u0 + q * kGsBlock;
      const int e = head + 2 * u;
      v[q].x = u < m2 ? value(e) : 0.0;
      v[q].y = u < m2 ? value(e + 1) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kGsUnits; ++q)
      if (u0 + q * kGsBlock < m2) __builtin_nontemporal_store(v[q], d2 + u0 + q * kGsBlock);
  }
  if (((n - head) & 1) && tid == 0) __builtin_nontemporal_store(value(n - 1), out + n - 1);
}

// LDS of a compose block: [template ints | prefix codes | per-instant doubles | per-instant ints]
__device__ __forceinline__ void gs_stage_tables(const KParams& P, const GsGeo& g, int k0, int n_inst, int32_t* tl, int ntl,
                                                uint8_t* pcl) {
  const int t0 = g.T[0];
  for (int i = threadIdx.x; i < ntl; i += kGsBlock) tl[i] = P.gs_tmpl[t0 + i];
  const int np = n_inst * g.Psum;
  const uint8_t* src = P.gs_pcode + g.pc0 + (int64_t)k0 * g.Psum;
  for (int i = threadIdx.x; i < np; i += kGsBlock) pcl[i] = src[i];
}
__device__ __forceinline__ int gs_tmpl_len(const GsGeo& g) {   // select chain: a runtime index into g puts it in scratch
  int n = 0;
#pragma unroll
  for (int r = 0; r < kGsRowTypes; ++r)
    if (r == g.nrt - 1) n = g.T[r] + g.L[r] - g.P[r] - g.T[0];
  return n;
}

// RangeOfMotion composer. Per instant in LDS: R[9] | HL[4] | Ag[9] | HA[4] | Jx.dx[3] v[3] | sums[3][4]
// (stride kRomC, odd) and cur | qa[3].
constexpr int kRomC = 45;
__global__ void __launch_bounds__(kGsBlock, 1) towr_rom_stream_kernel(KParams P, const double* rec, int64_t ldr, int32_t ni) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);   // a problem's blocks share an XCD
  if (w >= total) return;
  const int b = w / P.ntiles;
  const GsBlock bl = P.gs_blk[w % P.ntiles];
  const GsGeo g = P.gs_geo[bl.geo];
  const int ntl = gs_tmpl_len(g);
  double* cd = smem;
  int32_t* ci = reinterpret_cast<int32_t*>(cd + kRomC * kGsInstRom);
  int32_t* tl = ci + 4 * kGsInstRom;
  uint8_t* pcl = reinterpret_cast<uint8_t*>(tl + ((ntl + 3) & ~3));
  gs_stage_tables(P, g, bl.k0, bl.n_inst, tl, ntl, pcl);
  const int tid = threadIdx.x;
  if (tid < bl.n_inst) {
    const int k = tid;
    const double* r = rec + (int64_t)b * ldr + g.rec0 + bl.k0 + k;
    double* d = cd + k * kRomC;
    for (int f = 0; f < 26; ++f) d[f] = r[(int64_t)f * ni];
    const int poly = (int)r[26 * (int64_t)ni];
    double H[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) H[q] = r[(int64_t)(27 + q) * ni];
#pragma unroll
    for (int f = 0; f < 6; ++f) d[26 + f] = r[(int64_t)(31 + f) * ni];
    ci[4 * k] = (int)r[37 * (int64_t)ni];
    gs_window(P, sp_motion(g.ee), poly, H, d + 32, ci + 4 * k + 1);
  }
  __syncthreads();
  if (!P.want_jac) return;
  GsRows G;
  G.load(g, g.T[0]);
  const int nph = P.sched[g.ee].n_phases;
  auto entry = [&](int k, int r, int j, int pl, int to, int po) -> double {
    const double* d = cd + k * kRomC;
    if (j < pl) {   // base prefix (eval_rom groups 0 and 1)
      const int code = pcl[k * g.Psum + po + j];
      const int e = (code >> 2) & 3, bb = code & 3;
      return (code >> 4) == 0 ? -d[3 * e + r] * d[9 + bb]     // -R[e][r] * HL[b]
                              : d[13 + 3 * e + r] * d[22 + bb];   // Ag[e][r] * HA[b]
    }
    const int32_t t = tl[to + j - pl];
    if (t < 0) {   // R^T d pos / d schedule (:123-130)
      const int col = t & 0xFFFF, cur = ci[4 * k];
      return d[r] * gs_sched_val(d + 26, d + 29, cur, nph, 0, col) + d[3 + r] * gs_sched_val(d + 26, d + 29, cur, nph, 1, col) +
             d[6 + r] * gs_sched_val(d + 26, d + 29, cur, nph, 2, col);
    }
    const int e = (t >> 22) & 3, q = t & 0x3FFFFF;   // motion PhaseCol: R[e][r] * basis sum (emit_dim)
    const unsigned rel = (unsigned)(q - ci[4 * k + 1 + e]);
    return rel < (unsigned)kGsAct ? d[3 * e + r] * d[32 + e * kGsAct + rel] : 0.0;
  };
  gs_stream_out(P.V + (int64_t)b * P.ldv + bl.v0, bl.nv, G, entry);
}

// Dynamic composer. Per instant in LDS, base part (kDynCB doubles): fs[3] | Lp[3] | HpL[4] | HaL[4] |
// M[axis][p v a][r] (27) | HpA HvA HaA (12); per endeffector (kDynCE): Fp[3] | rv[3] | Jf.dx v[6] |
// Jx.dx v[6] | sums[kind][dim][4] (36); ints per endeffector: curF, curX, qa[kind][dim].
constexpr int kDynCB = 53, kDynCE = 54, kDynCI = 11;
TG_HD constexpr int dyn_cstride(int E) { return (kDynCB + kDynCE * E) | 1; }
__global__ void __launch_bounds__(kGsBlock, 1) towr_dyn_stream_kernel(KParams P, const double* rec, int64_t ldr, int32_t K) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= total) return;
  const int b = w / P.ntiles;
  const GsBlock bl = P.gs_blk[w % P.ntiles];
  const GsGeo g = P.gs_geo[bl.geo];
  const int E = P.rb.n_ee, CS = dyn_cstride(E);
  const int ntl = gs_tmpl_len(g);
  double* cd = smem;
  int32_t* ci = reinterpret_cast<int32_t*>(cd + CS * kGsInstDyn);
  int32_t* nph = ci + kDynCI * TOWR_MAX_EE * kGsInstDyn;   // phases of each endeffector
  int32_t* tl = nph + TOWR_MAX_EE;
  uint8_t* pcl = reinterpret_cast<uint8_t*>(tl + ((ntl + 3) & ~3));
  gs_stage_tables(P, g, bl.k0, bl.n_inst, tl, ntl, pcl);
  const int tid = threadIdx.x;
  if (tid < E) nph[tid] = P.sched[tid].n_phases;
  const double* Rb = rec + (int64_t)b * ldr;
  const double* Rax = Rb + (int64_t)kDynBaseRec * K;
  const double* Rh = Rax + (int64_t)3 * kDynAxisRec * K;
  const double* Ree = Rh + (int64_t)kDynHangRec * K;
  const int64_t es = (int64_t)E * K;   // field stride of the endeffector records
  if (tid < bl.n_inst) {   // base lanes: the instant's g rows (dyn_g0_b, the sums in endeffector order) and base part
    const int kk = tid, k = g.rec0 + bl.k0 + kk;
    double* d = cd + kk * CS;
    double Lp[3], ab[3], La[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) { ab[e] = Rb[(int64_t)e * K + k]; La[e] = Rb[(int64_t)(3 + e) * K + k]; Lp[e] = Rb[(int64_t)(6 + e) * K + k]; }
    double fs[3] = {0, 0, 0}, ts[3] = {0, 0, 0};
    for (int ee = 0; ee < E; ++ee) {   // dyn_ee_terms
      const double* r = Ree + ee * K + k;
      double F[3], Tq[3], M[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) { F[e] = r[e * es]; Tq[e] = r[(3 + e) * es]; M[e] = r[(6 + e) * es]; }
      const double rr[3] = {Lp[0] - M[0], Lp[1] - M[1], Lp[2] - M[2]};
      double cr[3]; cross3(F, rr, cr);
#pragma unroll
      for (int e = 0; e < 3; ++e) { ts[e] += cr[e] + Tq[e]; fs[e] += F[e]; }
    }
    if (P.want_g) {
      double* Gb = P.G + (int64_t)b * P.ldg + P.gs_inst[k].row0;
      const double grav[3] = {0.0, 0.0, -P.rb.m * P.rb.g};
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        __builtin_nontemporal_store(ab[e] - ts[e], Gb + AX + e);
        __builtin_nontemporal_store(P.rb.m * La[e] - fs[e] - grav[e], Gb + LX + e);
      }
    }
#pragma unroll
    for (int e = 0; e < 3; ++e) { d[e] = fs[e]; d[3 + e] = Lp[e]; }
#pragma unroll
    for (int q = 0; q < 8; ++q) d[6 + q] = Rb[(int64_t)(9 + q) * K + k];
    for (int f = 0; f < kDynAxisRec; ++f)
#pragma unroll
      for (int e = 0; e < 3; ++e) d[14 + 9 * e + f] = Rax[((int64_t)f * 3 + e) * K + k];
#pragma unroll
    for (int q = 0; q < 12; ++q) d[41 + q] = Rh[(int64_t)q * K + k];
  } else if (tid >= 64 && tid - 64 < bl.n_inst * E) {   // endeffector lanes
    const int x = tid - 64, ee = x / bl.n_inst, kk = x - ee * bl.n_inst, k = g.rec0 + bl.k0 + kk;
    const double* r = Ree + ee * K + k;
    double* d = cd + kk * CS + kDynCB + ee * kDynCE;
    int32_t* ii = ci + (kk * TOWR_MAX_EE + ee) * kDynCI;
    double Lp[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) Lp[e] = Rb[(int64_t)(6 + e) * K + k];
#pragma unroll
    for (int e = 0; e < 3; ++e) { d[e] = r[e * es]; d[3 + e] = Lp[e] - r[(6 + e) * es]; }   // Fp, rv = L.p - P.p (eval_dyn)
#pragma unroll
    for (int f = 0; f < 6; ++f) { d[6 + f] = r[(24 + f) * es]; d[12 + f] = r[(31 + f) * es]; }
    ii[0] = (int)r[30 * es];
    ii[1] = (int)r[37 * es];
#pragma unroll
    for (int kind = 0; kind < 3; ++kind) {   // motion, force, torque
      const int f0 = kind == 0 ? 19 : kind == 1 ? 9 : 14;
      const int s = kind == 0 ? sp_motion(ee) : kind == 1 ? sp_force(ee) : sp_torque(ee);
      double H[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) H[q] = r[(f0 + 1 + q) * es];
      gs_window(P, s, (int)r[f0 * es], H, d + 18 + kind * 3 * kGsAct, ii + 2 + 3 * kind);
    }
  }
  __syncthreads();
  if (!P.want_jac) return;
  GsRows G;
  G.load(g, g.T[0]);
  const double mass = P.rb.m;
  auto entry = [&](int kk, int r, int j, int pl, int to, int po) -> double {
    const double* d = cd + kk * CS;
    if (j < pl) {   // base prefix
      const int code = pcl[kk * g.Psum + po + j];
      const int e = (code >> 2) & 3, bb = code & 3;
      if ((code >> 4) == 0)   // base-linear: -Cross(sum f)[r][e] Hp (dyn_g0_b), m Ha (dyn_g0_a)
        return r < 3 ? -cross_el(d, r, e) * d[6 + bb] : mass * d[10 + bb];
      // base-angular: Ap[r] Hp + Av[r] Hv + Aa[r] Ha of axis e (eval_dyn group 1)
      return d[14 + 9 * e + r] * d[41 + bb] + d[14 + 9 * e + 3 + r] * d[45 + bb] + d[14 + 9 * e + 6 + r] * d[49 + bb];
    }
    const int32_t t = tl[to + j - pl];
    if (t < 0) {   // d/d ee schedule (eval_dyn, dynamic_constraint.cc:116-122)
      const int ee = (t >> 16) & 7, col = t & 0xFFFF;
      const double* de = d + kDynCB + ee * kDynCE;
      const int32_t* ii = ci + (kk * TOWR_MAX_EE + ee) * kDynCI;
      const int n = nph[ee];
      if (r >= 3) return -gs_sched_val(de + 6, de + 9, ii[0], n, r - 3, col);
      const int e1 = r == 2 ? 0 : r + 1, e2 = r == 0 ? 2 : r - 1;
      const double a = cross_el(de + 3, r, e1) * gs_sched_val(de + 6, de + 9, ii[0], n, e1, col) +
                       cross_el(de + 3, r, e2) * gs_sched_val(de + 6, de + 9, ii[0], n, e2, col);
      const double bq = cross_el(de, r, e1) * gs_sched_val(de + 12, de + 15, ii[1], n, e1, col) +
                        cross_el(de, r, e2) * gs_sched_val(de + 12, de + 15, ii[1], n, e2, col);
      return a + bq;
    }
    const int kind = (t >> 28) & 3, ee = (t >> 25) & 7, e = (t >> 22) & 3, q = t & 0x3FFFFF;
    const double* de = d + kDynCB + ee * kDynCE;
    const int32_t* ii = ci + (kk * TOWR_MAX_EE + ee) * kDynCI;
    const unsigned rel = (unsigned)(q - ii[2 + 3 * kind + e]);
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double v = de[18 + (kind * 3 + e) * kGsAct + rel];
    // emit_dim scales: motion Cross(f)[r][e]; force Cross(rv)[r][e] (angular) or -1 (linear); torque -1
    const double sc = kind == 0 ? cross_el(de, r, e) : kind == 1 ? (r < 3 ? cross_el(de + 3, r, e) : -1.0) : -1.0;
    return sc * v;
  };
  gs_stream_out(P.V + (int64_t)b * P.ldv + bl.v0, bl.nv, G, entry);
}

}  // namespace

// LDS (bytes) of the compose kernels, per class: per-instant doubles and ints, the template, prefix codes
size_t gs_stream_lds(const Layout& L, int cls) {
  const int E = L.rb.n_ee;
  size_t d = cls == GS_ROM ? (size_t)kRomC * kGsInstRom : (size_t)dyn_cstride(E) * kGsInstDyn;
  size_t i = cls == GS_ROM ? 4 * (size_t)kGsInstRom : (size_t)kDynCI * TOWR_MAX_EE * kGsInstDyn + TOWR_MAX_EE;
  i += ((size_t)L.gs_tmpl_max[cls] + 3) & ~(size_t)3;
  const size_t pc = (size_t)L.gs_pcode_max[cls] * (cls == GS_ROM ? kGsInstRom : kGsInstDyn);
  return 8 * d + 4 * i + ((pc + 15) & ~(size_t)15);
}
int64_t gs_record_doubles(const Layout& L, int cls) {
  const int64_t K = (int64_t)L.gs_inst[cls].size();
  return cls == GS_ROM ? kRomRec * K : dyn_rec_doubles((int)K, L.rb.n_ee);
}
const void* gs_rec_kernel(int cls, bool rotvec) {
  if (cls == GS_ROM) return rotvec ? reinterpret_cast<const void*>(&towr_rom_rec_kernel<true>) : reinterpret_cast<const void*>(&towr_rom_rec_kernel<false>);
  return rotvec ? reinterpret_cast<const void*>(&towr_dyn_rec_kernel<true>) : reinterpret_cast<const void*>(&towr_dyn_rec_kernel<false>);
}
const void* gs_stream_kernel(int cls) {
  return cls == GS_ROM ? reinterpret_cast<const void*>(&towr_rom_stream_kernel) : reinterpret_cast<const void*>(&towr_dyn_stream_kernel);
}
int gs_rec_block() { return kGsRecBlock; }

}  // namespace tg
