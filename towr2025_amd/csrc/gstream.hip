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

#include <type_traits>

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
__global__ void __launch_bounds__(kGsRecBlock, 2) towr_rom_rec_kernel(KParams P, double* rec, int64_t ldr, int32_t ni, int32_t) {
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

// Dynamic (dynamic_constraint.cc:63-148, single_rigid_body_dynamics.cc:76-204, eval_dyn), in two phases:
//   1. one lane per instant forms the base-angular converter state (dyn_euler_state / dyn_rv_state) into
//      LDS and writes the base record (dyn_g0_a's terms: ab = I_w wd + w x I_w w, the base-linear state and
//      bases); meanwhile one lane per (endeffector, instant) evaluates the force / torque / motion
//      PhaseSplines and their schedule Jacobians;
//   2. after a barrier, one wave per base-angular axis e, one lane per instant, reads the instant's state
//      from LDS and writes that axis's coefficients (dyn_euler_axis / dyn_rv_column<e>): the per-axis
//      chains no longer recompute the shared state, and the state is not held in registers across them.
// The g rows need the endeffector sums and are written by the composer.
template <bool ROTVEC>
struct DynState { using type = typename std::conditional<ROTVEC, DynRvState, DynEulerState>::type; };
template <bool ROTVEC>
size_t dyn_state_bytes() { return sizeof(typename DynState<ROTVEC>::type); }

template <bool ROTVEC>
__global__ void __launch_bounds__(kGsRecBlock, 2) towr_dyn_rec_kernel(KParams P, double* rec, int64_t ldr, int32_t K, int32_t st_off) {
  using State = typename DynState<ROTVEC>::type;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  Ctx c = gait_record_setup<kGsRecBlock>(P, b, smem);
  c.rotvec = ROTVEC;
  State* S = reinterpret_cast<State*>(smem + st_off);   // one per instant, after the staging (gs_rec_lds)
  const int E = P.rb.n_ee, tid = threadIdx.x;
  double* Rb = rec + (int64_t)b * ldr;
  const int EK = E * K;
  // phase 1: instant lanes [0, K) (the first waves), endeffector lanes after them (whole waves)
  const int ee0 = (K + 63) & ~63;
  for (int i = tid; i < ee0 + EK; i += kGsRecBlock) {
    if (i < K) {
      const int k = i;
      const GsInst gi = P.gs_inst[k];
      c.row = gi.seg;
      State& st = S[k];   // formed in place in LDS: the state is never held whole in registers
      if constexpr (ROTVEC) dyn_rv_state(c, gi.t, st);
      else dyn_euler_state(c, gi.t, st);
      SplinePt L;
      spline_eval(c, SP_BASE_LIN, gi.t, L);
      double a[3], bb3[3];   // dyn_g0_a: ab = I_w wd + w x (I_w w)
      mat3_vec(st.Iw, st.wd, a);
      cross3(st.w, st.Iww, bb3);
      double* r = Rb + k;
      auto put = [&](int f, double v) { r[(int64_t)f * K] = v; };
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(e, a[e] + bb3[e]); put(3 + e, L.a[e]); put(6 + e, L.p[e]); }
      double H[4];
      spline_basis(L, kPos, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) put(9 + q, H[q]);
      spline_basis(L, kAcc, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) put(13 + q, H[q]);
      double* h = Rb + (int64_t)(kDynBaseRec + 3 * kDynAxisRec) * K + k;   // the base-angular bases
      spline_basis(st.A, kPos, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) h[(int64_t)q * K] = H[q];
      spline_basis(st.A, kVel, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) h[(int64_t)(4 + q) * K] = H[q];
      spline_basis(st.A, kAcc, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) h[(int64_t)(8 + q) * K] = H[q];
    } else if (i >= ee0) {   // endeffector ee of instant k
      const int idx = i - ee0;
      const int ee = idx / K, k = idx - ee * K;
      const GsInst gi = P.gs_inst[k];
      c.row = gi.seg;
      const double t = gi.t;
      SplinePt F, Tq, M;
      spline_eval(c, sp_force(ee), t, F);
      spline_eval(c, sp_torque(ee), t, Tq);
      spline_eval(c, sp_motion(ee), t, M);
      double* r = Rb + (int64_t)(kDynBaseRec + 3 * kDynAxisRec + kDynHangRec) * K + idx;
      const int64_t st = (int64_t)EK;
      auto put = [&](int f, double v) { r[f * st] = v; };
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(e, F.p[e]); put(3 + e, Tq.p[e]); put(6 + e, M.p[e]); }
      double H[4];
      put(9, (double)F.poly);
      spline_basis(F, kPos, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) put(10 + q, H[q]);
      put(14, (double)Tq.poly);
      spline_basis(Tq, kPos, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) put(15 + q, H[q]);
      put(19, (double)M.poly);
      spline_basis(M, kPos, H);
#pragma unroll
      for (int q = 0; q < 4; ++q) put(20 + q, H[q]);
      SchedJac Jf, Jx;   // force and ee-position terms (dynamic_constraint.cc:116-122; no torque term)
      sched_jac(c, sp_force(ee), t, F, Jf);
      sched_jac(c, sp_motion(ee), t, M, Jx);
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(24 + e, Jf.dx[e]); put(27 + e, Jf.v[e]); put(31 + e, Jx.dx[e]); put(34 + e, Jx.v[e]); }
      put(30, (double)Jf.cur);
      put(37, (double)Jx.cur);
    }
  }
  __syncthreads();
  // phase 2: wave w % 4 takes axis e = w % 4 (< 3) of instants lane, lane + 64, ...
  const int wave = tid >> 6, lane = tid & 63;
  if (wave >= 3) return;
  const int e = wave;
  for (int k = lane; k < K; k += 64) {
    double Ap[3], Av[3], Aa[3];
    if constexpr (ROTVEC) {
      if (e == 0) dyn_rv_column<0>(S[k], Ap, Av, Aa);
      else if (e == 1) dyn_rv_column<1>(S[k], Ap, Av, Aa);
      else dyn_rv_column<2>(S[k], Ap, Av, Aa);
    } else {
      dyn_euler_axis(c, S[k], e, Ap, Av, Aa);
    }
    double* r = Rb + (int64_t)kDynBaseRec * K + e * K + k;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      r[(int64_t)(q) * 3 * K] = Ap[q];
      r[(int64_t)(3 + q) * 3 * K] = Av[q];
      r[(int64_t)(6 + q) * 3 * K] = Aa[q];
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

// Per-class pieces of the composer (towr_gs_stream_kernel):
//   CS / CI: doubles and ints of one instant's record in LDS; load(): a prologue lane fills them;
//   poly(): the active polynomial of a PhaseSpline segment's spline at the instant;
//   value(): value q of a segment at the instant (the tile path's expression for that entry).
// RangeOfMotion: doubles R[9] | HL[4] | Ag[9] | HA[4] | Jx.dx[3] v[3] | sums[3][4]; ints cur | qa[3] | poly.
struct RomCls {
  static constexpr int kCS = 45, kCI = 5;
  static constexpr int kLoadLanes = 1;   // prologue lanes per instant
  __device__ static int stride_d(int) { return kCS; }
  __device__ static int stride_i(int) { return kCI; }
  __device__ static void load(const KParams& P, const GsGeo& g, const double* rec, int ni, int k, int lane, double* d, int32_t* ci, double*) {
    const double* r = rec + k;
    for (int f = 0; f < 26; ++f) d[f] = r[(int64_t)f * ni];
    const int poly = (int)r[26 * (int64_t)ni];
    double H[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) H[q] = r[(int64_t)(27 + q) * ni];
#pragma unroll
    for (int f = 0; f < 6; ++f) d[26 + f] = r[(int64_t)(31 + f) * ni];
    ci[0] = (int)r[37 * (int64_t)ni];
    ci[4] = poly;
    gs_window(P, sp_motion(g.ee), poly, H, d + 32, ci + 1);
  }
  __device__ static int poly(const int32_t* ci, int, int) { return ci[4]; }
  __device__ static double value(const KParams& P, const int32_t* tmpl, const GsSeg& sg, int pos, const double* d, const int32_t* ci,
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

// Dynamic: doubles, base part fs[3] | Lp[3] | HpL[4] | HaL[4] | M[axis][p v a][r] (27) | HpA HvA HaA (12),
// then per endeffector Fp[3] | rv[3] | Jf.dx v[6] | Jx.dx v[6] | sums[kind][dim][4] (36);
// ints per endeffector curF, curX, qa[kind][dim], poly[kind]. The first prologue lane of an instant
// also writes its 6 g rows (dyn_g0_b: the endeffector sums in order).
struct DynCls {
  static constexpr int kCB = 53, kCE = 54, kCIE = 14;
  static constexpr int kLoadLanes = 1 + TOWR_MAX_EE;
  __device__ static int stride_d(int E) { return (kCB + kCE * E) | 1; }
  __device__ static int stride_i(int E) { return kCIE * E; }
  __device__ static void load(const KParams& P, const GsGeo& g, const double* Rb, int K, int k, int lane, double* d, int32_t* ci, double* Gp) {
    const int E = P.rb.n_ee;
    const double* Rax = Rb + (int64_t)kDynBaseRec * K;
    const double* Rh = Rax + (int64_t)3 * kDynAxisRec * K;
    const double* Ree = Rh + (int64_t)kDynHangRec * K;
    const int64_t es = (int64_t)E * K;   // field stride of the endeffector records
    if (lane == 0) {   // base part and the instant's g rows
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
        double* Gb = Gp + P.gs_inst[k].row0;
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
      return;
    }
    const int ee = lane - 1;
    if (ee >= E) return;
    const double* r = Ree + ee * K + k;
    double* de = d + kCB + ee * kCE;
    int32_t* ii = ci + ee * kCIE;
#pragma unroll
    for (int e = 0; e < 3; ++e) de[e] = r[e * es];
#pragma unroll
    for (int e = 0; e < 3; ++e) de[3 + e] = Rb[(int64_t)(6 + e) * K + k] - r[(6 + e) * es];   // rv = L.p - P.p (eval_dyn)
#pragma unroll
    for (int f = 0; f < 6; ++f) { de[6 + f] = r[(24 + f) * es]; de[12 + f] = r[(31 + f) * es]; }
    ii[0] = (int)r[30 * es];
    ii[1] = (int)r[37 * es];
#pragma unroll
    for (int kind = 0; kind < 3; ++kind) {   // motion, force, torque
      const int f0 = kind == 0 ? 19 : kind == 1 ? 9 : 14;
      const int s = kind == 0 ? sp_motion(ee) : kind == 1 ? sp_force(ee) : sp_torque(ee);
      double H[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) H[q] = r[(f0 + 1 + q) * es];
      const int poly = (int)r[f0 * es];
      ii[11 + kind] = poly;
      gs_window(P, s, poly, H, de + 18 + kind * 3 * kGsAct, ii + 2 + 3 * kind);
    }
  }
  __device__ static int poly(const int32_t* ci, int kind, int ee) { return ci[ee * kCIE + 11 + kind]; }
  __device__ static double value(const KParams& P, const int32_t* tmpl, const GsSeg& sg, int pos, const double* d, const int32_t* ci,
                                 const uint8_t* pcl, const int32_t* nph) {
    const int r = sg.r;
    if (sg.type == 0) {   // base prefix
      const int code = pcl[sg.toff + pos];
      const int e = (code >> 2) & 3, bb = code & 3;
      if ((code >> 4) == 0)   // base-linear: -Cross(sum f)[r][e] Hp (dyn_g0_b), m Ha (dyn_g0_a)
        return r < 3 ? -cross_el(d, r, e) * d[6 + bb] : P.rb.m * d[10 + bb];
      // base-angular: Ap[r] Hp + Av[r] Hv + Aa[r] Ha of axis e (eval_dyn group 1)
      return d[14 + 9 * e + r] * d[41 + bb] + d[14 + 9 * e + 3 + r] * d[45 + bb] + d[14 + 9 * e + 6 + r] * d[49 + bb];
    }
    const int32_t t = tmpl[sg.toff + pos];
    const int ee = sg.ee;
    const double* de = d + kCB + ee * kCE;
    const int32_t* ii = ci + ee * kCIE;
    if (sg.type == 2) {   // d/d ee schedule (eval_dyn, dynamic_constraint.cc:116-122)
      const int col = t & 0xFFFF, n = nph[ee];
      if (r >= 3) return -gs_sched_val(de + 6, de + 9, ii[0], n, r - 3, col);
      const int e1 = r == 2 ? 0 : r + 1, e2 = r == 0 ? 2 : r - 1;
      const double a = cross_el(de + 3, r, e1) * gs_sched_val(de + 6, de + 9, ii[0], n, e1, col) +
                       cross_el(de + 3, r, e2) * gs_sched_val(de + 6, de + 9, ii[0], n, e2, col);
      const double bq = cross_el(de, r, e1) * gs_sched_val(de + 12, de + 15, ii[1], n, e1, col) +
                        cross_el(de, r, e2) * gs_sched_val(de + 12, de + 15, ii[1], n, e2, col);
      return a + bq;
    }
    const int kind = sg.kind, e = (t >> 22) & 3, q = t & 0x3FFFFF;
    const unsigned rel = (unsigned)(q - ii[2 + 3 * kind + e]);
    if (rel >= (unsigned)kGsAct) return 0.0;
    const double v = de[18 + (kind * 3 + e) * kGsAct + rel];
    // emit_dim scales: motion Cross(f)[r][e]; force Cross(rv)[r][e] (angular) or -1 (linear); torque -1
    const double sc = kind == 0 ? cross_el(de, r, e) : kind == 1 ? (r < 3 ? cross_el(de + 3, r, e) : -1.0) : -1.0;
    return sc * v;
  }
};

// The composer: one block per (problem, GsBlock).
//   1. the block's prefix codes and the geometry's position -> segment map to LDS;
//   2. prologue lanes load their instant's record (CLS::load);
//   3. per (instant, segment): the window start in the instant and the segment's value base (wp);
//   4. per (instant, value): the value (CLS::value), one lane each;
//   5. the CSR range [v0, v0 + nv) streams out, kGsUnits 16-byte units composed per lane before their
//      stores, every entry one lookup: its segment, the window, the value or 0.
// LDS: [the geometry's blob (segments, value map, template, position -> segment, prefix codes, window
// starts; layout.h gs_blob) | values | records (doubles) | wp (int2) | record ints | nph].
constexpr int kGsUnits = 4;
template <int CLS>
__global__ void __launch_bounds__(kGsBlock, 1) towr_gs_stream_kernel(KParams P, const double* rec, int64_t ldr, int32_t ni) {
  using C = typename std::conditional<CLS == GS_ROM, RomCls, DynCls>::type;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);   // a problem's blocks share an XCD
  if (w >= total) return;
  const int b = w / P.ntiles;
  const GsBlock bl = P.gs_blk[w % P.ntiles];
  const GsGeo g = P.gs_geo[bl.geo];
  const int E = P.rb.n_ee, n = bl.n_inst, tid = threadIdx.x;
  const int CS = C::stride_d(E), CI = C::stride_i(E), vt = g.vt, ns = g.ns;
  // LDS: [blob | values | records (doubles) | wp (int2) | record ints | nph]
  char* blob = reinterpret_cast<char*>(smem);
  double* val = smem + 2 * g.blob_n16;
  double* cd = val + ((n * vt + 1) & ~1);
  int2* wp = reinterpret_cast<int2*>(cd + ((n * CS + 1) & ~1));
  int32_t* ci = reinterpret_cast<int32_t*>(wp + n * ns);
  int32_t* nph = ci + n * CI;
  stage16<kGsBlock>(reinterpret_cast<uint4*>(blob), P.gs_blob + g.blob0, g.blob_n16);
  if (tid < E) nph[tid] = P.sched[tid].n_phases;
  const GsSeg* segs = reinterpret_cast<const GsSeg*>(blob);
  const uint32_t* vmap = reinterpret_cast<const uint32_t*>(blob + g.o_vmap);
  const int32_t* tmpl = reinterpret_cast<const int32_t*>(blob + g.o_tmpl);
  const uint8_t* tsg = reinterpret_cast<const uint8_t*>(blob + g.o_tseg);
  const uint8_t* pcl = reinterpret_cast<const uint8_t*>(blob + g.o_pcode) + bl.k0 * g.Psum;
  const int16_t* wsl = reinterpret_cast<const int16_t*>(blob + g.o_ws);
  const double* Rb = rec + (int64_t)b * ldr;
  if (tid < n * C::kLoadLanes) {
    const int kk = tid % n, lane = tid / n;
    C::load(P, g, CLS == GS_ROM ? Rb + g.rec0 : Rb, ni, (CLS == GS_ROM ? 0 : g.rec0) + bl.k0 + kk, lane, cd + kk * CS, ci + kk * CI,
            P.G + (int64_t)b * P.ldg);
  }
  __syncthreads();
  for (int t = tid; t < n * ns; t += kGsBlock) {   // window starts and value bases
    const int kk = t / ns, sid = t - kk * ns;
    const GsSeg sg = segs[sid];
    int ws = 0;
    if (sg.type == 1) ws = wsl[sg.wsoff + C::poly(ci + kk * CI, sg.kind, sg.ee)];
    wp[t] = make_int2(sg.p0 + ws, ((int)sg.W << 16) | (kk * vt + sg.vbase));
  }
  __syncthreads();
  for (int t = tid; t < n * vt; t += kGsBlock) {   // every value of every instant, once
    const int kk = t / vt, v = t - kk * vt;
    const uint32_t vm = vmap[v];
    const int sid = (int)(vm >> 16), q = (int)(vm & 0xFFFF);
    const GsSeg sg = segs[sid];
    const int pos = wp[kk * ns + sid].x + q;   // position in the instant
    double x = 0.0;
    if (pos < sg.p0 + sg.len) {
      if constexpr (CLS == GS_ROM) x = C::value(P, tmpl, sg, pos, cd + kk * CS, ci + kk * CI, pcl + kk * g.Psum, nph[g.ee]);
      else x = C::value(P, tmpl, sg, pos, cd + kk * CS, ci + kk * CI, pcl + kk * g.Psum, nph);
    }
    val[t] = x;
  }
  __syncthreads();
  if (!P.want_jac) return;
  const int Li = g.Li;
  const float invLi = 1.0f / (float)Li;
  auto value = [&](int e) -> double {
    const int kk = (int)(((float)e + 0.5f) * invLi);   // exact for block ranges < 2^20
    const int rr = e - kk * Li;
    const int2 p = wp[kk * ns + tsg[rr]];
    const unsigned q = (unsigned)(rr - p.x);
    return q < (unsigned)(p.y >> 16) ? val[(p.y & 0xFFFF) + q] : 0.0;
  };
  double* out = P.V + (int64_t)b * P.ldv + bl.v0;
  const int nv = bl.nv;
  const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
  if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
  const int m2 = (nv - head) >> 1;
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
  if (((nv - head) & 1) && tid == 0) __builtin_nontemporal_store(value(nv - 1), out + nv - 1);
}

}  // namespace

// LDS (bytes) of the composer of class cls: sized for the class's largest geometry (GsGeo)
size_t gs_stream_lds(const Layout& L, int cls) {
  const int E = L.rb.n_ee;
  const size_t n = (size_t)L.gs_nmax[cls];
  const size_t ns = (size_t)L.gs_geo_max[cls][1], vt = (size_t)L.gs_geo_max[cls][2], blob = (size_t)L.gs_geo_max[cls][3];
  const size_t CS = cls == GS_ROM ? RomCls::kCS : (size_t)((DynCls::kCB + DynCls::kCE * E) | 1);
  const size_t CI = cls == GS_ROM ? RomCls::kCI : (size_t)DynCls::kCIE * E;
  size_t b = blob + 8 * (((n * vt + 1) & ~(size_t)1) + ((n * CS + 1) & ~(size_t)1));
  b += 8 * n * ns + 4 * (n * CI + TOWR_MAX_EE);
  return (b + 15) & ~(size_t)15;
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
  return cls == GS_ROM ? reinterpret_cast<const void*>(&towr_gs_stream_kernel<GS_ROM>) : reinterpret_cast<const void*>(&towr_gs_stream_kernel<GS_DYN>);
}
int gs_rec_block() { return kGsRecBlock; }
size_t gs_dyn_state_bytes(bool rotvec) { return rotvec ? dyn_state_bytes<true>() : dyn_state_bytes<false>(); }

}  // namespace tg
