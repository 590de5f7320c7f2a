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
//   compose: one block per (problem group, GsBlock) reads its instants' records, forms each value of
//            an instant once, then streams its whole CSR range with 16-byte non-temporal stores, each
//            unit written once, zeros included. The ForceConstraintDiscretized compose blocks
//            (their records: fdisc_records) run in the same launch (towr_gait_compose_kernel).
// Every entry is the tile path's own expression (eval_rom / eval_dyn, cited per case), so parity is
// the tile path's parity.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"
#include "gs_cls.h"
#include "tile_emit.h"

namespace tg {
namespace {


// ------------------------------------------------------------------------------------------------
// ForceConstraintDiscretized records (layout.h FsBlock, kFsRS). Every Jacobian row of the class is the
// force set's full PhaseSpline pattern plus the schedule columns, ~90 % exact zeros whose positions move
// with x. One lane per instant: fdisc_instant's result in the composer's form — the basis sums of the
// kFsWin columns the force polynomial can touch (phase_basis_sum over the instant's window of the
// template), the 5 pyramid rows b, d force / d schedule, the window start and dimension codes — goes to
// the per-problem record array; the instant's g rows go straight out. Records are chunk-major per
// FsBlock (field f of the block's instant kk at kFsRS t0 + f n + kk), so a compose block's prologue is
// one contiguous copy.
// ------------------------------------------------------------------------------------------------
// FDISC instant k (fs_t order) of the problem in c: its record fields through put(field, value) and its 5 g
// rows (when wanted) straight to Gb
// the FDISC tables a record lane reads after its instant: in LDS (staged by towr_gait_frec_kernel) or global memory
struct FsTabs { const FsBlock* fsb; const int32_t* ws; const int32_t* tmpl; };
template <class Put>
__device__ __forceinline__ void fdisc_record(const KParams& P, const FsTabs& T, const Ctx& c, int k, double* Gb, Put&& put) {
  // every global load of the lane before its first store: a load issued after stores waits for them (vmcnt)
  const int row = P.want_g ? P.fs_irow[k] : 0;
  const FsBlock fb = T.fsb[P.fs_iblk[k]];
  FdiscInstant o;
  fdisc_instant(c, P.fs_iee[k], P.fs_t[k], o);
  TG_STAMP(P, 4);
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int e = 0; e < 3; ++e) put(kFsB + 3 * i + e, o.b[i][e]);
#pragma unroll
  for (int e = 0; e < 3; ++e) { put(kFsDx + e, o.Jf.dx[e]); put(kFsV + e, o.Jf.v[e]); }
  if (P.want_g)
#pragma unroll
    for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(o.g[i], Gb + row + i);
  TG_STAMP(P, 5);
  const int poly = o.poly;
  const int ws = T.ws[3 * (fb.wsoff + poly)], wd = T.ws[3 * (fb.wsoff + poly) + 1], wq = T.ws[3 * (fb.wsoff + poly) + 2];
  put(kFsND, gs_int2(ws, wd));
  put(kFsND + 1, gs_int2(o.Jf.cur, wq));
  double h0 = o.H[0], h1 = o.H[1], h2 = o.H[2], h3 = o.H[3];
  asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
  const SplineMeta m = c.spl[sp_force(P.fs_iee[k])];
  const int32_t* aw = c.pact + m.pact_off + 2 * poly;   // dimension 0's active window
  const int a = aw[0], z = aw[1];
#pragma unroll
  for (int q = 0; q < kFsS; ++q)   // the active window's basis sums (one set: the dimensions coincide)
    put(q, a + q <= z ? phase_basis_sum(c.pcols[m.pcol_off[0] + a + q], poly, h0, h1, h2, h3) : 0.0);
  TG_STAMP(P, 6);
}
__device__ __forceinline__ void fdisc_records(const KParams& P, const FsTabs& T, const Ctx& c, int b, double* rec, int64_t ldr, int32_t k0,
                                              int32_t k1) {
  double* Gb = P.G + (int64_t)b * P.ldg;
  double* R = rec + (int64_t)b * ldr;
  for (int k = k0 + threadIdx.x; k < k1; k += blockDim.x) {
    const FsBlock fb = T.fsb[P.fs_iblk[k]];
    const int kk = k - fb.t0, nb = fb.n_inst;
    double* r = R + (int64_t)kFsRS * fb.t0 + kk;
    fdisc_record(P, T, c, k, Gb, [&](int f, double v) { r[f * nb] = v; });
  }
}

// field f of class-global instant k of a record (layout.h: chunk-major, field-major in the chunk)
__device__ __forceinline__ double* gs_field(double* R, int RS, int k, const GsInst& gi, int f) {
  return R + (int64_t)RS * (k - gi.kk) + f * gi.nb + gi.kk;
}

// ------------------------------------------------------------------------------------------------
// TorqueConstraintDiscretized records (layout.h record format, GS_TQ). Every row of the class is the torque
// set's full PhaseSpline pattern (rows 2, 3 also the force set's) plus the schedule columns; on a terrain
// without curvature the motion block is skipped (every scale is exactly 0.0,
// torque_constraint_discretized.cc:57). One lane per instant: eval_tqdisc's quantities in the composer's
// form — the terrain basis t1, t2, n, the force row scale b = -k mu n, d torque / d schedule and d force /
// d schedule, the active-window basis sums of the torque and force polynomials — go to the record; the 4
// g rows go straight out (:101-125).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void tq_records(const KParams& P, const RecArgs& A, Ctx c, int b) {
  constexpr int RS = kTqND + kTqNI;
  const int K = A.g.K[GS_TQ];
  const GsInst* inst = A.g.inst[GS_TQ];
  double* Gb = P.G + (int64_t)b * P.ldg;
  double* R = A.frec + (int64_t)b * A.fldr + A.tq_off;
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    const GsInst gi = inst[k];
    c.row = gi.seg;
    double g[4];
    tq_record(c, gi, [&](int f, double v) { *gs_field(R, RS, k, gi, f) = v; }, g);
    if (P.want_g)
#pragma unroll
      for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(g[i], Gb + gi.row0 + i);
  }
}

// ------------------------------------------------------------------------------------------------
// RangeOfMotion / Dynamic records
// ------------------------------------------------------------------------------------------------
// One block per problem records both classes (layout.h, record format): the staging of x and the
// PhaseSpline tables (gait_record_setup) is done once for RangeOfMotion and Dynamic. Lanes, whole
// waves per kind:
//   [0, Kd)                  Dynamic instant k: the base-angular converter state (dyn_euler_state /
//                            dyn_rv_state) into LDS; the base-linear and base-angular bases; ab, La, Lp
//                            to the scratch;
//   [ee0, ee0 + 3 E Kd)      Dynamic (spline kind, endeffector, instant): the motion / force / torque
//                            PhaseSpline, its active-window sums and schedule Jacobian; F, Tq, M to the
//                            scratch (one chain per lane: the three splines no longer run in series);
//   [r0, r0 + Kr)            RangeOfMotion instant (range_of_motion_constraint.cc:72-131, eval_rom); its
//                            3 g rows go straight out;
// then, after a barrier, per Dynamic instant: one lane per base-angular axis e reads the state and writes
// that axis's coefficients (dyn_euler_axis / dyn_rv_column<e>), one lane forms the endeffector sums
// (fs, rv = Lp - M per endeffector) and the instant's 6 g rows (dyn_g0_b: the endeffectors in order).
template <bool ROTVEC>
struct DynState { using type = typename std::conditional<ROTVEC, DynRvState, DynEulerState>::type; };
template <bool ROTVEC>
size_t dyn_state_bytes() { return sizeof(typename DynState<ROTVEC>::type); }


template <bool ROTVEC>
// part: 0 every lane, 1 the Dynamic lanes only, 2 the RangeOfMotion lanes only (a small batch spreads the
// role over two blocks)
__device__ __forceinline__ void gs_records(const KParams& P, const GsRecArgs& A, Ctx c, int b, double* smem, int part = 0) {
  using State = typename DynState<ROTVEC>::type;
  c.rotvec = ROTVEC;
  State* S = reinterpret_cast<State*>(smem + A.st_off);   // one per Dynamic instant
  double* scr = smem + A.scr_off;
  const int E = P.rb.n_ee, tid = threadIdx.x, nthr = blockDim.x;
  const int Kd = A.K[GS_DYN], Kr = A.K[GS_ROM], EK = E * Kd;
  double* Rr = A.rec + (int64_t)b * A.ldr;
  double* Rd = Rr + A.dyn_off;
  double* Gb = P.G + (int64_t)b * P.ldg;
  const int RSr = gs_rec_fields(GS_ROM, E), RSd = gs_rec_fields(GS_DYN, E), NDd = gs_rec_nd(GS_DYN, E);
  const int ee0 = (Kd + 63) & ~63, r0 = (ee0 + 3 * EK + 63) & ~63;
  for (int i = (part == 2 ? r0 : 0) + tid; i < (part == 1 ? r0 : r0 + Kr); i += nthr) {
    if (i < Kd) {   // Dynamic instant
      const int k = i;
      const GsInst gi = A.inst[GS_DYN][k];
      c.row = gi.seg;
      State& st = S[k];   // formed in place in LDS: the state is never held whole in registers
      if constexpr (ROTVEC) dyn_rv_state(c, gi.t, st);
      else dyn_euler_state(c, gi.t, st);
      SplinePt L;
      spline_eval(c, SP_BASE_LIN, gi.t, L);
      // the five bases (segment-table loads) before the lane's first record store: a load issued after stores waits
      // for them (vmcnt counts stores)
      double HLp[4], HLa[4], HAp[4], HAv[4], HAa[4];
      spline_basis(L, kPos, HLp);
      spline_basis(L, kAcc, HLa);
      spline_basis(st.A, kPos, HAp);
      spline_basis(st.A, kVel, HAv);
      spline_basis(st.A, kAcc, HAa);
      double a[3], bb3[3];   // dyn_g0_a: ab = I_w wd + w x (I_w w)
      mat3_vec(st.Iw, st.wd, a);
      cross3(st.w, st.Iww, bb3);
      double* sk = scr + 9 * k;
#pragma unroll
      for (int e = 0; e < 3; ++e) { sk[e] = a[e] + bb3[e]; sk[3 + e] = L.a[e]; sk[6 + e] = L.p[e]; }
      auto put = [&](int f, double v) { *gs_field(Rd, RSd, k, gi, f) = v; };
#pragma unroll
      for (int e = 0; e < 3; ++e) put(3 + e, L.p[e]);
#pragma unroll
      for (int q = 0; q < 4; ++q) { put(6 + q, HLp[q]); put(10 + q, HLa[q]); put(41 + q, HAp[q]); put(45 + q, HAv[q]); put(49 + q, HAa[q]); }
    } else if (i >= ee0 && i < ee0 + 3 * EK) {   // Dynamic (spline kind, endeffector ee, instant k)
      const int idx = i - ee0;
      const int kind = idx / EK, rem = idx - kind * EK;   // kind 0 motion, 1 force, 2 torque
      const int ee = rem / Kd, k = rem - ee * Kd;
      const GsInst gi = A.inst[GS_DYN][k];
      c.row = gi.seg;
      const double t = gi.t;
      const int sp = kind == 0 ? sp_motion(ee) : kind == 1 ? sp_force(ee) : sp_torque(ee);
      SplinePt Sp;
      spline_eval(c, sp, t, Sp);
      double* sk = scr + 9 * Kd + 9 * rem + (kind == 0 ? 6 : kind == 1 ? 0 : 3);   // F | Tq | M
#pragma unroll
      for (int e = 0; e < 3; ++e) sk[e] = Sp.p[e];
      const int fd = kDynBaseND + kDynEeND * ee, fi = NDd + kDynEeNI * ee;
      auto put = [&](int f, double v) { *gs_field(Rd, RSd, k, gi, f) = v; };
      int qa[3];
      {   // the active window's basis sums
        double H[4], sums[3][kGsAct];
        spline_basis(Sp, kPos, H);
        gs_window(c, sp, Sp.poly, H, sums, qa);
#pragma unroll
        for (int e = 0; e < 3; ++e)
          if (kind == 0 || e == 0)   // force and torque: one set for the three dimensions (layout.h)
#pragma unroll
            for (int q = 0; q < kGsAct; ++q) put(fd + dyn_sum_field(kind, e, q), sums[e][q]);
      }
      // the lane's ints (layout.h: curX | qaX[3] | polyX | - | curF | qaF | polyF | - | qaT | polyT)
      if (kind < 2) {   // force and ee-position schedule terms (dynamic_constraint.cc:116-122; no torque term)
        SchedJac J;
        sched_jac(c, sp, t, Sp, J);
        const int o = kind == 1 ? 6 : 12;
#pragma unroll
        for (int e = 0; e < 3; ++e) { put(fd + o + e, J.dx[e]); put(fd + o + 3 + e, J.v[e]); }
        if (kind == 1) {
#pragma unroll
          for (int e = 0; e < 3; ++e) put(fd + e, Sp.p[e]);
          put(fi + 3, gs_int2(J.cur, qa[0]));
          put(fi + 4, gs_int2(Sp.poly, 0));
        } else {
          put(fi, gs_int2(J.cur, qa[0]));
          put(fi + 1, gs_int2(qa[1], qa[2]));
          put(fi + 2, gs_int2(Sp.poly, 0));
        }
      } else {
        put(fi + 5, gs_int2(qa[0], Sp.poly));
      }
    } else if (i >= r0) {   // RangeOfMotion instant
      const int k = i - r0;
      const GsInst gi = A.inst[GS_ROM][k];
      c.row = gi.seg;
      const double t = gi.t;
      SplinePt L, Ab, M;
      spline_eval(c, SP_BASE_LIN, t, L);
      spline_eval(c, SP_BASE_ANG, t, Ab);
      spline_eval(c, sp_motion(gi.ee), t, M);
      double HL[4], HA[4];   // (segment-table loads before the lane's first store, as the Dynamic lanes)
      spline_basis(L, kPos, HL);
      spline_basis(Ab, kPos, HA);
      double R[3][3];
      Trig q{};
      if constexpr (ROTVEC) rv_rodrigues(Ab.p, R);
      else { q = trig(Ab.p); euler_R(q, R); }
      const double rW[3] = {M.p[0] - L.p[0], M.p[1] - L.p[1], M.p[2] - L.p[2]};
      if (P.want_g)
        for (int j = 0; j < 3; ++j) __builtin_nontemporal_store(R[0][j] * rW[0] + R[1][j] * rW[1] + R[2][j] * rW[2], Gb + gi.row0 + j);
      auto put = [&](int f, double v) { *gs_field(Rr, RSr, k, gi, f) = v; };
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int l = 0; l < 3; ++l) put(3 * j + l, R[j][l]);
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) put(9 + bb, HL[bb]);
      // base-angular coefficients Ag[e][r]: the entry at (axis e, basis b) of row r is Ag[e][r] HA[b]
      if constexpr (ROTVEC) {   // DerivOfRotVecMult(t, r_W, inverse = true): R^T [r_W]x J_L
        double JL[3][3], Am[3][3];
        rv_left_jac(Ab.p, JL);
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
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) put(22 + bb, HA[bb]);
      double H[4];
      spline_basis(M, kPos, H);
      int qa[3];
      {
        double sums[3][kGsAct];
        gs_window(c, sp_motion(gi.ee), M.poly, H, sums, qa);
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
          for (int qq = 0; qq < kGsAct; ++qq) put(32 + e * kGsAct + qq, sums[e][qq]);
      }
      SchedJac Jx;
      sched_jac(c, sp_motion(gi.ee), t, M, Jx);   // b_R_w * d pos / d schedule (:123-130)
#pragma unroll
      for (int e = 0; e < 3; ++e) { put(26 + e, Jx.dx[e]); put(29 + e, Jx.v[e]); }
      put(kRomND, gs_int2(Jx.cur, qa[0]));   // ints cur | qa[3] | poly
      put(kRomND + 1, gs_int2(qa[1], qa[2]));
      put(kRomND + 2, gs_int2(M.poly, 0));
    }
  }
  if (Kd == 0 || part == 2) return;
  __syncthreads();
  // phase 2: part 0-2 = base-angular axis e, part 3 = the endeffector sums and g rows; whole waves per part
  const int Kp = (Kd + 63) & ~63;
  for (int i = tid; i < 4 * Kp; i += nthr) {
    const int part = i / Kp, k = i - part * Kp;
    if (k >= Kd) continue;
    const GsInst gi = A.inst[GS_DYN][k];
    auto put = [&](int f, double v) { *gs_field(Rd, RSd, k, gi, f) = v; };
    if (part < 3) {
      const int e = part;
      double Ap[3], Av[3], Aa[3];
      if constexpr (ROTVEC) {
        if (e == 0) dyn_rv_column<0>(S[k], Ap, Av, Aa);
        else if (e == 1) dyn_rv_column<1>(S[k], Ap, Av, Aa);
        else dyn_rv_column<2>(S[k], Ap, Av, Aa);
      } else {
        dyn_euler_axis(c, S[k], e, Ap, Av, Aa);
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) { put(14 + 9 * e + r, Ap[r]); put(17 + 9 * e + r, Av[r]); put(20 + 9 * e + r, Aa[r]); }
      continue;
    }
    const double* sk = scr + 9 * k;   // dyn_ee_terms, endeffectors in order
    double fs[3] = {0, 0, 0}, ts[3] = {0, 0, 0};
    for (int ee = 0; ee < E; ++ee) {
      const double* se = scr + 9 * Kd + 9 * (ee * Kd + k);
      const double F[3] = {se[0], se[1], se[2]}, Tq[3] = {se[3], se[4], se[5]};
      const double rr[3] = {sk[6] - se[6], sk[7] - se[7], sk[8] - se[8]};
      double cr[3]; cross3(F, rr, cr);
#pragma unroll
      for (int e = 0; e < 3; ++e) { ts[e] += cr[e] + Tq[e]; fs[e] += F[e]; put(kDynBaseND + kDynEeND * ee + 3 + e, rr[e]); }
    }
#pragma unroll
    for (int e = 0; e < 3; ++e) put(e, fs[e]);
    if (P.want_g) {
      double* G = Gb + gi.row0;
      const double grav[3] = {0.0, 0.0, -P.rb.m * P.rb.g};
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        __builtin_nontemporal_store(sk[e] - ts[e], G + AX + e);
        __builtin_nontemporal_store(P.rb.m * sk[3 + e] - fs[e] - grav[e], G + LX + e);
      }
    }
  }
}

// The record launch: per problem RecArgs::nparts blocks, block r doing part (parts >> 4 r) & 15
// (layout.h RecPart): the FDISC records, the TorqueConstraintDiscretized records, or the RangeOfMotion /
// Dynamic records (all lanes, or one class's lanes when a small batch spreads them over two blocks), each
// block staging x and the PhaseSpline tables itself (gait_record_setup). towr_gpu.hip launch_stream_path
// chooses the parts: at large batch sizes one launch per chain, at small ones (B = 1) every part in one.
// Instantiated per role set (ROLES bit 0 the FDISC part, bit 1 the RangeOfMotion / Dynamic parts, bit 2 the
// TQDISC part), so a launch carries only its parts' registers: the FDISC records alone 110 VGPRs (4 waves per
// SIMD), with the TQDISC code 170 (2 waves per SIMD; ANYmal gait, B = 1024: FDISC 0.389 -> 0.419 ms). With the RangeOfMotion / Dynamic role: 4 waves per SIMD
// (128 VGPRs, a few spilled): at the unconstrained 166 VGPRs a second 5-wave block did not fit a CU (MI355X,
// ANYmal gait B = 1024: 122 us, 100 us at 4 waves per SIMD)
template <bool ROTVEC, int ROLES>
__device__ __forceinline__ void rec_body(const KParams& P, const RecArgs& A, double* smem) {
  const int np = A.nparts;
  const int b = (int)blockIdx.x / np, part = (A.parts >> (4 * ((int)blockIdx.x % np))) & 15;
  int32_t* d = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(smem) + A.fs_lds);
  if constexpr ((ROLES & 1) != 0) {
    if (A.fs_lds > 0) {   // the FDISC tables to LDS beside the staging (gait_record_setup's barrier covers them)
      const int32_t* sb = reinterpret_cast<const int32_t*>(P.fsb);
      for (int i = threadIdx.x; i < A.fs_nb + A.fs_nws + A.fs_ntm; i += blockDim.x)
        d[i] = i < A.fs_nb ? sb[i] : i < A.fs_nb + A.fs_nws ? P.fs_ws[i - A.fs_nb] : P.fs_tmpl[i - A.fs_nb - A.fs_nws];
    }
  }
  const Ctx c = gait_record_setup<0>(P, b, smem);
  if constexpr ((ROLES & 1) != 0)
    if (part == kRecFdisc) {
      // two instances, so that every table pointer has one address space: a pointer that may be LDS or global is a
      // flat one, and a flat load waits for the lane's earlier record stores too (vmcnt counts stores): the 12 window
      // loads after the record stores then took ~6 of a ~24 us record block (MI355X, ANYmal gait, tools/stamps.py)
      if (A.fs_lds > 0) fdisc_records(P, FsTabs{reinterpret_cast<const FsBlock*>(d), d + A.fs_nb, d + A.fs_nb + A.fs_nws}, c, b, A.frec, A.fldr, 0, A.ni);
      else fdisc_records(P, FsTabs{P.fsb, P.fs_ws, P.fs_tmpl}, c, b, A.frec, A.fldr, 0, A.ni);
      TG_STAMP(P, 3);
      return;
    }
  if constexpr ((ROLES & 4) != 0)
    if (part == kRecTq) { tq_records(P, A, c, b); TG_STAMP(P, 3); return; }
  if constexpr ((ROLES & 2) != 0) gs_records<ROTVEC>(P, A.g, c, b, smem, part == kRecGsDyn ? 1 : part == kRecGsRom ? 2 : 0);
  TG_STAMP(P, 3);
}
template <bool ROTVEC, int ROLES>
__global__ void __launch_bounds__(kGsRecMaxBlock) __attribute__((amdgpu_waves_per_eu(4))) towr_gait_rec_kernel(KParams P, RecArgs A) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  rec_body<ROTVEC, ROLES>(P, A, smem);
}
template <int ROLES>   // FDISC and / or TQDISC records only
// (5 or 6 waves per SIMD: 96 / 80 VGPRs with 48 / 120 bytes of spill, gait step 0.645-0.651 / 0.665-0.667 vs
// 0.630-0.631 ms; with Torque 1.24 / 1.30-1.31 vs 1.21)
__global__ void __launch_bounds__(kGsRecMaxBlock) __attribute__((amdgpu_waves_per_eu(4))) towr_gait_frec_kernel(KParams P, RecArgs A) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  rec_body<false, ROLES>(P, A, smem);
}

// ------------------------------------------------------------------------------------------------
// composers
// ------------------------------------------------------------------------------------------------
// The composer: one block per (GsBlock, group of problems b = g, g + ng, ...), the geometry's blob
// staged to LDS once. Per problem:
//   1. the block's record chunk (one contiguous range, prefetched into registers while the previous
//      problem streamed) to LDS, ints converted;
//   2. per (instant, segment): the window start in the instant and the segment's value base (wp);
//   3. per (instant, value): the value (CLS::value), one lane each;
//   4. the next problem's chunk is fetched; the CSR range [v0, v0 + nv) streams out, kGsUnits 16-byte
//      units composed per lane before their stores, every entry one lookup: its segment, the window,
//      the value or 0.
// LDS: [the geometry's blob (segments, value map, template, position -> segment, prefix codes, window
// starts; layout.h gs_blob) | values | records (doubles) | wp (int2) | record ints | nph].
// ForceConstraintDiscretized compose block: FsBlock jt for the problems g0, g0 + ng, ...
// LDS: [per-instant records (stride kFsCS) | row window values (5 n x kFsWin) | row window starts (5 n)]
// 16-byte units composed per lane before their stores (experiment builds: -DTOWR_FS_UNITS / -DTOWR_GS_UNITS). One unit
// per lane: the composers then leave CU time and memory slots to the launches beside them. MI355X, ANYmal gait, B = 1024,
// same box, 4 runs each (gpurun_out/r05q_ab.log), (FDISC units, GsBlock units) -> step ms, + Torque ms:
// (4, 4) 0.624-0.638, 1.208-1.211; (2, 2) 0.612-0.620, 1.178-1.180; (1, 2) 0.614-0.616, 1.181-1.186;
// (1, 1) 0.606-0.618, 1.162-1.167; (8, 8) 0.715-0.719, 1.310-1.316 (r05o). The FDISC compose alone is slower with fewer
// units (0.383 -> 0.397 ms at 2), the overlapped step faster.
#ifndef TOWR_FS_UNITS
#define TOWR_FS_UNITS 1
#endif
#ifndef TOWR_GS_UNITS
#define TOWR_GS_UNITS 1
#endif
constexpr int kFsUnits = TOWR_FS_UNITS;
// The row window values and starts of an FsBlock's rows from its instants' records in LDS (cd: instant kk's record at
// kk * kFsCS): window value q of row r = b[i][e(q)] * basis sum q (emit_dim; 0.0 where the sum is exactly 0)
template <int BLOCK>
__device__ __forceinline__ void fs_rows(const FsBlock& fb, const double* cd, double* rowv, int32_t* wsr) {
  const int tid = threadIdx.x, nr = 5 * fb.n_inst;
  auto ci = [&](int k, int f) -> int { return reinterpret_cast<const int32_t*>(cd + k * kFsCS + kFsND)[f]; };   // ws, wd, cur, wq
  for (int t = tid; t < nr * kFsWin; t += BLOCK) {
    const int r = t / kFsWin, q = t - r * kFsWin;
    const int k = r / 5, i = r - 5 * k;
    const int ed = (ci(k, 1) >> (2 * q)) & 3;   // 3: not an active column
    const double v = ed == 3 ? 0.0 : cd[k * kFsCS + ((ci(k, 3) >> (2 * q)) & 3)];
    rowv[t] = v == 0.0 ? 0.0 : cd[k * kFsCS + kFsB + 3 * i + ed] * v;
  }
  for (int t = tid; t < nr; t += BLOCK) wsr[t] = ci(t / 5, 0);
}
// The FsBlock's CSR range [v0, v0 + nv) of problem b with 16-byte non-temporal stores, UNITS units composed per lane
// before their stores (UNITS stores in flight instead of one per LDS round trip); every entry one lookup: a schedule
// column from the instant's d force / d schedule and pyramid row (eval_fdisc's arithmetic, see fdisc_sched_value), a
// force column from the row's window, else 0
template <int BLOCK, int UNITS>
__device__ __forceinline__ void fs_stream(const KParams& P, const FsBlock& fb, int b, const double* cd, const double* rowv,
                                          const int32_t* wsr) {
  // no contraction: a schedule entry is a sum of three products that cancels to a rounding residue where the force is
  // flat, and the fused / record + compose instantiations must form it with the same operations (with contraction the
  // compiler fused different products in the two kernels: 391 of 241,250 residues differed by up to 3e-13)
#pragma clang fp contract(off)
  const int tid = threadIdx.x;
  const int Lr = fb.L, js0 = fb.js0, ns1 = fb.ns1;
  const float invL = 1.0f / (float)Lr;   // exact row for block ranges below kFloatDivMax (layout.h, checked by build_fstream)
  auto ci = [&](int k, int f) -> int { return reinterpret_cast<const int32_t*>(cd + k * kFsCS + kFsND)[f]; };
  // entry j of row r (instant k = r / 5, pyramid row i): eval_fdisc's value (see fdisc_sched_value / emit_dim)
  auto entry = [&](int r, int j) -> double {
#pragma clang fp contract(off)   // (lambda bodies: the enclosing function's pragma is not relied on)
    const unsigned js = (unsigned)(j - js0);
    if (js < (unsigned)ns1) {   // schedule column js: sched_val per dimension, then the b-weighted sum
      const int k = r / 5, i = r - 5 * k;
      const double* d = cd + k * kFsCS;
      const int cur = ci(k, 2), col = (int)js;
      const bool last = cur == ns1;   // J.cur == J.n - 1
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
      if (col == cur && !last) {
        s0 = d[kFsDx + 0]; s1 = d[kFsDx + 1]; s2 = d[kFsDx + 2];
      } else if (col < cur) {
        const double v0 = d[kFsV + 0], v1 = d[kFsV + 1], v2 = d[kFsV + 2];
        if (last) {
          s0 = -v0 - d[kFsDx + 0]; s1 = -v1 - d[kFsDx + 1]; s2 = -v2 - d[kFsDx + 2];
        } else {
          s0 = -v0; s1 = -v1; s2 = -v2;
        }
      }
      return d[kFsB + 3 * i] * s0 + d[kFsB + 3 * i + 1] * s1 + d[kFsB + 3 * i + 2] * s2;
    }
    const unsigned q = (unsigned)(j - wsr[r]);
    return q < (unsigned)kFsWin ? rowv[r * kFsWin + q] : 0.0;
  };
  auto value = [&](int e) -> double {
    const int r = (int)(((float)e + 0.5f) * invL);
    return entry(r, e - r * Lr);
  };
  double* out = P.V + (int64_t)b * P.ldv + fb.v0;
  const int nv = fb.nv;
  const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
  if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
  const int m2 = (nv - head) >> 1;
  dbl2_t* d2 = reinterpret_cast<dbl2_t*>(out + head);
  for (int u0 = tid - trip_skew<0>(d2); u0 < m2; u0 += BLOCK * UNITS) {
    dbl2_t v[UNITS];
#pragma unroll
    for (int q = 0; q < UNITS; ++q) {
      const int u = max(u0 + q * BLOCK, 0);
      const int e = head + 2 * u;
      const int r = (int)(((float)e + 0.5f) * invL);
      const int j = e - r * Lr;
#ifdef TOWR_FS_PURE   // experiment build: the stream without the entries' arithmetic (bandwidth of the store pattern)
      v[q].x = (double)r; v[q].y = (double)j;
#else
      v[q].x = u < m2 ? entry(r, j) : 0.0;
      v[q].y = u < m2 ? (j + 1 < Lr ? entry(r, j + 1) : entry(r + 1, 0)) : 0.0;
#endif
    }
#pragma unroll
    for (int q = 0; q < UNITS; ++q)
#ifdef TOWR_FS_PLAIN
      if ((unsigned)(u0 + q * BLOCK) < (unsigned)m2) d2[u0 + q * BLOCK] = v[q];
#else
      if ((unsigned)(u0 + q * BLOCK) < (unsigned)m2) __builtin_nontemporal_store(v[q], d2 + u0 + q * BLOCK);
#endif
  }
  if (((nv - head) & 1) && tid == 0) __builtin_nontemporal_store(value(nv - 1), out + nv - 1);
}

template <int BLOCK>
__device__ __forceinline__ void fdisc_compose(const KParams& P, const double* rec, int64_t ldr, int ng, int jt, int g0, double* smem) {
  constexpr int kFsPre = (kFsInst * kFsRS + BLOCK - 1) / BLOCK;   // prefetched record doubles per thread
  const FsBlock fb = P.fsb[jt];
  const int tid = threadIdx.x, n = fb.n_inst, nr = 5 * n;
  double* cd = smem;
  double* rowv = cd + ((n * kFsCS + 1) & ~1);
  int32_t* wsr = reinterpret_cast<int32_t*>(rowv + nr * kFsWin);
  // the chunk: element e = f * n + kk -> LDS kk * kFsCS + f
  const int nch = n * kFsRS;
  const int64_t chunk0 = (int64_t)kFsRS * fb.t0;
  int dst[kFsPre];
#pragma unroll
  for (int q = 0; q < kFsPre; ++q) {
    const int e = tid + q * BLOCK;
    const int f = e / n, kk = e - f * n;
    dst[q] = e >= nch ? -1 : kk * kFsCS + f;
  }
  double pre[kFsPre];
  auto fetch = [&](int b) {
    const double* src = rec + (int64_t)b * ldr + chunk0;
#pragma unroll
    for (int q = 0; q < kFsPre; ++q) pre[q] = dst[q] >= 0 ? src[tid + q * BLOCK] : 0.0;
  };
  int b = g0;
  // (the compose block forming its instants' records itself from x and the PhaseSpline tables in global
  // memory, instead of reading them: FDISC 0.42 -> 2.7 ms per 1024 problems, the dependent table loads;
  // from tables staged in LDS, a fused kernel of round 5: 0.76 vs 0.63 ms per gait step)
  TG_STAMP(P, 0);
  fetch(b);
  int it = 0;
  for (;;) {
#pragma unroll
    for (int q = 0; q < kFsPre; ++q)
      if (dst[q] >= 0) cd[dst[q]] = pre[q];
    __syncthreads();
    if (it == 0) TG_STAMP(P, 1);
    fs_rows<BLOCK>(fb, cd, rowv, wsr);
    __syncthreads();
    if (it == 0) TG_STAMP(P, 2);
    const int bn = b + ng;
    if (bn < P.B) fetch(bn);   // in flight while this problem streams
    fs_stream<BLOCK, kFsUnits>(P, fb, b, cd, rowv, wsr);
    if (it == 0) TG_STAMP(P, 3);
    ++it;
    if (bn >= P.B) break;
    b = bn;
    __syncthreads();   // this problem's records and row values read before the next deposit
  }
  TG_STAMP(P, 4);
}

constexpr int kGsUnits = TOWR_GS_UNITS;
template <int CLS, int BLOCK>
__device__ __forceinline__ void gs_compose(const KParams& P, const GsBlock* blks, const double* rec, int64_t ldr, int ng, int j, int g0,
                                           double* smem) {
  using C = typename std::conditional<CLS == GS_ROM, RomCls, typename std::conditional<CLS == GS_TQ, TqCls, DynCls>::type>::type;
  constexpr int kGsPre = kGsChunkMax / BLOCK;   // prefetched record doubles per thread
  const GsBlock bl = blks[j];
  const GsGeo g = P.gs_geo[bl.geo];
  const int E = P.rb.n_ee, n = bl.n_inst, tid = threadIdx.x;
  const int ND = gs_rec_nd(CLS, E), NI = gs_rec_ni(CLS, E), RS = ND + NI;
  const int CS = RS | 1, vt = g.vt, ns = g.ns;
  // LDS: [blob | values | records | wp (int2) | nph]
  char* blob = reinterpret_cast<char*>(smem);
  double* val = smem + 2 * g.blob_n16;
  double* cd = val + ((n * vt + 1) & ~1);
  int2* wp = reinterpret_cast<int2*>(cd + ((n * CS + 1) & ~1));
  int32_t* nph = reinterpret_cast<int32_t*>(wp + n * ns);
  stage16<BLOCK>(reinterpret_cast<uint4*>(blob), P.gs_blob + g.blob0, g.blob_n16);
  if (tid < E) nph[tid] = P.sched[tid].n_phases;
  const GsSeg* segs = reinterpret_cast<const GsSeg*>(blob);
  const uint32_t* vmap = reinterpret_cast<const uint32_t*>(blob + g.o_vmap);
  const int32_t* tmpl = reinterpret_cast<const int32_t*>(blob + g.o_tmpl);
  const uint8_t* tsg = reinterpret_cast<const uint8_t*>(blob + g.o_tseg);
  const uint8_t* pcl = reinterpret_cast<const uint8_t*>(blob + g.o_pcode) + bl.k0 * g.Psum;
  const int16_t* wsl = reinterpret_cast<const int16_t*>(blob + g.o_ws);
  // the chunk: element e = f * n + kk -> LDS kk * CS + f
  const int nch = n * RS;
  const int64_t chunk0 = (int64_t)RS * (g.rec0 + bl.k0);
  int dst[kGsPre];
#pragma unroll
  for (int q = 0; q < kGsPre; ++q) {
    const int e = tid + q * BLOCK;
    const int f = e / n, kk = e - f * n;
    dst[q] = e >= nch ? -1 : kk * CS + f;
  }
  double pre[kGsPre];
  auto fetch = [&](int b) {
    const double* src = rec + (int64_t)b * ldr + chunk0;
#pragma unroll
    for (int q = 0; q < kGsPre; ++q) pre[q] = dst[q] >= 0 ? src[tid + q * BLOCK] : 0.0;
  };
  auto deposit = [&]() {
#pragma unroll
    for (int q = 0; q < kGsPre; ++q)
      if (dst[q] >= 0) cd[dst[q]] = pre[q];
  };
  const int Li = g.Li;
  const float invLi = 1.0f / (float)Li;
  auto value = [&](int e) -> double {
    const int kk = (int)(((float)e + 0.5f) * invLi);   // exact below kFloatDivMax (layout.h, checked by build_gstream_class)
    const int rr = e - kk * Li;
    const int2 p = wp[kk * ns + tsg[rr]];
    const unsigned q = (unsigned)(rr - p.x);
    return q < (unsigned)(p.y >> 16) ? val[(p.y & 0xFFFF) + q] : 0.0;
  };
  const int nv = bl.nv;
  int b = g0;
  TG_STAMP(P, 0);
  fetch(b);
  int it = 0;
  for (;;) {
    deposit();
    __syncthreads();
    if (it == 0) TG_STAMP(P, 1);
    for (int t = tid; t < n * ns; t += BLOCK) {   // window starts and value bases
      const int kk = t / ns, sid = t - kk * ns;
      const GsSeg sg = segs[sid];
      int ws = 0;
      if (sg.type == 1) ws = wsl[sg.wsoff + C::poly(reinterpret_cast<const int32_t*>(cd + kk * CS + ND), sg.kind, sg.ee)];
      wp[t] = make_int2(sg.p0 + ws, ((int)sg.W << 16) | (kk * vt + sg.vbase));
    }
    __syncthreads();
    if (it == 0) TG_STAMP(P, 2);
    // (2 or 4 values per thread formed before their LDS stores, so that their load chains overlap: the value phase is
    // 3.6 / 5.6 of a 15 / 19 us Dynamic / RangeOfMotion block (tools/stamps.py), but the gait step measured 0.595-0.603
    // vs 0.594-0.607 ms and + Torque 1.19-1.20 vs 1.16 ms: not kept)
    // every value of every instant, once; instant-fastest lanes (t = v n + kk), so that a wave's lanes share a few value
    // slots and with them one segment's code path (instant-major lanes mixed 2-3 segment kinds in most waves)
    const float invn = 1.0f / (float)n;   // exact: n vt < kFloatDivMax (build_gstream_class's encodings)
    for (int t = tid; t < n * vt; t += BLOCK) {
      const int v = (int)(((float)t + 0.5f) * invn), kk = t - v * n;
      const uint32_t vm = vmap[v];
      const int sid = (int)(vm >> 16), q = (int)(vm & 0xFFFF);
      const GsSeg sg = segs[sid];
      const int pos = wp[kk * ns + sid].x + q;   // position in the instant
      double x = 0.0;
      if (pos < sg.p0 + sg.len) {
        const double* d = cd + kk * CS;
        const int32_t* ci = reinterpret_cast<const int32_t*>(d + ND);
        if constexpr (CLS == GS_DYN) x = C::value(P.rb, tmpl, sg, pos, d, ci, pcl + kk * g.Psum, nph);
        else x = C::value(P.rb, tmpl, sg, pos, d, ci, pcl + kk * g.Psum, nph[g.ee]);
      }
      val[kk * vt + v] = x;
    }
    __syncthreads();
    if (it == 0) TG_STAMP(P, 3);
    const int bn = b + ng;
    if (bn < P.B) fetch(bn);   // in flight while this problem streams
    double* out = P.V + (int64_t)b * P.ldv + bl.v0;
    const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
    if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
    const int m2 = (nv - head) >> 1;
    dbl2_t* d2 = reinterpret_cast<dbl2_t*>(out + head);
    for (int u0 = tid - (CLS == GS_TQ ? trip_skew<3>(d2) : trip_skew<1>(d2)); u0 < m2; u0 += BLOCK * kGsUnits) {
      dbl2_t v[kGsUnits];
#pragma unroll
      for (int q = 0; q < kGsUnits; ++q) {
        const int u = u0 + q * BLOCK;
        const int e = head + 2 * max(u, 0);
        v[q].x = (unsigned)u < (unsigned)m2 ? value(e) : 0.0;
        v[q].y = (unsigned)u < (unsigned)m2 ? value(e + 1) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < kGsUnits; ++q)
        if ((unsigned)(u0 + q * BLOCK) < (unsigned)m2) __builtin_nontemporal_store(v[q], d2 + u0 + q * BLOCK);
    }
    if (((nv - head) & 1) && tid == 0) __builtin_nontemporal_store(value(nv - 1), out + nv - 1);
    if (it == 0) TG_STAMP(P, 4);
    ++it;
    if (bn >= P.B) break;
    b = bn;
    __syncthreads();   // this problem's wp / values / records read before the next deposit
  }
  TG_STAMP(P, 5);
}


// The composer launch: every compose block of every problem in one grid. Per problem group the units are
// [FDISC FsBlocks | TQDISC GsBlocks | RangeOfMotion GsBlocks | Dynamic GsBlocks | small-kind groups] (A.nt),
// so the write-bound FDISC blocks and the Dynamic blocks' longer value phases interleave on every CU, and one
// launch replaces several (at B = 1 a launch boundary costs more than a compose block). XCD-aware: blocks
// are dealt round-robin over the 8 XCDs; XCD x takes the contiguous range [x per, (x + 1) per) of (group,
// unit) pairs, so each XCD writes whole problems' CSR ranges.
template <int BLOCK, int MASK>   // MASK: the roles of this instantiation (bit 0 FDISC, 1 RangeOfMotion, 2 Dynamic, 3 small kinds, 4 TQDISC)
__global__ void __launch_bounds__(BLOCK, 1) towr_gait_compose_kernel(KParams P, ComposeArgs A) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int NT = A.nt[0] + A.nt[1] + A.nt[2] + A.nt[3] + A.nt[4];
  const int per = (int)((gridDim.x + 7) / 8);
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  int j = w % NT;
  const int g0 = w / NT;
  if (g0 >= A.ng || g0 >= P.B) return;   // the grid is rounded up to a multiple of 8
  if constexpr ((MASK & 1) != 0)
    if (j < A.nt[0]) { fdisc_compose<BLOCK>(P, A.frec, A.fldr, A.ng, j, g0, smem); return; }
  j -= A.nt[0];
  if constexpr ((MASK & 16) != 0)
    if (j < A.nt[4]) { gs_compose<GS_TQ, BLOCK>(P, A.blk[GS_TQ], A.frec + A.tq_off, A.fldr, A.ng, j, g0, smem); return; }
  j -= A.nt[4];
  if constexpr ((MASK & 2) != 0)
    if (j < A.nt[1]) { gs_compose<GS_ROM, BLOCK>(P, A.blk[GS_ROM], A.grec, A.gldr, A.ng, j, g0, smem); return; }
  j -= A.nt[1];
  if constexpr ((MASK & 4) != 0)
    if (j < A.nt[2]) { gs_compose<GS_DYN, BLOCK>(P, A.blk[GS_DYN], A.grec + A.gdyn_off, A.gldr, A.ng, j, g0, smem); return; }
  j -= A.nt[2];
  if constexpr ((MASK & 8) != 0)   // a small-kind group (tile_emit.h misc_body) of each of the block's problems
    for (int b = g0; b < P.B; b += A.ng) {
      misc_body<true, BLOCK>(P, smem, b, j, A.misc_x_off);
      __syncthreads();
    }
}

}  // namespace

// LDS (bytes) of the composer of class cls: sized for the class's largest geometry (GsGeo)
size_t gs_stream_lds(const Layout& L, int cls) {
  const int E = L.rb.n_ee;
  const size_t n = (size_t)L.gs_nmax[cls];
  const size_t ns = (size_t)L.gs_geo_max[cls][1], vt = (size_t)L.gs_geo_max[cls][2], blob = (size_t)L.gs_geo_max[cls][3];
  const size_t CS = (size_t)(gs_rec_fields(cls, E) | 1);
  size_t b = blob + 8 * (((n * vt + 1) & ~(size_t)1) + ((n * CS + 1) & ~(size_t)1));
  b += 8 * n * ns + 4 * TOWR_MAX_EE;
  return (b + 15) & ~(size_t)15;
}
int64_t gs_record_doubles(const Layout& L, int cls) {
  const int64_t K = (int64_t)L.gs_inst[cls].size();
  return ((int64_t)gs_rec_fields(cls, L.rb.n_ee) * K + 1) & ~(int64_t)1;
}
const void* gait_rec_kernel(bool rotvec, int roles) {   // roles: bit 0 FDISC, 1 RangeOfMotion / Dynamic, 2 TQDISC
  if ((roles & 2) == 0)
    return roles == 1 ? reinterpret_cast<const void*>(&towr_gait_frec_kernel<1>) : roles == 4 ? reinterpret_cast<const void*>(&towr_gait_frec_kernel<4>)
                      : reinterpret_cast<const void*>(&towr_gait_frec_kernel<5>);
  if (roles == 2) return rotvec ? reinterpret_cast<const void*>(&towr_gait_rec_kernel<true, 2>) : reinterpret_cast<const void*>(&towr_gait_rec_kernel<false, 2>);
  if (roles == 3) return rotvec ? reinterpret_cast<const void*>(&towr_gait_rec_kernel<true, 3>) : reinterpret_cast<const void*>(&towr_gait_rec_kernel<false, 3>);
  return rotvec ? reinterpret_cast<const void*>(&towr_gait_rec_kernel<true, 7>) : reinterpret_cast<const void*>(&towr_gait_rec_kernel<false, 7>);
}
template <int MASK>
const void* compose_fn() { return reinterpret_cast<const void*>(&towr_gait_compose_kernel<(MASK & 25) ? kComposeBlock : kComposeBlockRD, MASK>); }
const void* gait_compose_kernel(int mask) {
  // the instantiations the host launches (towr_gpu.hip launch_stream_path, layout.h kComposeMasks): at small
  // batch sizes every role in one launch; at large ones the FDISC (+ TQDISC) chain beside the Dynamic and
  // RangeOfMotion launches (one class alone: the per-class timings); block sizes: compose_block
  switch (mask) {
    case 1: return compose_fn<1>();
    case 2: return compose_fn<2>();
    case 4: return compose_fn<4>();
    case 6: return compose_fn<6>();
    case 7: return compose_fn<7>();
    case 15: return compose_fn<15>();
    case 16: return compose_fn<16>();
    case 17: return compose_fn<17>();
    case 23: return compose_fn<23>();
    default: return compose_fn<31>();
  }
}
size_t fs_compose_lds(const Layout& L) {   // records, row window values, row window starts
  return sizeof(double) * ((size_t)(((kFsInst * kFsCS + 1) & ~1) + 5 * kFsInst * kFsWin + (5 * kFsInst + 1) / 2 + 1) & ~(size_t)1);
}
size_t gs_dyn_state_bytes(bool rotvec) { return rotvec ? dyn_state_bytes<true>() : dyn_state_bytes<false>(); }

}  // namespace tg
