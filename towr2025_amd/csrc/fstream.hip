// fstream.hip — the streaming ForceConstraintDiscretized kernels (phase-duration optimisation on a
// terrain without curvature; layout.h FsBlock, towr_gpu.hip launch_fstream). Own translation unit so
// the kernel iterates without recompiling the tile kernels.
#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"


namespace tg {
namespace {

// Streaming ForceConstraintDiscretized under phase-duration optimisation (layout.h FsBlock). Every
// Jacobian row of the path is the force set's full PhaseSpline pattern plus the schedule columns,
// ~90 % exact zeros whose positions move with x. The tile path zero-filled the rows and scattered
// 8-byte value stores over them (partial lines written twice, 1.25x the algorithmic bytes) and
// evaluated each instant once per row. Here two launches split the work:
//   A. towr_fdisc_inst_kernel, one block per problem, one lane per instant: fdisc_instant's result
//      (the force polynomial, its position basis, the terrain basis n t1 t2, d force / d schedule)
//      goes to a per-problem record array in HBM (the handle's scratch, kFsRec doubles per instant,
//      field-major so a wave's stores coalesce); the instant's g rows go straight out;
//   B. towr_fdisc_stream_kernel, one block per (problem, FsBlock): the block's records come in, each
//      instant's pyramid rows b and the basis sums of the kFsWin columns its force polynomial can
//      touch are formed in LDS, and the block's whole CSR range streams out with 16-byte
//      non-temporal stores, each unit written once: an entry is b[i][e] * (basis sum) inside its
//      instant's window, the schedule combination in the schedule columns, else 0.0
//      (pyramid / phase_basis_sum / fdisc_sched_value: eval_fdisc's operations).
// A is latency-bound but holds every instant of the batch in flight at once; B carries no
// evaluation chain, so its blocks are small (LDS ~20 KB) and many, and it streams at the write ceiling.
constexpr int kFsRec = 21;   // record: H[4] | n t1 t2 [9] | Jf.dx[3] | Jf.v[3] | poly | cur
constexpr int kFsInstBlock = 512;
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK, 1) towr_fdisc_inst_kernel(KParams P, double* rec, int64_t ldr, int32_t ni) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  double* Gb = P.G + (int64_t)b * P.ldg;
  double* R = rec + (int64_t)b * ldr;
  const int tid = threadIdx.x;
  Ctx c = gait_record_setup<BLOCK>(P, b, smem);
  for (int k = tid; k < ni; k += BLOCK) {
    FdiscInstant o;
    fdisc_instant(c, P.fs_iee[k], P.fs_t[k], o);
    double* r = R + k;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q * (int64_t)ni] = o.H[q];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 3; ++e) r[(4 + 3 * q + e) * (int64_t)ni] = o.nb[q][e];
#pragma unroll
    for (int e = 0; e < 3; ++e) { r[(13 + e) * (int64_t)ni] = o.Jf.dx[e]; r[(16 + e) * (int64_t)ni] = o.Jf.v[e]; }
    r[19 * (int64_t)ni] = (double)o.poly;
    r[20 * (int64_t)ni] = (double)o.Jf.cur;
    if (P.want_g) {
      const int row = P.fs_irow[k];
#pragma unroll
      for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(o.g[i], Gb + row + i);
    }
  }
}

// B. LDS: [per-instant records kFsInst x kFsD doubles | ints ws, wd, cur (kFsInst x 3) | PhaseCol per template entry]
// Records are instant-major with an odd stride: a wave's lanes mostly read different fields of one or
// two instants, which then fall in different banks (field-major, every field of an instant sat in
// the same bank and the window reads serialized).
constexpr int kFsUnits = 4;   // 16-byte units composed per lane before their stores
constexpr int kFsD = 33;   // doubles per instant: window sums, b, d force / d schedule (dx, v)
constexpr int kFsHv = 0, kFsB = kFsWin, kFsDx = kFsWin + 15, kFsV = kFsWin + 18;
static_assert(kFsV + 3 == kFsD, "FsBlock LDS record");
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK, 1) towr_fdisc_stream_kernel(KParams P, const double* rec, int64_t ldr, int32_t ni) {
  static_assert(BLOCK >= kFsInst, "one lane per instant in the prologue");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);   // a problem's blocks share an XCD
  if (w >= total) return;
  const int b = w / P.ntiles;
  const FsBlock fb = P.fsb[w % P.ntiles];
  const int tid = threadIdx.x;
  double* cd = smem;
  int32_t* ci = reinterpret_cast<int32_t*>(smem + kFsD * kFsInst);
  PhaseCol* pcl = reinterpret_cast<PhaseCol*>(ci + 3 * kFsInst);
  for (int j = tid; j < fb.L; j += BLOCK) {
    const int32_t te = P.fs_tmpl[fb.tmpl + j];
    // schedule entries: n = 0, a zero basis sum (never read: schedule columns are tested first)
    const PhaseCol pq = P.pcols[te >= 0 ? (te & 0xFFFFFF) : 0];
    pcl[j] = pq;
    if (te < 0) pcl[j].n = 0;
  }
  __syncthreads();
  if (tid < fb.n_inst) {   // the instant's record -> b, window sums, schedule terms
    const int k = tid;
    const double* r = rec + (int64_t)b * ldr + fb.t0 + k;
    double h[4], nb[3][3], bb[5][3];
#pragma unroll
    for (int q = 0; q < 4; ++q) h[q] = r[q * (int64_t)ni];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int e = 0; e < 3; ++e) nb[q][e] = r[(4 + 3 * q + e) * (int64_t)ni];
#pragma unroll
    for (int e = 0; e < 3; ++e) { cd[k * kFsD + kFsDx + e] = r[(13 + e) * (int64_t)ni]; cd[k * kFsD + kFsV + e] = r[(16 + e) * (int64_t)ni]; }
    const int poly = (int)r[19 * (int64_t)ni];
    ci[3 * k + 2] = (int)r[20 * (int64_t)ni];
    const double mu = P.terrains[P.terrain_per_problem ? b : 0].friction_coeff;
    pyramid(nb[0], nb[1], nb[2], mu, bb);
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int e = 0; e < 3; ++e) cd[k * kFsD + kFsB + 3 * i + e] = bb[i][e];
    const int ws = P.fs_ws[2 * (fb.wsoff + poly)], wd = P.fs_ws[2 * (fb.wsoff + poly) + 1];
    double h0 = h[0], h1 = h[1], h2 = h[2], h3 = h[3];
    asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
#pragma unroll
    for (int q = 0; q < kFsWin; ++q) {
      const int pos = ws + q;
      double v = 0.0;
      if (pos < fb.L) {
        const PhaseCol pq = pcl[pos];
        v = phase_basis_sum(pq, poly, h0, h1, h2, h3);
      }
      cd[k * kFsD + kFsHv + q] = v;
    }
    ci[3 * k] = ws; ci[3 * k + 1] = wd;
  }
  __syncthreads();
  const int Lr = fb.L, js0 = fb.js0, ns1 = fb.ns1;
  const float invL = 1.0f / (float)Lr;   // exact row of element e < 2^20 for rows <= 4096 long (|err| << 0.5 / Lr)
  // entry j of row r (instant k = r / 5, pyramid row i): eval_fdisc's value (see fdisc_sched_value / emit_dim)
  auto entry = [&](int r, int j) -> double {
    const int k = r / 5, i = r - 5 * k;
    const unsigned js = (unsigned)(j - js0);
    if (js < (unsigned)ns1) {   // schedule column js: sched_val per dimension, then the b-weighted sum
      const int cur = ci[3 * k + 2], col = (int)js;
      const bool last = cur == ns1;   // J.cur == J.n - 1
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
      if (col == cur && !last) {
        s0 = cd[k * kFsD + kFsDx + 0]; s1 = cd[k * kFsD + kFsDx + 1]; s2 = cd[k * kFsD + kFsDx + 2];
      } else if (col < cur) {
        const double v0 = cd[k * kFsD + kFsV + 0], v1 = cd[k * kFsD + kFsV + 1], v2 = cd[k * kFsD + kFsV + 2];
        if (last) {
          s0 = -v0 - cd[k * kFsD + kFsDx + 0]; s1 = -v1 - cd[k * kFsD + kFsDx + 1]; s2 = -v2 - cd[k * kFsD + kFsDx + 2];
        } else {
          s0 = -v0; s1 = -v1; s2 = -v2;
        }
      }
      return cd[k * kFsD + kFsB + 3 * i] * s0 + cd[k * kFsD + kFsB + 3 * i + 1] * s1 +
             cd[k * kFsD + kFsB + 3 * i + 2] * s2;
    }
    const unsigned q = (unsigned)(j - ci[3 * k]);
    if (q < (unsigned)kFsWin) {
      const double v = cd[k * kFsD + kFsHv + q];
      if (v == 0.0) return 0.0;
      const int ed = (ci[3 * k + 1] >> (2 * q)) & 3;
      return cd[k * kFsD + kFsB + 3 * i + ed] * v;
    }
    return 0.0;
  };
  auto value = [&](int e) -> double {
    const int r = (int)(((float)e + 0.5f) * invL);
    return entry(r, e - r * Lr);
  };
  if (P.want_jac) {
    double* out = P.V + (int64_t)b * P.ldv + fb.v0;
    const int n = fb.nv;
    const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
    if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
    const int m2 = (n - head) >> 1;
    dbl2_t* d2 = reinterpret_cast<dbl2_t*>(out + head);
    // kFsUnits units per lane composed into registers first, then stored together, so a lane keeps
    // kFsUnits stores in flight instead of one store per LDS round trip
    for (int u0 = tid; u0 < m2; u0 += BLOCK * kFsUnits) {
      dbl2_t v[kFsUnits];
#pragma unroll
      for (int q = 0; q < kFsUnits; ++q) {
        const int u = u0 + q * BLOCK;
        const int e = head + 2 * u;
        const int r = (int)(((float)e + 0.5f) * invL);
        const int j = e - r * Lr;
        v[q].x = u < m2 ? entry(r, j) : 0.0;
        v[q].y = u < m2 ? (j + 1 < Lr ? entry(r, j + 1) : entry(r + 1, 0)) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < kFsUnits; ++q)
        if (u0 + q * BLOCK < m2) __builtin_nontemporal_store(v[q], d2 + u0 + q * BLOCK);
    }
    if (((n - head) & 1) && tid == 0) __builtin_nontemporal_store(value(n - 1), out + n - 1);
  }
}


}  // namespace

size_t fs_region(const Layout& L) {   // stream kernel (B) LDS in doubles: records, ints, template PhaseCols
  return (size_t)((kFsD * kFsInst + (3 * kFsInst) / 2 + (L.fs_tmpl_max * sizeof(PhaseCol) + 7) / 8 + 1) & ~1);
}
int64_t fs_record_doubles() { return kFsRec; }
const void* fs_inst_kernel() { return reinterpret_cast<const void*>(&towr_fdisc_inst_kernel<kFsInstBlock>); }
const void* fs_stream_kernel() { return reinterpret_cast<const void*>(&towr_fdisc_stream_kernel<kFsBlock>); }
int fs_inst_block() { return kFsInstBlock; }
}  // namespace tg
