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
// ~90 % exact zeros whose positions move with x. Two launches:
//   A. towr_fdisc_inst_kernel, one block per problem, one lane per instant: fdisc_instant's result
//      in the stream kernel's form — the basis sums of the kFsWin columns the force polynomial can
//      touch (phase_basis_sum over the instant's window of the template), the 5 pyramid rows b,
//      d force / d schedule, the window start and dimension codes — goes to a per-problem record
//      array in HBM (the handle's scratch); the instant's g rows go straight out. Records are
//      chunk-major per FsBlock (field f of the block's instant kk at kFsRS t0 + f n + kk), so a
//      stream block's prologue is one contiguous copy;
//   B. towr_fdisc_stream_kernel, one block per (FsBlock, group of problems): per problem the block's
//      record chunk (prefetched into registers while the previous problem streamed) goes to LDS,
//      each row's window values b[i][e] * (basis sum) are formed once, and the block's whole CSR range
//      streams out with 16-byte non-temporal stores, each unit written once: an entry is its row's
//      window value inside the window, the schedule combination in the schedule columns, else 0.0
//      (pyramid / phase_basis_sum / fdisc_sched_value: eval_fdisc's operations).
// record: Hv[kFsWin] | b[5][3] | Jf.dx[3] | Jf.v[3] | ints ws, wd, cur (64-bit integer bit patterns)
constexpr int kFsB = kFsWin, kFsDx = kFsWin + 15, kFsV = kFsWin + 18, kFsND = kFsWin + 21;
constexpr int kFsRS = kFsND + 3, kFsCS = kFsRS | 1;   // record fields; LDS stride per instant
constexpr int kFsInstBlock = 512;
__device__ __forceinline__ double fs_int(int v) { return __longlong_as_double((long long)v); }

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
    const FsBlock fb = P.fsb[P.fs_iblk[k]];
    const int kk = k - fb.t0, nb = fb.n_inst;
    double* r = R + (int64_t)kFsRS * fb.t0 + kk;
    auto put = [&](int f, double v) { r[f * nb] = v; };
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int e = 0; e < 3; ++e) put(kFsB + 3 * i + e, o.b[i][e]);
#pragma unroll
    for (int e = 0; e < 3; ++e) { put(kFsDx + e, o.Jf.dx[e]); put(kFsV + e, o.Jf.v[e]); }
    put(kFsND + 2, fs_int(o.Jf.cur));
    if (P.want_g) {
      const int row = P.fs_irow[k];
#pragma unroll
      for (int i = 0; i < 5; ++i) __builtin_nontemporal_store(o.g[i], Gb + row + i);
    }
    const int poly = o.poly;
    const int ws = P.fs_ws[2 * (fb.wsoff + poly)], wd = P.fs_ws[2 * (fb.wsoff + poly) + 1];
    put(kFsND, fs_int(ws));
    put(kFsND + 1, fs_int(wd));
    double h0 = o.H[0], h1 = o.H[1], h2 = o.H[2], h3 = o.H[3];
    asm volatile("" : "+v"(h0), "+v"(h1), "+v"(h2), "+v"(h3));
    const int32_t* tm = P.fs_tmpl + fb.tmpl;
#pragma unroll 4
    for (int q = 0; q < kFsWin; ++q) {   // the window's basis sums (schedule entries: never read, 0)
      const int pos = ws + q;
      const int32_t te = pos < fb.L ? tm[pos] : -1;
      put(q, te >= 0 ? phase_basis_sum(c.pcols[te & 0xFFFFFF], poly, h0, h1, h2, h3) : 0.0);
    }
  }
}

// B. LDS: [per-instant records (stride kFsCS) | row window values (5 n x kFsWin) | row window starts (5 n)]
constexpr int kFsUnits = 4;   // 16-byte units composed per lane before their stores
constexpr int kFsPre = (kFsInst * kFsRS + kFsBlock - 1) / kFsBlock;   // prefetched record doubles per thread
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK, 1) towr_fdisc_stream_kernel(KParams P, const double* rec, int64_t ldr, int32_t ng) {
  static_assert(BLOCK == kFsBlock, "the prefetch is sized for kFsBlock");
  extern __shared__ __attribute__((aligned(16))) double smem[];
  // XCD-aware: blocks are dealt round-robin over the 8 XCDs; XCD x takes the contiguous range
  // [x per, (x + 1) per) of (group, block) pairs, so each XCD writes whole problems' CSR ranges
  const int per = (int)((gridDim.x + 7) / 8);
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  const int jt = w % P.ntiles, g0 = w / P.ntiles;
  if (g0 >= ng || g0 >= P.B) return;   // the grid is rounded up to a multiple of 8
  const FsBlock fb = P.fsb[jt];
  const int tid = threadIdx.x, n = fb.n_inst, nr = 5 * n;
  double* cd = smem;
  double* rowv = cd + ((n * kFsCS + 1) & ~1);
  int32_t* wsr = reinterpret_cast<int32_t*>(rowv + nr * kFsWin);
  auto ci = [&](int k, int f) -> int { return *reinterpret_cast<const int32_t*>(cd + k * kFsCS + kFsND + f); };   // ws, wd, cur
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
  const int Lr = fb.L, js0 = fb.js0, ns1 = fb.ns1;
  const float invL = 1.0f / (float)Lr;   // exact row of element e < 2^20 for rows <= 4096 long (|err| << 0.5 / Lr)
  // entry j of row r (instant k = r / 5, pyramid row i): eval_fdisc's value (see fdisc_sched_value / emit_dim)
  auto entry = [&](int r, int j) -> double {
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
  int b = g0;
  fetch(b);
  for (;;) {
#pragma unroll
    for (int q = 0; q < kFsPre; ++q)
      if (dst[q] >= 0) cd[dst[q]] = pre[q];
    __syncthreads();
    for (int t = tid; t < nr * kFsWin; t += BLOCK) {   // window value q of row r: b[i][e(q)] * basis sum (emit_dim)
      const int r = t / kFsWin, q = t - r * kFsWin;
      const int k = r / 5, i = r - 5 * k;
      const double v = cd[k * kFsCS + q];
      const int ed = (ci(k, 1) >> (2 * q)) & 3;
      rowv[t] = v == 0.0 ? 0.0 : cd[k * kFsCS + kFsB + 3 * i + ed] * v;
    }
    for (int t = tid; t < nr; t += BLOCK) wsr[t] = ci(t / 5, 0);
    __syncthreads();
    const int bn = b + ng;
    if (bn < P.B) fetch(bn);   // in flight while this problem streams
    if (P.want_jac) {
      double* out = P.V + (int64_t)b * P.ldv + fb.v0;
      const int nv = fb.nv;
      const int head = (reinterpret_cast<uintptr_t>(out) & 15) ? 1 : 0;
      if (head && tid == 0) __builtin_nontemporal_store(value(0), out);
      const int m2 = (nv - head) >> 1;
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
      if (((nv - head) & 1) && tid == 0) __builtin_nontemporal_store(value(nv - 1), out + nv - 1);
    }
    if (bn >= P.B) break;
    b = bn;
    __syncthreads();   // this problem's records and row values read before the next deposit
  }
}

}  // namespace

size_t fs_region(const Layout& L) {   // stream kernel (B) LDS in doubles: records, row window values, row window starts
  return (size_t)(((kFsInst * kFsCS + 1) & ~1) + 5 * kFsInst * kFsWin + (5 * kFsInst + 1) / 2 + 1) & ~(size_t)1;
}
int64_t fs_record_doubles() { return kFsRS; }
const void* fs_inst_kernel() { return reinterpret_cast<const void*>(&towr_fdisc_inst_kernel<kFsInstBlock>); }
const void* fs_stream_kernel() { return reinterpret_cast<const void*>(&towr_fdisc_stream_kernel<kFsBlock>); }
int fs_inst_block() { return kFsInstBlock; }
}  // namespace tg
