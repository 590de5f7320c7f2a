// cost_traj.hip — the objective kernel (IpoptAdapter::eval_f / eval_grad_f) and the
// trajectory-export kernel (SaveTrajectoryToCSV, §4b) of the engine; the host side (towr_gpu.hip)
// reaches them through cost_kernel_for / traj_kernel_for (kernel_common.h).
#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"

namespace tg {
namespace {

// Objective and gradient (IpoptAdapter::eval_f / eval_grad_f): one block per problem. The block
// stages x and the node table in LDS and keeps the problem's dense gradient there; lanes take the
// cost work items round-robin (grouped by kind, so waves mostly run one path) and add their
// gradient entries with LDS atomics (ds_add_f64); f is reduced over the block. The gradient then
// leaves with 16-byte non-temporal stores. The gradient's summation order is not fixed (atomics),
// so it is reproducible to rounding only; f's order is fixed.
template <bool GRAD>
struct CostEmit {
  double* grad;   // LDS; the dump slot at index n absorbs constant node values
  double f = 0.0;
  static constexpr bool kSparse = true;   // zero gradient contributions need no atomic
  __device__ __forceinline__ void skip(int) {}
  __device__ __forceinline__ void operator()(int, int col, double v, bool pres) {
    if constexpr (GRAD)
      if (pres && v != 0.0) atomicAdd(grad + col, v);
  }
};

template <bool GAIT, bool GRAD, bool ROTVEC>
__global__ void __launch_bounds__(kCostBlock, 1) towr_cost_kernel(KParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int b = blockIdx.x;
  double* gs = smem;                       // [n_pad] gradient (+ dump slot at n)
  double* xs = smem + P.n_pad;             // [n_pad] x (+ zero slot at n)
  int32_t* ns = reinterpret_cast<int32_t*>(smem + 2 * P.n_pad);
  double* red = smem + P.lds_red_off;     // [kCostBlock / 64] per-wave partial objectives
  stage_x<kCostBlock, true>(P, P.X + (int64_t)b * P.ldx, xs, ns);
  if constexpr (GRAD)
    for (int i = threadIdx.x; i < P.n_pad; i += kCostBlock) gs[i] = 0.0;
  __syncthreads();
  CostEmit<GRAD> em{gs};
  Ctx c;
  c.x = xs; c.nodecol = ns; c.spl = P.spl; c.dur = P.dur;
  c.ter = P.terrains + (P.terrain_per_problem ? b : 0);
  c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
  c.gait = GAIT; c.pinfo = P.pinfo; c.pcols = P.pcols; c.pact = P.pact; c.sched = P.sched; c.eelin = P.eelin; c.lin = P.lin;
  c.rotvec = ROTVEC;
  c.dyn_scratch = nullptr;
  c.cq = P.cq;
  for (int i = threadIdx.x; i < P.n_citems; i += kCostBlock) {
    const CostItem it = P.citems[i];
    c.seg = nullptr; c.sg = P.sg; c.row = it.seg;
    eval_cost_item(c, it, em);
  }
  // SoftConstraint terms (soft_constraint.cc:52-69): 0.5 (g - b)^T (g - b) and J^T (g - b) over the
  // wrapped sets' rows, from the soft child's g and CSR values of this problem (one row per lane)
  if (P.s_m > 0) {
    const double* sg = P.sG + (int64_t)b * P.s_ldg;
    for (int r = threadIdx.x; r < P.s_m; r += kCostBlock) {
      const double d = sg[r] - P.s_b[r];
      em.f += (0.5 * d) * d;
      if constexpr (GRAD) {
        const double* sv = P.sV + (int64_t)b * P.s_ldv;
        for (int k = P.s_rp[r]; k < P.s_rp[r + 1]; ++k) {
          const double v = sv[k] * d;
          if (v != 0.0) atomicAdd(gs + P.s_col[k], v);
        }
      }
    }
  }
  // f: wave butterfly, then the waves' partials in order
  double f = em.f;
  for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < kCostBlock / 64; ++w) s += red[w];
    P.F[b] = s;
  }
  if constexpr (GRAD) copy_out(gs, P.GR + (int64_t)b * P.ldgr, P.n, threadIdx.x, kCostBlock);
}
// Trajectory export (SaveTrajectoryToCSV): one 64-lane block per (problem, 64 sample times). Each
// lane evaluates its sample's row into an LDS buffer kept column-major with an odd stride (writes and
// reads both conflict-free); the block's rows are one contiguous output range, copied out coalesced.
template <bool GAIT>
__global__ void __launch_bounds__(kTrajBlock, 1) towr_traj_kernel(KParams P, const double* times, int ns, TrajPhases ph,
                                                                   double* OUT, int64_t ldo, int32_t lds_x_off) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int nb = (ns + kTrajBlock - 1) / kTrajBlock;
  const int b = blockIdx.x / nb, k0 = (blockIdx.x % nb) * kTrajBlock;
  const int cols = traj_cols(P.rb.n_ee), stride = kTrajBlock + 1;
  double* rows = smem;
  double* xs = smem + lds_x_off;
  int32_t* nsp = reinterpret_cast<int32_t*>(xs + P.n_pad);
  stage_x<kTrajBlock, true>(P, P.X + (int64_t)b * P.ldx, xs, nsp);
  __syncthreads();
  const int k = k0 + (int)threadIdx.x;
  if (k < ns) {
    Ctx c;
    c.seg = nullptr; c.row = -1;
    c.x = xs; c.nodecol = nsp; c.spl = P.spl; c.dur = P.dur;
    c.ter = P.terrains; c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
    c.gait = GAIT; c.pinfo = P.pinfo; c.pcols = P.pcols; c.pact = P.pact; c.sched = P.sched; c.eelin = P.eelin; c.lin = P.lin;
    c.rotvec = false; c.dyn_scratch = nullptr;
    traj_row(c, ph, times[k], rows + threadIdx.x, stride);
  }
  __syncthreads();
  const int cnt = min(kTrajBlock, ns - k0);
  double* out = OUT + (int64_t)b * ldo + (int64_t)k0 * cols;
  for (int i = threadIdx.x; i < cnt * cols; i += kTrajBlock) {
    const int r = i / cols, col = i - r * cols;
    __builtin_nontemporal_store(rows[col * stride + r], out + i);
  }
}

}  // namespace

template <bool GAIT, bool GRAD>
const void* cost_kernel_rv(bool rotvec) {
  return rotvec ? reinterpret_cast<const void*>(&towr_cost_kernel<GAIT, GRAD, true>)
                : reinterpret_cast<const void*>(&towr_cost_kernel<GAIT, GRAD, false>);
}
const void* cost_kernel_for(bool gait, bool grad, bool rotvec) {
  if (gait) return grad ? cost_kernel_rv<true, true>(rotvec) : cost_kernel_rv<true, false>(rotvec);
  return grad ? cost_kernel_rv<false, true>(rotvec) : cost_kernel_rv<false, false>(rotvec);
}

const void* traj_kernel_for(bool gait) {
  return gait ? reinterpret_cast<const void*>(&towr_traj_kernel<true>) : reinterpret_cast<const void*>(&towr_traj_kernel<false>);
}

}  // namespace tg
