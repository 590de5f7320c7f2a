// cost_traj.hip — the objective kernel (IpoptAdapter::eval_f / eval_grad_f) and the
// trajectory-export kernel (SaveTrajectoryToCSV, §4b) of the engine; the host side (towr_gpu.hip)
// reaches them through cost_kernel_for / traj_kernel_for (kernel_common.h).
#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"

namespace tg {
namespace {

// Objective and gradient (IpoptAdapter::eval_f / eval_grad_f): one block per problem. The block stages x
// and the node table in LDS; lanes take the cost work items round-robin (grouped by kind, so waves mostly
// run one path). f is reduced over the block in a fixed order. The gradient is deterministic: every call
// on the same x gives the same bits, whatever the scheduling of the block's waves.
//   ACC = kAccSlots (fixed phase durations): an item writes each present entry to its slot, the slots ordered
//     by column (Layout::cost_cslot, CostItem::cslot), then one lane per column sums the column's slots
//     [cost_cptr[j], cost_cptr[j + 1]) in order. Both tables are staged in LDS once per block: plain LDS
//     stores and loads, no atomics.
//   ACC = kAccLimbs (phase-duration optimisation: the PhaseSpline windows a sample touches move with x):
//     each entry is added as an exact fixed-point number v * 2^60 in three signed 42-bit limbs with
//     64-bit integer LDS atomics. Integer addition is associative, so the sums are order-independent;
//     a column's value is formed from its limbs once. Resolution 2^-60 (8.7e-19, far below the parity
//     floor of 1e-12); |v| >= 2^65 or a NaN / inf entry makes the whole gradient NaN.
//   ACC = kAccNone: f only.
// SoftConstraint terms add J^T (g - b) per column from the soft child's CSR values, in row order
// (towr_gpu.hip's column lists of the soft pattern).
enum { kAccNone = 0, kAccSlots = 1, kAccLimbs = 2 };

// Blocks are persistent (the host launches as many as fit the device at once, cost_grid): a block stages the
// node table and the slot tables once, then takes problems blockIdx.x, + gridDim.x, ...; the next problem's x
// is in flight (XStage registers) while the block evaluates the current one, and goes to LDS after it.
template <int ACC, bool GAIT, bool ROTVEC>
__global__ void __launch_bounds__(kCostBlock, 1) towr_cost_kernel(KParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* xs = smem + P.lds_x_off;         // [n_pad] x (+ zero slot at n), then the node table
  int32_t* ns = reinterpret_cast<int32_t*>(xs + P.n_pad);
  double* red = smem + P.lds_red_off;      // [kCostBlock / 64] per-wave partial objectives
  double* cs = smem;                       // kAccSlots: [cost_nslot] contributions
  unsigned long long* acc = reinterpret_cast<unsigned long long*>(smem);   // kAccLimbs: [3][n_pad]
  int* bad = reinterpret_cast<int*>(red + kCostBlock / 64);
  // kAccSlots: the slot tables after the node table (16-byte units: cost_cslot, then cost_cptr)
  uint16_t* cslot = reinterpret_cast<uint16_t*>(xs + P.n_pad + ((P.n_nodecol + 3) >> 2) * 2);
  const int n16s = (P.c_nslot + 7) >> 3;
  uint16_t* cptr = cslot + 8 * n16s;
  if constexpr (ACC == kAccSlots) {
    stage16<kCostBlock>(reinterpret_cast<uint4*>(cslot), reinterpret_cast<const uint4*>(P.c_cslot), n16s);
    stage16<kCostBlock>(reinterpret_cast<uint4*>(cptr), reinterpret_cast<const uint4*>(P.c_cptr), (P.n + 8) >> 3);
  }
  int b = blockIdx.x;
  const int G = gridDim.x;
  stage_x<kCostBlock, true>(P, P.X + (int64_t)b * P.ldx, xs, ns);
  Ctx c;
  c.x = xs; c.nodecol = ns; c.spl = P.spl; c.dur = P.dur;
  c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
  c.gait = GAIT; c.pinfo = P.pinfo; c.pcols = P.pcols; c.pact = P.pact; c.sched = P.sched; c.eelin = P.eelin; c.lin = P.lin;
  c.rotvec = ROTVEC;
  c.dyn_scratch = nullptr;
  c.cq = P.cq;
  XStage<kCostBlock, false> next;
  for (; b < P.B; b += G) {   // the same trip count for every thread of the block
    if constexpr (ACC == kAccLimbs) {
      for (int i = threadIdx.x; i < 3 * P.n_pad; i += kCostBlock) acc[i] = 0;
      if (threadIdx.x == 0) *bad = 0;
    }
    __syncthreads();   // x (and the tables, the cleared limbs) in LDS
    const int bn = b + G;
    if (bn < P.B) next.issue(P, P.X + (int64_t)bn * P.ldx);
    c.ter = P.terrains + (P.terrain_per_problem ? b : 0);
    double f = 0.0;
    for (int i = threadIdx.x; i < P.n_citems; i += kCostBlock) {
      const CostItem it = P.citems[i];
      c.seg = nullptr; c.sg = P.sg; c.row = it.seg;
      if constexpr (ACC == kAccSlots) {
        CostSlotEmit em{cs, cslot + it.cslot, P.n};
        eval_cost_item(c, it, em);
        f += em.f;
      } else if constexpr (ACC == kAccLimbs) {
        CostLimbEmit em{acc, P.n_pad, bad};
        eval_cost_item(c, it, em);
        f += em.f;
      } else {
        CostFEmit em;
        eval_cost_item(c, it, em);
        f += em.f;
      }
    }
    // SoftConstraint terms (soft_constraint.cc:52-69): 0.5 (g - b)^T (g - b); the gradient J^T (g - b) below
    const double* sgp = P.sG + (int64_t)b * P.s_ldg;
    for (int r = threadIdx.x; r < P.s_m; r += kCostBlock) {
      const double d = sgp[r] - P.s_b[r];
      f += (0.5 * d) * d;
    }
    // f: wave butterfly, then the waves' partials in order
    for (int o = 32; o > 0; o >>= 1) f += __shfl_xor(f, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = f;
    __syncthreads();   // partials, and every gradient entry, in LDS
    if (threadIdx.x == 0) {
      double sf = 0.0;
      for (int w = 0; w < kCostBlock / 64; ++w) sf += red[w];
      P.F[b] = sf;
    }
    if constexpr (ACC != kAccNone) {
      double* gr = P.GR + (int64_t)b * P.ldgr;
      const double* sv = P.sV + (int64_t)b * P.s_ldv;
      const bool nan_all = ACC == kAccLimbs && *bad != 0;
      for (int j = threadIdx.x; j < P.n; j += kCostBlock) {
        double s = 0.0;
        if constexpr (ACC == kAccSlots) {
          // (round 6, ANYmal + every cost kind, B = 4096, one box: 0.1306 ms per batch; slots in item order with the
          // column reading its slot ids 0.1324; the item's slot ids from global memory instead of LDS 0.1554)
          const int k1 = cptr[j + 1];
          int k = cptr[j];
          for (; k + 4 <= k1; k += 4) {   // 4 loads in flight together; the sum stays in order
            const double a0 = cs[k], a1 = cs[k + 1], a2 = cs[k + 2], a3 = cs[k + 3];
            s += a0; s += a1; s += a2; s += a3;
          }
          for (; k < k1; ++k) s += cs[k];
        } else {
          s = limb_value((long long)acc[j], (long long)acc[P.n_pad + j], (long long)acc[2 * P.n_pad + j]);
          if (nan_all) s = __builtin_nan("");
        }
        if (P.s_m > 0)   // the soft child's column j, its rows in order
          for (int k = P.s_cptr[j]; k < P.s_cptr[j + 1]; ++k) {
            const int2 e = P.s_cent[k];   // (CSR index, row)
            s += sv[e.x] * (sgp[e.y] - P.s_b[e.y]);
          }
        __builtin_nontemporal_store(s, gr + j);
      }
    }
    __syncthreads();   // every lane is done with this problem's x, slots and partials
    if (bn < P.B) next.commit(P, P.X + (int64_t)bn * P.ldx, xs, ns);
  }
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

template <int ACC, bool GAIT>
const void* cost_kernel_rv(bool rotvec) {
  return rotvec ? reinterpret_cast<const void*>(&towr_cost_kernel<ACC, GAIT, true>)
                : reinterpret_cast<const void*>(&towr_cost_kernel<ACC, GAIT, false>);
}
// acc: 0 f only, 1 gradient through slots (fixed phase durations only), 2 gradient through limbs
const void* cost_kernel_for(bool gait, int acc, bool rotvec) {
  if (gait) return acc ? cost_kernel_rv<kAccLimbs, true>(rotvec) : cost_kernel_rv<kAccNone, true>(rotvec);
  return acc == 1 ? cost_kernel_rv<kAccSlots, false>(rotvec) : acc == 2 ? cost_kernel_rv<kAccLimbs, false>(rotvec)
                  : cost_kernel_rv<kAccNone, false>(rotvec);
}

const void* traj_kernel_for(bool gait) {
  return gait ? reinterpret_cast<const void*>(&towr_traj_kernel<true>) : reinterpret_cast<const void*>(&towr_traj_kernel<false>);
}

}  // namespace tg
