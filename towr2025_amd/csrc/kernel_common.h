// kernel_common.h — device-side definitions shared by the engine's translation units
// (tiles.hip: tile / small-kind / fused kernels; gstream.hip: the phase-duration path's record and
// compose kernels; cost_traj.hip; towr_gpu.hip: the C-ABI): the launch parameter block and the staging
// and copy-out helpers.
#pragma once

#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "layout.h"

namespace tg {

// one unit of the fused launch: a tile of a tile class, or a small-kind group (LC_MISC)
// a fused launch's unit: its class, tile (with a copy of the tile's descriptor, so a block's first load level holds it)
// and LDS offsets
struct UnitDesc {
  int32_t lc, tile, lds_x_off, lds_rows_off;
  TileDesc t;
};

struct KParams {
  const double* X; int64_t ldx;
  double* G; int64_t ldg;
  double* V; int64_t ldv;
  const ItemDesc* items;
  const SlotGroup* slots;
  const TileDesc* tiles;
  const int32_t* nodecol;
  const SplineMeta* spl;
  const double* dur;
  SegSoA sg;                     // segment table (structure of arrays)
  const PolyPhase* pinfo;        // phase-duration optimisation tables (see engine_math.h)
  const PhaseCol* pcols;
  const int32_t* pact;
  const SchedInfo* sched;
  const EELinDef* eelin;
  const LinNz* lin;              // LinearEqualityConstraint rows
  const uint4* gtab;             // GAIT: the PhaseSpline tables in one blob (GaitTables), staged per tile block
  const ItemDirect* idir;        // GAIT: per item (lane) direct-position ranges
  int32_t gt_off[5], gt_n16;
  int32_t n_pinfo, ph_stride;    // GAIT: the block's PhaseSpline timings (Ctx::pdur / pend / phend)
  int32_t gt_ntime;              // GAIT: doubles of those timings (the terrain's LDS copy follows them)
  int32_t n_spl;
  const towr_terrain_t* terrains;
  int32_t terrain_per_problem;
  int32_t B, tile0, ntiles;
  int32_t lds_rows_off;          // start of the g buffer in the dynamic LDS (doubles)
  int32_t lds_x_off;             // start of the staged x (+ zero slot) and node-column table
  int32_t lds_scr_off;           // DYN: per-instant endeffector sum terms (instants x n_ee x 6)
  double* rvc;                   // DYN, fixed gait, RotVec: the pre-pass's base-angular coefficients (kRvCoef per instant)
  const RvInst* rvi;             // ... and its instants (n_rvi per problem)
  int32_t n_rvi;
  int32_t n, n_pad, n_nodecol;
  int32_t want_g, want_jac, fdisc_motion;
  const int32_t* misc_tiles;      // merged small-kind launch: kMiscWaves tile ids per group
  const int32_t* misc_lds;        // per (group, wave): LDS offset, g-row offset
  const MiscWave* misc_wave;      // per (group, wave): the tile's ranges and LDS offsets (layout.h MiscWave)
  const ItemDesc* misc_items;     // per (group, wave, lane): the tile's items
  const int32_t* xspan;           // the small kinds' x spans (Layout::misc_xspan), n_xspan pairs; 0 = all of x
  int32_t n_xspan;
  RobotC rb;
  const UnitDesc* units;          // fused launch: a problem's units (UnitDesc), n_units per problem
  int32_t n_units;
  const FsBlock* fsb;             // streaming ForceConstraintDiscretized (layout.h FsBlock)
  const double* fs_t;
  const int32_t* fs_tmpl;
  const int32_t* fs_ws;
  const int32_t* fs_iee;          // per FDISC instant: endeffector, first g row
  const int32_t* fs_irow;
  const int32_t* fs_iblk;
  const GsGeo* gs_geo;            // streaming RangeOfMotion / Dynamic (layout.h GsGeo)
  const GsBlock* gs_blk;          // the launched class's compose blocks
  const int32_t* gs_tmpl;
  const uint8_t* gs_pcode;
  const GsSeg* gs_segs;
  const uint8_t* gs_tseg;
  const uint32_t* gs_vmap;
  const int16_t* gs_ws;
  const uint4* gs_blob;
  const CostItem* citems;         // cost launch: work items, objective and gradient outputs
  const double* cq;               // cost launch: CT_ENERGYQ Gram matrices
  int32_t n_citems, lds_red_off;
  const uint16_t* c_cptr;         // cost launch, slot gradient (Layout::cost_cptr / cost_cslot, padded to 16 bytes)
  const uint16_t* c_cslot;
  int32_t c_nslot;
  double* F;
  double* GR; int64_t ldgr;
  // cost launch, SoftConstraint terms: the soft child's g (and CSR values) of this batch, its CSR
  // pattern, b = the bounds' mid-points; s_m = 0 without soft terms
  const double* sG; int64_t s_ldg;
  const double* sV; int64_t s_ldv;
  const double* s_b;
  int32_t s_m;
  const int32_t* s_cptr;          // the soft pattern by column: entries s_cent[s_cptr[j] .. s_cptr[j + 1]) =
  const int2* s_cent;             // (CSR index, row), rows ascending
  // experiment build only (-DTOWR_STAMPS, tools/stamps.py): per-block timestamp slots of this launch, or null
  unsigned long long* stamps;
};

// In-kernel phase timestamps of the experiment build (make variant VFLAGS=-DTOWR_STAMPS): lane 0 of each wave
// stores the 100 MHz real-time counter into slot k of its wave (64 slots per block: 8 waves x 8 phases); the
// product build compiles them out.
#ifdef TOWR_STAMPS
#define TG_STAMP(P, k)                                                                                              \
  do {                                                                                                              \
    if ((P).stamps && (threadIdx.x & 63) == 0 && threadIdx.x < 512)                                                 \
      (P).stamps[(size_t)blockIdx.x * 64 + (threadIdx.x >> 6) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
#else
#define TG_STAMP(P, k) do { } while (0)
#endif

// global -> LDS copy of n16 16-byte units: each thread issues up to K independent loads before its
// first LDS write, so the staging costs one memory latency rather than one per loop trip
// (BLOCK 0: the launch's block size, blockDim.x)
template <int BLOCK>
__device__ __forceinline__ void stage16(uint4* __restrict__ dst, const uint4* __restrict__ src, int n16) {
  const int S = BLOCK > 0 ? BLOCK : (int)blockDim.x;
  for (int i = threadIdx.x; i < n16; i += 4 * S) {   // 4 loads in flight per thread
    const int i1 = i + S, i2 = i + 2 * S, i3 = i + 3 * S;
    const uint4 r0 = src[i];
    uint4 r1{}, r2{}, r3{};
    if (i1 < n16) r1 = src[i1];
    if (i2 < n16) r2 = src[i2];
    if (i3 < n16) r3 = src[i3];
    dst[i] = r0;
    if (i1 < n16) dst[i1] = r1;
    if (i2 < n16) dst[i2] = r2;
    if (i3 < n16) dst[i3] = r3;
  }
}

// LDS -> HBM, 16-byte non-temporal stores where the destination allows it. The outputs are
// streamed (never re-read by the kernel); plain stores cost ~25 % more kernel time on MI355X
// (ANYmal, B = 4096: 0.532 -> 0.444 ms per step with non-temporal stores).
typedef double dbl2_t __attribute__((ext_vector_type(2)));
// 16-byte units of a destination before its next 1 KB boundary: a stream loop whose lanes start at unit -skew (skipping
// the negative units) issues every wave's 64 x 16-byte store on one whole 1 KB of HBM. TOWR_ALIGN_TRIPS: the loops that
// align (bit 0 the FDISC composer, 1 the RangeOfMotion / Dynamic / TQDISC composer, 2 the tile copy-out, 3 the TQDISC
// composer). tools/stride_probe.hip, the FDISC composer's pattern as pure stores: 4.2 -> 5.4 TB/s. In the kernels
// (MI355X, ANYmal gait, B = 1024, one box, 3 runs, ms per step gait / + Torque): none 0.613-0.622 / 1.168-1.169; the
// FDISC composer 0.591-0.605 / 1.163-1.167; the other composers 0.616-0.621 / 1.159-1.163; both 0.596-0.616 /
// 1.195-1.196; every loop incl. the tile copy-out: the headline step 0.2355-0.2364 -> 0.2399-0.2408 ms (B = 4096).
#ifndef TOWR_ALIGN_TRIPS
#define TOWR_ALIGN_TRIPS 1
#endif
template <int LOOP>
__device__ __forceinline__ int trip_skew(const void* d2) {
  if constexpr (((TOWR_ALIGN_TRIPS >> LOOP) & 1) != 0) return (int)((reinterpret_cast<uintptr_t>(d2) & 1023) >> 4);
  (void)d2;
  return 0;
}
__device__ __forceinline__ void copy_out(const double* __restrict__ src, double* __restrict__ dst, int n,
                                         int tid, int nthr) {
  if (n <= 0) return;
  const int head = (reinterpret_cast<uintptr_t>(dst) & 15) ? 1 : 0;
  if (head && tid == 0) __builtin_nontemporal_store(src[0], dst);
  const int m = (n - head) >> 1;
  dbl2_t* d2 = reinterpret_cast<dbl2_t*>(dst + head);
  const int k = trip_skew<2>(d2);
  for (int i = tid - k; i < m; i += nthr) {
    if (i < 0) continue;
    dbl2_t v;
    v.x = src[head + 2 * i];
    v.y = src[head + 2 * i + 1];
    __builtin_nontemporal_store(v, d2 + i);
  }
  if (((n - head) & 1) && tid == 0) __builtin_nontemporal_store(src[n - 1], dst + n - 1);
}

// Split staging: issue() puts the first K 16-byte units per thread of x (and the node table) in
// flight before the block's item / slot-table loads, commit() stores them to LDS afterwards, so the
// staging's memory latency overlaps the item loads instead of following them. Units beyond K per
// thread (problems larger than the bench's) go through stage16 in commit().
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <int BLOCK, bool NODES>
struct XStage {
  static constexpr int K = 3;   // named native-vector registers (HIP's uint4 class or an array goes to scratch)
  u32x4_t x0 = {}, x1 = {}, x2 = {}, n0 = {}, n1 = {}, n2 = {};
  bool aligned;
  __device__ __forceinline__ void issue(const KParams& P, const double* xg) {
    aligned = (reinterpret_cast<uintptr_t>(xg) & 15) == 0;
    const int nx = P.n >> 1, i = threadIdx.x;
    const u32x4_t* sx = reinterpret_cast<const u32x4_t*>(xg);
    if (aligned) {
      if (i < nx) x0 = sx[i];
      if (i + BLOCK < nx) x1 = sx[i + BLOCK];
      if (i + 2 * BLOCK < nx) x2 = sx[i + 2 * BLOCK];
    }
    if constexpr (NODES) {
      const int nn = (P.n_nodecol + 3) >> 2;
      const u32x4_t* sn = reinterpret_cast<const u32x4_t*>(P.nodecol);
      if (i < nn) n0 = sn[i];
      if (i + BLOCK < nn) n1 = sn[i + BLOCK];
      if (i + 2 * BLOCK < nn) n2 = sn[i + 2 * BLOCK];
    }
  }
  __device__ __forceinline__ void commit(const KParams& P, const double* xg, double* xs, int32_t* ns) {
    const int nx = P.n >> 1, i = threadIdx.x;
    if (aligned) {
      u32x4_t* dx = reinterpret_cast<u32x4_t*>(xs);
      if (i < nx) dx[i] = x0;
      if (i + BLOCK < nx) dx[i + BLOCK] = x1;
      if (i + 2 * BLOCK < nx) dx[i + 2 * BLOCK] = x2;
      if (nx > K * BLOCK)
        stage16<BLOCK>(reinterpret_cast<uint4*>(xs) + K * BLOCK, reinterpret_cast<const uint4*>(xg) + K * BLOCK, nx - K * BLOCK);
      if ((P.n & 1) && threadIdx.x == 0) xs[P.n - 1] = xg[P.n - 1];
    } else {
      for (int k = threadIdx.x; k < P.n; k += BLOCK) xs[k] = xg[k];
    }
    if (threadIdx.x == 0) xs[P.n] = 0.0;
    if constexpr (NODES) {
      const int nn = (P.n_nodecol + 3) >> 2;
      u32x4_t* dn = reinterpret_cast<u32x4_t*>(ns);
      if (i < nn) dn[i] = n0;
      if (i + BLOCK < nn) dn[i + BLOCK] = n1;
      if (i + 2 * BLOCK < nn) dn[i + 2 * BLOCK] = n2;
      if (nn > K * BLOCK)
        stage16<BLOCK>(reinterpret_cast<uint4*>(ns) + K * BLOCK, reinterpret_cast<const uint4*>(P.nodecol) + K * BLOCK, nn - K * BLOCK);
    }
  }
};

// Zero-fill of a GAIT tile's CSR range in HBM by its own block (TileEmit DIRECT), 16-byte stores.
// Plain stores: the scattered value stores that follow then mostly hit the same lines in L2.
__device__ __forceinline__ void zero_out(double* __restrict__ dst, int n, int tid, int nthr) {
  if (n <= 0) return;
  const int head = (reinterpret_cast<uintptr_t>(dst) & 15) ? 1 : 0;
  if (head && tid == 0) dst[0] = 0.0;
  const int m = (n - head) >> 1;
  dbl2_t* d2 = reinterpret_cast<dbl2_t*>(dst + head);
  const dbl2_t z = {0.0, 0.0};
  for (int i = tid; i < m; i += nthr) d2[i] = z;
  if (((n - head) & 1) && tid == 0) dst[n - 1] = 0.0;
}

// zero n doubles of LDS (16-byte stores; n rounded up to even, the tile regions are even-sized)
__device__ __forceinline__ void zero_lds(double* d, int n, int tid, int nthr) {
  dbl2_t* d2 = reinterpret_cast<dbl2_t*>(d);
  const dbl2_t z = {0.0, 0.0};
  for (int i = tid; i < (n + 1) >> 1; i += nthr) d2[i] = z;
}

// global -> LDS staging of the problem's x (+ zero slot at n) and optionally the node table
template <int BLOCK, bool NODES>
__device__ __forceinline__ void stage_x(const KParams& P, const double* xg, double* xs, int32_t* ns) {
  if ((reinterpret_cast<uintptr_t>(xg) & 15) == 0) {
    stage16<BLOCK>(reinterpret_cast<uint4*>(xs), reinterpret_cast<const uint4*>(xg), P.n >> 1);
    if ((P.n & 1) && threadIdx.x == 0) xs[P.n - 1] = xg[P.n - 1];
  } else {
    for (int i = threadIdx.x; i < P.n; i += (BLOCK > 0 ? BLOCK : (int)blockDim.x)) xs[i] = xg[i];
  }
  if (threadIdx.x == 0) xs[P.n] = 0.0;
  if constexpr (NODES)
    stage16<BLOCK>(reinterpret_cast<uint4*>(ns), reinterpret_cast<const uint4*>(P.nodecol), (P.n_nodecol + 3) >> 2);
}

// stage_x over the 16-byte spans of x in P.xspan (Layout::misc_xspan) when there are any: the small kinds read
// only the base and foot-motion nodes, about half of x (with the zero slot and the node table)
template <int BLOCK>
__device__ __forceinline__ void stage_x_spans(const KParams& P, const double* xg, double* xs, int32_t* ns) {
  if (P.n_xspan == 0 || (reinterpret_cast<uintptr_t>(xg) & 15) != 0) {
    stage_x<BLOCK, true>(P, xg, xs, ns);
    return;
  }
  // one pass when the spans' 16-byte units fit 3 per thread: every thread's units of the spans' concatenation and of
  // the node table in flight together, then their LDS stores (one memory latency; span by span it was one per span:
  // tools/stamps.py, MI355X, ANYmal, B = 4096: 2.8-3.6 us of a 5.8-6.6 us block). The unit holding x[n - 1] of an odd
  // n is one double (thread 0).
  const int nx = P.n >> 1, tid = (int)threadIdx.x;
  int u0 = -1, u1 = -1, u2 = -1, acc = 0;
  bool tail = false;
  for (int k = 0; k < P.n_xspan; ++k) {
    const int a = P.xspan[2 * k], l = P.xspan[2 * k + 1];
    tail = tail || 2 * (a + l) > P.n;
    const int len = min(l, nx - a);
    if (len <= 0) continue;
    const int j0 = tid - acc;
    if ((unsigned)j0 < (unsigned)len) u0 = a + j0;
    if ((unsigned)(j0 + BLOCK) < (unsigned)len) u1 = a + j0 + BLOCK;
    if ((unsigned)(j0 + 2 * BLOCK) < (unsigned)len) u2 = a + j0 + 2 * BLOCK;
    acc += len;
  }
  const int nn = (P.n_nodecol + 3) >> 2;
  // (a host-built table of every thread's units instead of the walk over the span list: 23.9 vs 23.2 us per 4096
  // problems, not kept)
  if (acc <= 3 * BLOCK) {
    const u32x4_t* sx = reinterpret_cast<const u32x4_t*>(xg);
    const u32x4_t* sn = reinterpret_cast<const u32x4_t*>(P.nodecol);
    u32x4_t x0 = {}, x1 = {}, x2 = {}, n0 = {}, n1 = {}, n2 = {};
    double xt = 0.0;
    if (u0 >= 0) x0 = sx[u0];
    if (u1 >= 0) x1 = sx[u1];
    if (u2 >= 0) x2 = sx[u2];
    if (tail && tid == 0) xt = xg[P.n - 1];
    if (tid < nn) n0 = sn[tid];
    if (tid + BLOCK < nn) n1 = sn[tid + BLOCK];
    if (tid + 2 * BLOCK < nn) n2 = sn[tid + 2 * BLOCK];
    u32x4_t* dx = reinterpret_cast<u32x4_t*>(xs);
    u32x4_t* dn = reinterpret_cast<u32x4_t*>(ns);
    if (u0 >= 0) dx[u0] = x0;
    if (u1 >= 0) dx[u1] = x1;
    if (u2 >= 0) dx[u2] = x2;
    if (tid == 0) {
      if (tail) xs[P.n - 1] = xt;
      xs[P.n] = 0.0;
    }
    if (tid < nn) dn[tid] = n0;
    if (tid + BLOCK < nn) dn[tid + BLOCK] = n1;
    if (tid + 2 * BLOCK < nn) dn[tid + 2 * BLOCK] = n2;
    if (nn > 3 * BLOCK) stage16<BLOCK>(reinterpret_cast<uint4*>(ns) + 3 * BLOCK, reinterpret_cast<const uint4*>(P.nodecol) + 3 * BLOCK, nn - 3 * BLOCK);
    return;
  }
  for (int k = 0; k < P.n_xspan; ++k) {
    const int a = P.xspan[2 * k], len = P.xspan[2 * k + 1];
    if (2 * (a + len) <= P.n) {
      stage16<BLOCK>(reinterpret_cast<uint4*>(xs) + a, reinterpret_cast<const uint4*>(xg) + a, len);
    } else {   // the last unit of an odd n: its first double only
      stage16<BLOCK>(reinterpret_cast<uint4*>(xs) + a, reinterpret_cast<const uint4*>(xg) + a, len - 1);
      if (threadIdx.x == 0) xs[P.n - 1] = xg[P.n - 1];
    }
  }
  if (threadIdx.x == 0) xs[P.n] = 0.0;
  stage16<BLOCK>(reinterpret_cast<uint4*>(ns), reinterpret_cast<const uint4*>(P.nodecol), nn);
}

// The x-dependent PhaseSpline timings of one problem (phase_spline_timings / phase_end_timings: pdur, pend per
// polynomial, phend per (endeffector, phase)) by the whole block: (1) each endeffector's last phase duration,
// parked in its phend slot; (2) one thread per polynomial forms its duration (the divisions in parallel; the entry's
// spline from PolyPhase::spl); (3) one thread per spline / endeffector forms the running sums in the reference's order,
// its operands loaded 8 at a time ahead of the dependent additions. Every value is the one thread-per-spline loop's
// (same operations, same order). MI355X, ANYmal gait, B = 1024 (tools/stamps.py): this prologue took 5.3 us of a
// 27 us record block with a per-entry scan over the splines and one LDS round trip per running-sum step.
__device__ __forceinline__ void phase_timings_block(const Ctx& c, const KParams& P, double* tm) {
  double* pdur = tm;
  double* pend = tm + P.n_pinfo;
  double* phend = tm + 2 * P.n_pinfo;
  const int tid = threadIdx.x, nspl = P.n_spl, nee = P.rb.n_ee;
  if (tid < nee) {
    const SchedInfo si = c.sched[tid];
    if (si.col0 >= 0) phend[tid * P.ph_stride + si.n_phases - 1] = last_phase_duration(c, si);
  }
  __syncthreads();
  for (int i = tid; i < P.n_pinfo; i += blockDim.x) {
    const SplineMeta m = c.spl[c.pinfo[i].spl];
    const SchedInfo si = c.sched[m.ee];
    const double last = si.col0 >= 0 ? phend[m.ee * P.ph_stride + si.n_phases - 1] : last_phase_duration(c, si);
    pdur[i] = phase_poly_duration(c, m, si, last, i - m.pinfo_off);
  }
  __syncthreads();
  // running sums t += d[i] in order; the loads of a group of 8 issue together
  auto running = [](const double* d, double* out, int n, double t) {
    for (int i0 = 0; i0 < n; i0 += 8) {
      double v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = i0 + k < n ? d[i0 + k] : 0.0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (i0 + k < n) { t += v[k]; out[i0 + k] = t; }
    }
  };
  if (tid < nspl) {
    const SplineMeta m = c.spl[tid];
    if (m.ee >= 0) running(pdur + m.pinfo_off, pend + m.pinfo_off, m.n_polys, 0.0);
  } else if (tid < nspl + nee) {
    const int ee = tid - nspl;
    const SchedInfo si = c.sched[ee];
    if (si.col0 >= 0) {
      // phase_duration: the schedule variables x[col0 ..], then the last phase (parked in ph[n - 1] by step 1)
      double* ph = phend + ee * P.ph_stride;
      const double last = ph[si.n_phases - 1];
      double acc = 0.0;
      for (int k0 = 0; k0 < si.n_phases; k0 += 8) {
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = k0 + k < si.n_phases ? phase_duration(c, si, last, k0 + k) : 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (k0 + k < si.n_phases) { acc += v[k]; ph[k0 + k] = acc; }
      }
    }
  }
  __syncthreads();
}

// Prologue of the per-problem record kernel under phase-duration optimisation (gstream.hip): x (+ zero slot), the node table, the PhaseSpline tables and the terrain staged in LDS
// ([x | node table | tables | timings | terrain], fs_inst_lds_bytes), then the x-dependent PhaseSpline
// timings formed once per block (as tile_body does); returns the evaluation context over them.
template <int BLOCK>
__device__ __forceinline__ Ctx gait_record_setup(const KParams& P, int b, double* smem) {
  const double* xg = P.X + (int64_t)b * P.ldx;
  double* xs = smem;
  int32_t* ns = reinterpret_cast<int32_t*>(xs + P.n_pad);
  char* gt = reinterpret_cast<char*>(xs + P.n_pad + ((P.n_nodecol + 3) >> 2) * 2);
  towr_terrain_t* ters = reinterpret_cast<towr_terrain_t*>(gt + 16 * P.gt_n16 + 8 * P.gt_ntime);
  const int tid = threadIdx.x;
  TG_STAMP(P, 0);
  stage_x<BLOCK, true>(P, xg, xs, ns);
  stage16<BLOCK>(reinterpret_cast<uint4*>(gt), P.gtab, P.gt_n16);
  if (tid < (int)(sizeof(towr_terrain_t) / 8))
    reinterpret_cast<double*>(ters)[tid] = reinterpret_cast<const double*>(P.terrains + (P.terrain_per_problem ? b : 0))[tid];
  __syncthreads();
  Ctx c;
  c.seg = nullptr; c.sg = P.sg; c.row = -1;
  c.x = xs; c.nodecol = ns; c.dur = P.dur;
  c.ter = ters;
  c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
  c.gait = true; c.eelin = P.eelin; c.lin = P.lin;
  c.spl = reinterpret_cast<const SplineMeta*>(gt + P.gt_off[0]);
  c.sched = reinterpret_cast<const SchedInfo*>(gt + P.gt_off[1]);
  c.pinfo = reinterpret_cast<const PolyPhase*>(gt + P.gt_off[2]);
  c.pact = reinterpret_cast<const int32_t*>(gt + P.gt_off[3]);
  c.pcols = reinterpret_cast<const PhaseCol*>(gt + P.gt_off[4]);
  c.rotvec = false;
  c.dyn_scratch = nullptr;
  double* tmg = reinterpret_cast<double*>(gt + 16 * P.gt_n16);
  TG_STAMP(P, 1);
  phase_timings_block(c, P, tmg);
  TG_STAMP(P, 2);
  c.pdur = tmg; c.pend = tmg + P.n_pinfo; c.phend = tmg + 2 * P.n_pinfo; c.ph_stride = P.ph_stride;
  return c;
}

// Kernels of the other translation units, for the host side (towr_gpu.hip): tiles.hip (tile, small-kind
// and fused kernels), cost_traj.hip (objective, trajectory export)
const void* tile_kernel_for(int type, bool gait, bool rotvec);
const void* misc_kernel_for(bool gait);
const void* step_kernel_for(bool gait, bool rotvec, int kblock);
const void* cost_kernel_for(bool gait, int acc, bool rotvec);   // acc: 0 f only, 1 slots, 2 limbs
const void* traj_kernel_for(bool gait);
const void* rv_coef_kernel();
constexpr int kRvCoefBlock = 256;   // the RotVec coefficient pre-pass: 4 waves, one component each
// objective kernel: persistent blocks of 256 threads, one problem at a time per block (Layout's wave schedule of
// the cost items assumes kCostLanes threads). (512-thread blocks, one per CU with the CU's whole LDS: 0.179 vs 0.130
// ms per 4096 problems.)
constexpr int kCostBlock = kCostLanes;
constexpr int kTrajBlock = 64;    // trajectory kernel: one block per (problem, 64 sample times)

// The heavy kinds read spline nodes through the segment records; with phase-duration optimisation
// (GAIT) their PhaseSplines evaluate polynomials from the node table, which is then staged too.
constexpr bool stages_nodes(int type, bool gait) { return gait || is_misc_kind(type); }
// Split staging (XStage: x loads issued before the item / slot loads) where it measured faster on
// MI355X (ANYmal, B = 4096): Dynamic 0.0617 -> 0.0582 ms, ForceConstraintDiscretized 0.1018 ->
// 0.098 ms; RangeOfMotion got slower (0.0838 -> 0.0878 ms) and the small kinds were unchanged, so
// they stage after their item loads as before.
constexpr bool early_stage(int type) { return type == IT_DYN || type == IT_FDISC; }

}  // namespace tg
