// tiles.hip — the tile kernels of the eval_g / eval_jac_g engine (include/towr_gpu.h):
// one block per (problem, tile) of a constraint class, the merged small-kind launch and the fused
// launch of several classes (towr_step_kernel). The host side (towr_gpu.hip) reaches them through the
// getters at the end of this file (kernel_common.h).
//   * block = (problem, group of LDS tiles); blocks of one problem are placed on one XCD
//     (blockIdx % 8 round-robin), so x is fetched from HBM once per problem;
//   * the problem's x (NodesVariables / PhaseDurations values) is staged in LDS;
//   * a tile = consecutive instances of one constraint set whose CSR value range fits in LDS;
//     lanes evaluate work items (node-per-lane Hermite splines, SRBD, terrain) and accumulate
//     Jacobian candidates into LDS at precomputed slots; then the tile's contiguous CSR range and
//     g range are written with 16-byte coalesced stores.
// No MFMA: there is no dense contraction; the kernels are HBM-write bound.
#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"
#include "tile_emit.h"

namespace tg {
constexpr int kMiscMinWaves = 5;   // small kinds: minimum waves per SIMD (0.0267 -> 0.0257 ms per 4096 problems, A/B on one box)
namespace {


// Emitter for a fixed stretch of a lane's candidates J0 .. J0 + 8 NG - 1 whose slot groups are all
// loaded at construction: Dynamic group 0 builds it before the block barrier that separates its two
// phases, so phase B's slot loads complete during the barrier wait instead of once per 8 candidates
// after it. Candidate indices must be compile-time constants (fully unrolled emission).
template <int BLOCK, int J0, bool DIRECT = false>
struct TileEmitPre {   // four groups: candidates J0 - J0 % 8 .. + 31
  double* out;
  double* gout;
  int nvals = 0;   // DIRECT (see TileEmit): out / gout are V and g in HBM, dummy slots are not stored
  bool gon = true;
  SlotGroup q0, q1, q2, q3;   // named registers (a runtime-indexed array would go to scratch)
  int j = J0;
  __device__ __forceinline__ TileEmitPre(const SlotGroup* s, double* o, double* go, bool load) : out(o), gout(go) {
    if (load) {
      q0 = s[(J0 >> 3) * BLOCK]; q1 = s[((J0 >> 3) + 1) * BLOCK];
      q2 = s[((J0 >> 3) + 2) * BLOCK]; q3 = s[((J0 >> 3) + 3) * BLOCK];
    }
  }
  __device__ __forceinline__ void g(int row, double v) {   // gon: g requested (LDS rows: always on)
    if (gon) gout[row] = v;
  }
  __device__ __forceinline__ void operator()(int, int, double v, bool) {
    const int k = (j >> 3) - (J0 >> 3);
    SlotGroup q;
#pragma unroll
    for (int w = 0; w < 4; ++w) q.w[w] = k == 0 ? q0.w[w] : k == 1 ? q1.w[w] : k == 2 ? q2.w[w] : q3.w[w];
    const int s = slot_pick(q, j & 7);
    ++j;
    if (!DIRECT || s < nvals) out[s] = v;
  }
  __device__ __forceinline__ void flush() {}
};
static_assert(kDynG0Cand - (kDynG0PhaseA - kDynG0PhaseA % 8) <= 32, "phase B of Dynamic group 0 exceeds the preloaded groups");

// Slot-group prefetch depth. Deeper rings only pay off where the emission index is a compile-time
// constant: in a runtime loop, rotating the ring copies registers whose loads are still in flight
// and waits for the newest one (measured: depth 4 made RangeOfMotion's base-angular wave slower).
constexpr int slot_depth(int) { return 2; }
static_assert(slot_depth(IT_ROM) <= kSlotSpare, "slot prefetch past the spare groups");

// Slot groups preloaded by the gait (DIRECT) emitter per tile class: RangeOfMotion's base lanes emit
// 33-36 slot-path candidates each (5 groups); Dynamic's kernel is at 256 VGPRs already (more spills)
constexpr int gait_slot_pre(int type) { return type == IT_ROM ? 6 : 1; }

template <int TYPE, class Emit>
__device__ __forceinline__ void eval_typed(const Ctx& c, const ItemDesc& it, Emit& em) {
  if constexpr (TYPE == IT_DYN) eval_dyn(c, it, em);
  else if constexpr (TYPE == IT_ROM) eval_rom(c, it, em);
  else if constexpr (TYPE == IT_FDISC) eval_fdisc(c, it, em);
  else if constexpr (TYPE == IT_FNODE) eval_fnode(c, it, em);
  else if constexpr (TYPE == IT_TERR) eval_height(c, it, sp_motion(it.ee), 0.0, em);
  else if constexpr (TYPE == IT_BMOT) eval_bmot(c, it, em);
  else if constexpr (TYPE == IT_SACC) eval_sacc(c, it, em);
  else if constexpr (TYPE == IT_BHGT) eval_height(c, it, SP_BASE_LIN, it.p0, em);
  else if constexpr (TYPE == IT_SWING) eval_swing(c, it, em);
  else if constexpr (TYPE == IT_TDUR) eval_tdur(c, it, em);
  else if constexpr (TYPE == IT_TQDISC) eval_tqdisc(c, it, em);
}

// One block = one tile (consecutive instances of one constraint kind) of one problem; one item per
// thread, laid out so every wave runs a single code path. Blocks of one problem share an XCD (the
// mapping below), so its ~9 KB x is fetched from HBM once and then served by that XCD's L2.
// Candidates land in an LDS tile (no global store before the end, so no load ever waits behind a
// store: gfx950's vmcnt counts both); the tile's contiguous CSR range and g rows then leave with
// 16-byte coalesced stores. Every kernel stages the problem's x in LDS (spline items gather their
// nodes through the segment record's columns); node-value kinds also stage the node->column table.



// Body of one tile block. TBLOCK = the tile's lane count (its slot-table stride), KBLOCK = the
// launch's block size (>= TBLOCK): in the fused launch a 192-lane tile runs in a 256-thread block,
// whose extra wave only helps stage x and copy out.
template <int TYPE, int TBLOCK, int KBLOCK, bool GAIT, bool ROTVEC>
// (T by value: a reference into global memory is reloaded after the tile's stores, and on gfx950 such a load waits for them)
__device__ __forceinline__ void tile_body(const KParams& P, double* smem, int b, const TileDesc T, int lds_x_off, int lds_rows_off) {
  TG_STAMP(P, 0);
  double* Vb = P.V + (int64_t)b * P.ldv;
  double* Gb = P.G + (int64_t)b * P.ldg;
  const double* xg = P.X + (int64_t)b * P.ldx;
  // issue the lane's item, first slot groups and (below) the x / node-table staging loads together
  // x (+ a zero at index n for constant node values) and, for node-value kinds, the node table:
  // loads in flight first, then the lane's item and slot groups, then the LDS stores
  XStage<KBLOCK, stages_nodes(TYPE, GAIT)> xst;
  if constexpr (early_stage(TYPE)) xst.issue(P, xg);
  ItemDesc it;
  // (the slot address from the tile descriptor, base + lane, instead of the item: no gain, MI355X, ANYmal, B = 4096,
  // one box: 0.2381-0.2394 vs 0.2381-0.2389 ms per step; for the small kinds 25.8 vs 23.2 us)
  if (KBLOCK == TBLOCK || (int)threadIdx.x < TBLOCK) {
    it = P.items[T.i0 + threadIdx.x];
  } else {
    it = ItemDesc{}; it.type = IT_NONE; it.slot = 0;
  }
  // GAIT: direct HBM emission into the zero-filled V (see TileEmit)
  // fixed gait, RotVec Dynamic: eval_dyn never takes group 1 (the pre-pass coefficients, kRvPre)
  // fixed-gait Dynamic writes its g rows (group 0, phase B: 6 complete rows per instant, after every load) straight to
  // HBM: without the LDS rows the block fits three per CU at <= 168 VGPRs (layout.hip, the Dynamic LDS)
  constexpr bool kGDirect = TYPE == IT_DYN && !GAIT;
  TileEmit<TBLOCK, slot_depth(TYPE), GAIT, gait_slot_pre(TYPE), (TYPE == IT_DYN && ROTVEC && !GAIT) ? 1 : 0> em(
      P.slots + it.slot, GAIT ? Vb + T.v0 : smem, GAIT || kGDirect ? Gb : smem + lds_rows_off - T.r0);
  if constexpr (kGDirect) em.gon = P.want_g != 0;
  if constexpr (GAIT) {
    if (it.rsel > 0) { em.flo = it.row0 + rsel_first(it.rsel); em.fcnt = rsel_count(it.rsel); }
    em.nvals = P.want_jac ? T.v1 - T.v0 : 0;
    em.gon = P.want_g != 0;
    if (KBLOCK == TBLOCK || (int)threadIdx.x < TBLOCK) em.dd = P.idir[T.i0 + threadIdx.x];
  }
  double* xs = smem + lds_x_off;
  int32_t* ns = reinterpret_cast<int32_t*>(smem + lds_x_off + P.n_pad);
  char* gt = reinterpret_cast<char*>(smem + lds_x_off + P.n_pad + ((P.n_nodecol + 3) >> 2) * 2);   // GAIT tables
  // GAIT: the block zero-fills its tile's CSR range first; the value stores of any lane come after
  // the barrier below, which waits for these stores to complete (vmcnt(0)), so they land on top.
  // FDISC / TQDISC lanes own whole rows (row-split), so there each wave zero-fills its own rows
  // after the staging instead (below), and waits for them only at its first value store.
  constexpr bool kWaveZero = GAIT && (TYPE == IT_FDISC || TYPE == IT_TQDISC);
  if constexpr (GAIT && !kWaveZero)
    if (P.want_jac) zero_out(Vb + T.v0, T.v1 - T.v0, threadIdx.x, KBLOCK);
  if constexpr (early_stage(TYPE)) xst.commit(P, xg, xs, ns);
  else stage_x<KBLOCK, stages_nodes(TYPE, GAIT)>(P, xg, xs, ns);
  towr_terrain_t* ters = reinterpret_cast<towr_terrain_t*>(gt + 16 * P.gt_n16 + 8 * P.gt_ntime);   // GAIT: the terrain
  if constexpr (GAIT) {
    stage16<KBLOCK>(reinterpret_cast<uint4*>(gt), P.gtab, P.gt_n16);
    if (threadIdx.x < sizeof(towr_terrain_t) / 8)
      reinterpret_cast<double*>(ters)[threadIdx.x] = reinterpret_cast<const double*>(P.terrains + (P.terrain_per_problem ? b : 0))[threadIdx.x];
    if constexpr (!kWaveZero) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  TG_STAMP(P, 1);
  Ctx c;
  c.seg = nullptr; c.sg = P.sg; c.row = it.seg;
  c.x = xs; c.nodecol = ns; c.spl = P.spl; c.dur = P.dur;
  c.ter = P.terrains + (P.terrain_per_problem ? b : 0);
  c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
  c.gait = GAIT; c.pinfo = P.pinfo; c.pcols = P.pcols; c.pact = P.pact; c.sched = P.sched; c.eelin = P.eelin; c.lin = P.lin;
  if constexpr (GAIT) {   // the PhaseSpline searches and window emission read their tables from LDS
    c.spl = reinterpret_cast<const SplineMeta*>(gt + P.gt_off[0]);
    c.sched = reinterpret_cast<const SchedInfo*>(gt + P.gt_off[1]);
    c.pinfo = reinterpret_cast<const PolyPhase*>(gt + P.gt_off[2]);
    c.pact = reinterpret_cast<const int32_t*>(gt + P.gt_off[3]);
    c.pcols = reinterpret_cast<const PhaseCol*>(gt + P.gt_off[4]);
  }
  c.rotvec = ROTVEC;
  c.dyn_scratch = TYPE == IT_DYN ? smem + P.lds_scr_off : nullptr;
  if constexpr (GAIT) {
    // the x-dependent PhaseSpline timings once per block (phase_timings_block) instead of a
    // division-carrying scan per lane and spline evaluation
    double* tm = reinterpret_cast<double*>(gt + 16 * P.gt_n16);
    phase_timings_block(c, P, tm);
    c.pdur = tm; c.pend = tm + P.n_pinfo; c.phend = tm + 2 * P.n_pinfo; c.ph_stride = P.ph_stride;
    c.ter = ters;   // LDS copy: no global load in the evaluation waits behind the zero-fill stores
    if constexpr (kWaveZero) {
      if (P.want_jac) {   // each lane's owned rows, zero-filled by its whole wave (512 B per store)
        double* vt = Vb + T.v0;
        const int lane = threadIdx.x & 63;
        for (int l = 0; l < 64; ++l) {
          const int z0 = __shfl(em.dd.z0, l, 64), z1 = __shfl(em.dd.z1, l, 64);
          for (int p = z0 + lane; p < z1; p += 64) vt[p] = 0.0;
        }
        em.fence = true;
      }
    }
  }
  DynG0 g0;   // DYN group 0 between its two phases
  // fixed gait, RotVec: the base-angular coefficients of each (instant, component) come from the pre-pass
  // (towr_rv_coef_kernel, launched before this kernel); the component lanes only form and emit their 12 entries
  constexpr bool kRvPre = TYPE == IT_DYN && ROTVEC && !GAIT;
  if (it.type == TYPE) {
    if constexpr (TYPE == IT_DYN) {
      if (it.group == 0) {
        if constexpr (kRvPre) dyn_g0_a<true>(c, it, em, g0, P.rvc + rv_at((int64_t)b * P.n_rvi + it.a0) + 64 * kRvAb, 64);
        else dyn_g0_a(c, it, em, g0);
      }
      else if (kRvPre && it.group == 1) {
        if (P.want_jac) dyn_rv_emit_pre(c, it, P.rvc + rv_at((int64_t)b * P.n_rvi + it.a0), 64, em);
      }
      else eval_dyn(c, it, em);   // group 1 and the endeffector groups (these deposit their sum terms)
    } else {
      eval_typed<TYPE>(c, it, em);
    }
    em.flush();
  }
  TG_STAMP(P, 2);
  if constexpr (TYPE == IT_DYN) {   // phase B of group 0: the endeffector sums from LDS
    const bool g0lane = it.type == TYPE && it.group == 0;
    TileEmitPre<TBLOCK, kDynG0PhaseA, GAIT> emb(P.slots + it.slot, GAIT ? Vb + T.v0 : smem,
                                                GAIT || kGDirect ? Gb : smem + lds_rows_off - T.r0, g0lane);
    if constexpr (kGDirect) emb.gon = P.want_g != 0;
    emb.nvals = P.want_jac ? T.v1 - T.v0 : 0;
    emb.gon = P.want_g != 0;
    __syncthreads();
    if (g0lane) {
      double fs[3] = {0, 0, 0}, ts[3] = {0, 0, 0};
      const double* d = c.dyn_scratch + it.a2 * P.rb.n_ee * 6;
      for (int ee = 0; ee < P.rb.n_ee; ++ee)
        for (int e = 0; e < 3; ++e) { ts[e] += d[ee * 6 + e]; fs[e] += d[ee * 6 + 3 + e]; }
      dyn_g0_b(c, it, emb, g0, fs, ts);
    }
  }
  __syncthreads();
  TG_STAMP(P, 3);
  if constexpr (!GAIT) {
    if (P.want_jac) copy_out(smem, Vb + T.v0, T.v1 - T.v0, threadIdx.x, KBLOCK);
    if (P.want_g && !kGDirect)
      for (int i = threadIdx.x; i < T.r1 - T.r0; i += KBLOCK) __builtin_nontemporal_store(smem[lds_rows_off + i], Gb + T.r0 + i);
  }
  TG_STAMP(P, 4);
}

template <int TYPE, int BLOCK, bool GAIT, bool ROTVEC>
// second argument: minimum waves per SIMD. Dynamic: 2 (fixed gait: 256 lanes, 2 blocks per CU; gait: the
// 512-lane row-split block, <= 256 VGPRs). Fixed-gait RotVec Dynamic: 3 (<= 168 VGPRs, a 44-byte spill; with
// the g rows out of LDS three blocks fit a CU: 0.097 -> 0.093 ms per 4096 problems incl. the pre-pass, RotVec step
// 0.325 -> 0.320 ms; the Euler tile at 3 spills 324 bytes per lane and slows 0.061 -> 0.076 ms)
__global__ void __launch_bounds__(BLOCK, TYPE == IT_DYN && !GAIT && ROTVEC ? 3 : TYPE == IT_DYN ? 2 : 1) towr_tile_kernel(KParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;
  const int per = (total + 7) / 8;
  // XCD-aware mapping: work ids w and w+1 (tiles of one problem) share blockIdx % 8
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= total) return;
  tile_body<TYPE, BLOCK, BLOCK, GAIT, ROTVEC>(P, smem, w / P.ntiles, P.tiles[P.tile0 + w % P.ntiles], P.lds_x_off, P.lds_rows_off);
}


// The small kinds (node-value constraints, SplineAcc, BaseMotion, TotalDuration: a few kB of output
// per problem each) in one launch: a block = kMiscWaves one-wave tiles of one problem, sharing the
// staged x and node table; each wave evaluates and writes out its own tile.
template <bool GAIT>
__global__ void __launch_bounds__(64 * kMiscWaves, kMiscMinWaves) towr_misc_kernel(KParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.ntiles;   // ntiles = groups per problem
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= total) return;
  misc_body<GAIT>(P, smem, w / P.ntiles, w % P.ntiles, P.lds_x_off);
}

// Fused launches: a fusion group's classes run in ONE launch. A problem's units (its tiles of the
// group's classes and its small-kind groups) are consecutive work ids, interleaved round-robin over
// the classes, so latency-bound units (Dynamic, small kinds) share the CUs with write-bound ones and
// no launch boundary drains the machine between the group's classes. Every unit runs the same code
// as its per-class kernel (tile_body / misc_body). KBLOCK = the group's block size: 256 when it holds
// Dynamic or the small kinds (192-lane tiles then leave the fourth wave to staging and copy-out),
// else 192. The unit table is uniform per block (scalar loads). The kernel's register allocation is
// the largest of its classes' (Dynamic: 242 VGPRs), which is what decides whether a group pays off.
template <bool GAIT, bool ROTVEC, int KBLOCK>
__global__ void __launch_bounds__(KBLOCK, (KBLOCK == 256 ? 2 : 1)) towr_step_kernel(KParams P) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int total = P.B * P.n_units;
  const int per = (total + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= total) return;
  const int b = w / P.n_units;
  const UnitDesc u = P.units[w % P.n_units];
  switch (u.lc) {
    case LC_ROM: tile_body<IT_ROM, 192, KBLOCK, GAIT, ROTVEC>(P, smem, b, u.t, u.lds_x_off, u.lds_rows_off); break;
    case LC_FDISC: tile_body<IT_FDISC, 192, KBLOCK, GAIT, false>(P, smem, b, u.t, u.lds_x_off, u.lds_rows_off); break;
    case LC_TQDISC: tile_body<IT_TQDISC, 192, KBLOCK, GAIT, false>(P, smem, b, u.t, u.lds_x_off, u.lds_rows_off); break;
    default:
      if constexpr (KBLOCK == 256) {
        if (u.lc == LC_DYN) tile_body<IT_DYN, 256, KBLOCK, GAIT, ROTVEC>(P, smem, b, u.t, u.lds_x_off, u.lds_rows_off);
        else misc_body<GAIT, KBLOCK>(P, smem, b, u.tile, u.lds_x_off);
      } else if constexpr (KBLOCK >= 64 * kMiscWaves) {
        if (u.lc == LC_MISC) misc_body<GAIT, KBLOCK>(P, smem, b, u.tile, u.lds_x_off);
      }
      break;
  }
}

// The base-angular coefficients (and the base terms ab of the angular rows) of the fixed-gait RotVec Dynamic block (dyn_rv_state + dyn_rv_column<e>,
// rotvec_converter.cc:148-561 through dynamic_constraint.cc:124-166) for every (problem, instant, component),
// before the Dynamic launch. In the tile, one lane per instant formed the converter state and three lanes its
// columns after a barrier: the block's life was that chain at 2 waves per SIMD (242 VGPRs). Here one lane per
// (problem, instant, component) at full occupancy; waves are component-uniform (wave w: component w % 3, 64
// consecutive (problem, instant) pairs), and the coefficients are stored in blocks of 64 pairs, field-major in a
// block (layout.h rv_at), so both this kernel's stores and the tile's loads coalesce.
__global__ void __launch_bounds__(kRvCoefBlock) towr_rv_coef_kernel(KParams P) {
  const int K = P.n_rvi;
  const int64_t pairs = (int64_t)P.B * K, chunks = (pairs + 63) / 64;
  const int64_t w = (int64_t)blockIdx.x * (kRvCoefBlock / 64) + threadIdx.x / 64;
  if (w >= 3 * chunks) return;
  const int e = (int)(w % 3);
  const int64_t pr = (w / 3) * 64 + (threadIdx.x & 63);
  if (pr >= pairs) return;
  const int b = (int)(pr / K), q = (int)(pr - (int64_t)b * K);
  const RvInst ri = P.rvi[q];
  Ctx c{};
  c.seg = nullptr; c.sg = P.sg; c.row = ri.seg;
  c.x = P.X + (int64_t)b * P.ldx;   // base-angular node values only: never a constant node (layout.hip checks)
  c.nodecol = P.nodecol; c.spl = P.spl; c.dur = P.dur; c.ter = P.terrains;
  c.rb = P.rb; c.gait = false; c.rotvec = true;
  DynRvState S;
  dyn_rv_state(c, ri.t, S);
  if (e == 0) {   // the instant's base terms for its group-0 lane (also without the Jacobian: the g rows need them)
    double ab[3];
    dyn_base_ab(c.rb, S.R, S.w, S.wd, ab);
    double* o = P.rvc + rv_at(pr) + 64 * kRvAb;
#pragma unroll
    for (int f = 0; f < 3; ++f) __builtin_nontemporal_store(ab[f], o + 64 * f);
  }
  if (!P.want_jac) return;
  double M[9];
  if (e == 0) dyn_rv_column<0>(S, M, M + 3, M + 6);
  else if (e == 1) dyn_rv_column<1>(S, M, M + 3, M + 6);
  else dyn_rv_column<2>(S, M, M + 3, M + 6);
  double* o = P.rvc + rv_at(pr) + 64 * 9 * e;
#pragma unroll
  for (int f = 0; f < 9; ++f) __builtin_nontemporal_store(M[f], o + 64 * f);
}

template <bool GAIT, bool ROTVEC>
const void* kernel_for_mode(int type) {
  switch (type) {
    case IT_DYN: return reinterpret_cast<const void*>(&towr_tile_kernel<IT_DYN, tile_block(IT_DYN, GAIT), GAIT, ROTVEC>);
    case IT_ROM: return reinterpret_cast<const void*>(&towr_tile_kernel<IT_ROM, tile_block(IT_ROM, GAIT), GAIT, ROTVEC>);
    case IT_FDISC: return reinterpret_cast<const void*>(&towr_tile_kernel<IT_FDISC, tile_block(IT_FDISC, GAIT), GAIT, false>);
    case IT_TQDISC: return reinterpret_cast<const void*>(&towr_tile_kernel<IT_TQDISC, tile_block(IT_TQDISC, GAIT), GAIT, false>);
  }
  return nullptr;
}

}  // namespace

template <int KBLOCK>
const void* step_kernel_kb(bool rotvec) {
  return rotvec ? reinterpret_cast<const void*>(&towr_step_kernel<false, true, KBLOCK>) : reinterpret_cast<const void*>(&towr_step_kernel<false, false, KBLOCK>);
}
// fused launches exist only with fixed phase durations (setup_fusion: the gait layouts' tile blocks differ)
const void* step_kernel_for(bool gait, bool rotvec, int kblock) {
  if (gait) return nullptr;
  return kblock == 256 ? step_kernel_kb<256>(rotvec) : step_kernel_kb<192>(rotvec);
}

const void* tile_kernel_for(int type, bool gait, bool rotvec) {
  if (gait) return rotvec ? kernel_for_mode<true, true>(type) : kernel_for_mode<true, false>(type);
  return rotvec ? kernel_for_mode<false, true>(type) : kernel_for_mode<false, false>(type);
}
const void* rv_coef_kernel() { return reinterpret_cast<const void*>(&towr_rv_coef_kernel); }
const void* misc_kernel_for(bool gait) {
  return gait ? reinterpret_cast<const void*>(&towr_misc_kernel<true>) : reinterpret_cast<const void*>(&towr_misc_kernel<false>);
}

}  // namespace tg
