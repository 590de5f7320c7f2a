// tile_emit.h — the LDS tile emitter (TileEmit) and the small-kind group body (misc_body), shared by
// tiles.hip (tile kernels, the small-kind launch, the fused launch) and gstream.hip (the small kinds as
// blocks of the phase-duration path's composer launch at small batch sizes).
#pragma once

#include <hip/hip_runtime.h>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"

namespace tg {
namespace {

// Stores candidate j of this lane into the LDS tile at its tile-relative CSR position. Positions
// come 8 per 16-byte SlotGroup; the next group is prefetched while the current one is consumed, so
// the slot-table latency (L2: the table is shared by every problem of the batch) hides behind 8
// candidates of arithmetic. The candidate's column is never needed on the device, and no item emits
// a column twice (engine_math.h), so every position receives exactly one plain LDS store; absent
// candidates (constant node values) go to a per-lane dummy slot, so the store needs no branch.
// DIRECT (phase-duration optimisation): there is no LDS tile. The full-pattern Jacobian is ~90 %
// zeros whose positions move with x, and an LDS tile of it held ~13 instants per block (one busy wave
// of three, 2 blocks per CU), so the launch was bound by the evaluation's latency at low occupancy.
// Instead each block zero-fills its tile's CSR range in V (zero_out), and after a barrier lanes store
// their present candidates straight to HBM: `out` is the tile's first CSR value in V, `gout` the problem's g,
// absent candidates (positions >= nvals, the dummy slots) are not stored. The lane's item may be
// row-split (ItemDesc::rsel): only its rows' candidates are emitted (and counted), exactly as the
// structure pass recorded them, and only those rows' g.
template <int BLOCK, int DEPTH, bool DIRECT = false, int PRE = 1, int DYNG = 0>
struct TileEmit {
  static constexpr int kDynGroups = DYNG;   // Dynamic groups this emitter's kernel evaluates (engine_math.h)
  static_assert(PRE >= 0 && PRE <= 6 && PRE <= kSlotSpare + 2, "preloaded slot groups: 0 .. 6, within the spare groups");
  const SlotGroup* slot;   // this lane's group 0; group g at slot[g * BLOCK]
  double* out;             // LDS tile, tile-relative (DIRECT: V at the tile's first value)
  double* gout;            // LDS g rows, tile-relative (DIRECT: the problem's g)
  SlotGroup q[DEPTH];      // groups g .. g + DEPTH - 1 in flight (q[0] = current)
  int j = 0;
  int flo = 0, fcnt = 0;   // DIRECT: the selected rows flo .. flo + fcnt - 1 (fcnt 0 = all rows)
  int nvals = 0;           // DIRECT: values of the tile
  ItemDirect dd{};         // DIRECT: column ranges stored at off + col without the slot table
  bool fence = false;      // DIRECT: the wave's own zero-fill stores must complete before the first value store
  int qg = 0;              // DIRECT: slot group held in q[0] (the ring reloads lazily, on use)
  static constexpr bool kFilter = DIRECT;
  __device__ __forceinline__ bool want(int row) const { return !DIRECT || fcnt == 0 || (unsigned)(row - flo) < (unsigned)fcnt; }
  // DIRECT: slot groups 0 .. kPre - 1 are loaded at construction into named registers (a runtime-
  // indexed array would go to scratch); on gfx950 vmcnt counts stores too, so a group loaded after the
  // lane's first value stores waits for all of them (measured: the RangeOfMotion base lanes, 36
  // slot-path candidates, were the gait tile's slowest waves)
  static constexpr int kPre = DIRECT ? PRE : 0;
  u32x4_t p0 = {}, p1 = {}, p2 = {}, p3 = {}, p4 = {}, p5 = {};   // native vectors: a SlotGroup (array) would go to scratch
  __device__ __forceinline__ TileEmit(const SlotGroup* s, double* o, double* go) : slot(s), out(o), gout(go) {
    if constexpr (DIRECT) {
      const u32x4_t* sv = reinterpret_cast<const u32x4_t*>(s);
      if (kPre > 0) p0 = sv[0];
      if (kPre > 1) p1 = sv[BLOCK];
      if (kPre > 2) p2 = sv[2 * BLOCK];
      if (kPre > 3) p3 = sv[3 * BLOCK];
      if (kPre > 4) p4 = sv[4 * BLOCK];
      if (kPre > 5) p5 = sv[5 * BLOCK];
      qg = -1;
    } else {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) q[d] = s[d * BLOCK];
    }
  }
  bool gon = true;         // DIRECT: g requested
  __device__ __forceinline__ void g(int row, double v) {   // (fixed-gait Dynamic: g straight to HBM, gon = g requested)
    if (!DIRECT) { if (gon) gout[row] = v; }
    else if (gon && want(row)) gout[row] = v;
  }
  // GAIT outputs are zero-filled before the evaluation (tile_body / misc_body), so candidates whose
  // value is 0 can be skipped: move to candidate j + k, reloading the slot ring if the group changes
  static constexpr bool kSparse = true;
  __device__ __forceinline__ void skip(int k) {
    if constexpr (DIRECT) {   // lazy: the next slot-path candidate loads its group
      j += k;
      return;
    }
    if (k <= 0) return;
    const int g0 = j >> 3;
    j += k;
    const int g1 = j >> 3;
    if (g1 != g0) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) q[d] = slot[(g1 + d) * BLOCK];
    }
  }
  __device__ __forceinline__ void operator()(int row, int col, double v, bool) {
    if constexpr (DIRECT) {
      // Direct-range candidates need no slot load. Slot-path groups load lazily: on gfx950 vmcnt
      // counts stores too, so a group prefetched across this lane's value stores would wait for them.
      if (!want(row)) return;
      int s;
      if (col >= dd.c0[0] && col < dd.c1[0]) {
        s = dd.off[0] + col;
      } else if (col >= dd.c0[1] && col < dd.c1[1]) {
        s = dd.off[1] + col;
      } else {
        const int g = j >> 3;
        if (g < kPre) {   // preloaded before any store of this lane (no wait behind the value stores)
          const u32x4_t v = g == 0 ? p0 : g == 1 ? p1 : g == 2 ? p2 : g == 3 ? p3 : g == 4 ? p4 : p5;
          const int k = j & 7;
          const uint32_t lo = (k & 2) ? v.y : v.x, hi = (k & 2) ? v.w : v.z;
          const uint32_t w = (k & 4) ? hi : lo;
          s = (k & 1) ? (int)(w >> 16) : (int)(w & 0xFFFFu);
        } else {
          if (g != qg) {
            q[0] = slot[g * BLOCK];
            qg = g;
          }
          s = slot_pick(q[0], j & 7);
        }
      }
      ++j;
      if (fence) {   // wave-level: the zero stores of this wave's rows (tile_body) land first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        fence = false;
      }
      if (s < nvals) out[s] = v;
      return;
    }
    const int s = slot_pick(q[0], j & 7);
    ++j;
    if ((j & 7) == 0) {
#pragma unroll
      for (int d = 0; d + 1 < DEPTH; ++d) q[d] = q[d + 1];
      q[DEPTH - 1] = slot[((j >> 3) + DEPTH - 1) * BLOCK];
    }
    out[s] = v;   // absent candidates land in the lane's dummy slot
  }
  __device__ __forceinline__ void flush() {}
};

// The small kinds (node-value constraints, SplineAcc, BaseMotion, TotalDuration: a few kB of output
// per problem each) in one launch: a block = kMiscWaves one-wave tiles of one problem, sharing the
// staged x and node table; each wave evaluates and writes out its own tile.
// BLOCK = the launch's block size (>= 64 kMiscWaves): waves past the group's tiles only help stage x.
template <bool GAIT, int BLOCK = 64 * kMiscWaves>
__device__ __forceinline__ void misc_body(const KParams& P, double* smem, int b, int group, int lds_x_off) {
  static_assert(BLOCK >= 64 * kMiscWaves, "a small-kind group needs a wave per tile");
  const int wave = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  TG_STAMP(P, 0);
  // the wave's descriptor and the lane's item: one load level, issued with the x staging (the chain group -> tile ->
  // items was three: tools/stamps.py, MI355X, ANYmal, B = 4096: 3.5 us to the staging barrier of a 6.6 us block)
  const int gw = group * kMiscWaves + wave;
  MiscWave T{};
  T.ti = -1;
  ItemDesc it{};
  it.type = IT_NONE;
  it.slot = 0;
  if (wave < kMiscWaves) {
    T = P.misc_wave[gw];
    it = P.misc_items[gw * 64 + lane];
  }
  const int ti = T.ti;
  const int32_t wl_off = ti >= 0 ? T.wl_off : 0;
  const int32_t rows_off = ti >= 0 ? T.rows_off : 0;
  double* wl = smem + wl_off;
  TileEmit<64, 3> em(P.slots + it.slot, wl, wl + rows_off - T.r0);
  double* xs = smem + lds_x_off;
  int32_t* ns = reinterpret_cast<int32_t*>(smem + lds_x_off + P.n_pad);
  if constexpr (GAIT)   // sparse PhaseSpline emission: each wave zero-fills its own tile
    if (ti >= 0) zero_lds(wl, T.v1 - T.v0, lane, 64);
  if constexpr (GAIT) stage_x<BLOCK, true>(P, P.X + (int64_t)b * P.ldx, xs, ns);
  else stage_x_spans<BLOCK>(P, P.X + (int64_t)b * P.ldx, xs, ns);
  __syncthreads();
  TG_STAMP(P, 1);
  if (it.type != IT_NONE) {
    Ctx c;
    c.seg = nullptr; c.sg = P.sg; c.row = it.seg;
    c.x = xs; c.nodecol = ns; c.spl = P.spl; c.dur = P.dur;
    c.ter = P.terrains + (P.terrain_per_problem ? b : 0);
    c.rb = P.rb; c.fdisc_motion = P.fdisc_motion;
    c.gait = GAIT; c.pinfo = P.pinfo; c.pcols = P.pcols; c.pact = P.pact; c.sched = P.sched; c.eelin = P.eelin; c.lin = P.lin;
    c.rotvec = false;   // no small kind uses the base orientation
    c.dyn_scratch = nullptr;
    switch (it.type) {   // wave-uniform: a wave holds one tile of one kind
      case IT_FNODE: eval_fnode(c, it, em); break;
      case IT_TERR: eval_height(c, it, sp_motion(it.ee), 0.0, em); break;
      case IT_BMOT: eval_bmot(c, it, em); break;
      case IT_SACC: eval_sacc(c, it, em); break;
      case IT_BHGT: eval_height(c, it, SP_BASE_LIN, it.p0, em); break;
      case IT_SWING: eval_swing(c, it, em); break;
      case IT_TDUR: eval_tdur(c, it, em); break;
      case IT_TQNODE: eval_tqnode(c, it, em); break;
      case IT_THARD: eval_thard(c, it, em); break;
      case IT_EELIN: eval_eelin(c, it, em); break;
      case IT_LINEQ: eval_lineq(c, it, em); break;
      default: break;
    }
  }
  __syncthreads();
  TG_STAMP(P, 2);
  if (ti < 0) return;
  double* Vb = P.V + (int64_t)b * P.ldv;
  double* Gb = P.G + (int64_t)b * P.ldg;
  if (P.want_jac) copy_out(wl, Vb + T.v0, T.v1 - T.v0, lane, 64);
  if (P.want_g)
    for (int i = lane; i < T.r1 - T.r0; i += 64) __builtin_nontemporal_store(wl[rows_off + i], Gb + T.r0 + i);
  TG_STAMP(P, 3);
}

}  // namespace
}  // namespace tg
