// layout.h — host-side problem builder for the HIP engine.
//
// Replaces, for the eval path, what the reference derives at setup in
//   NlpFormulation::GetVariableSets / GetConstraints (towr/src/nlp_formulation.cc:76-378),
//   NodesVariables*::GetPhaseBasedEEParameterization (nodes_variables_phase_based.cc:201-396),
//   TimeDiscretizationConstraint ctor (time_discretization_constraint.cc:37-50),
//   ifopt's Jacobian assembly (ConstraintSet::GetJacobian / setFromTriplets),
// and emits flat, batch-shared device tables: node->column map, polynomial durations, work items,
// CSR pattern, per-candidate slot table and LDS tiles.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "engine_math.h"

namespace tg {

struct TileDesc {
  int32_t i0, i1;   // items [i0, i1): exactly one item (or IT_NONE padding) per thread of the block
  int32_t r0, r1;   // rows  [r0, r1)
  int32_t v0, v1;   // values (CSR positions) [v0, v1)
  int32_t type, reserved;
};

// Wave w of small-kind group g (Layout::misc_tiles / misc_lds) as the device reads it: its tile's rows and values and
// its LDS offsets (ti -1: an empty wave), beside a copy of the tile's 64 items per (g, w) (towr_gpu.hip), so a block's
// descriptors are one load level instead of three (group -> tile -> items; tile_emit.h misc_body)
struct MiscWave {
  int32_t ti, r0, r1, v0, v1, wl_off, rows_off, reserved;
};

// Streaming composition of ForceConstraintDiscretized under phase-duration optimisation on a terrain
// without curvature (towr_gpu.hip fdisc_stream_body). One block per (problem, FsBlock) evaluates up to
// kFsInst instants once each (fdisc_instant), then writes the block's whole CSR range [v0, v0 + nv)
// — every 16-byte unit exactly once, zeros included — composing each entry from its instant's
// quantities. All rows of one constraint hold the same columns (checked): the force set's full
// PhaseSpline pattern and the schedule columns. Template entry j (fs_tmpl) = column j of a row:
//   >= 0: force column, PhaseCol index (bits 0-23) and dimension (bits 24-25); < 0: schedule column.
// The force entries polynomial p can make non-zero (its two nodes' variables) lie in the window
// [fs_ws[2 (wsoff + p)], + kFsWin) of row positions (checked); schedule columns at [js0, js0 + ns1).
#ifndef TOWR_FS_INST   // (experiment builds: -DTOWR_FS_INST)
#define TOWR_FS_INST 16
#endif
// measured on MI355X (ANYmal gait, B = 1024): 64 -> 0.501 ms, 32 -> 0.463, 16 -> 0.452, 8 -> 0.478 (round 3); with the
// round-5 composer (1 KB-aligned trips, 4 problems per block), step gait / + Torque: 16 0.584-0.593 / 1.144-1.152,
// 32 0.570-0.591 / 1.153-1.159, 8 0.638-0.650 / 1.203-1.205
constexpr int kFsInst = TOWR_FS_INST;
constexpr int kFsWin = 12;
// The composers (gstream.hip) find an entry's row (FsBlock) or instant (GsBlock) from its position e in the
// block's CSR range as (int)((e + 0.5f) * (1.0f / L)). The float product is within 2^-23 relative of
// (e + 0.5) / L, whose distance to the nearest integer is at least 0.5 / L; the result is exact while
// (e / L) 2^-23 < 0.5 / L, i.e. for e < 2^22. The layout keeps every block range below half that bound
// (build_fstream, build_gstream_class: fewer instants per block, or the tile path).
constexpr int kFloatDivMax = 1 << 21;
// FDISC record (gstream.hip fdisc_records -> the composer): S[kFsS] | b[5][3] | Jf.dx[3] | Jf.v[3] | ints ws, wd,
// cur, wq (two 32-bit ints per double, gs_int2). S = the basis sums of the force polynomial's active window in dimension 0;
// the three dimensions' windows hold PhaseCols of one structure (build_fstream checks it), so window position q
// holds S[slot q] (wq: 2 bits per position) times b[row][dim q] (wd: 2 bits per position, 3 = not an active column:
// 0). Round 5's record kept the 12 window positions' sums (36 fields instead of 29).
constexpr int kFsS = 4;   // = kGsAct (below)
constexpr int kFsB = kFsS, kFsDx = kFsS + 15, kFsV = kFsS + 18, kFsND = kFsS + 21;
constexpr int kFsRS = kFsND + 2, kFsCS = kFsRS | 1;   // record fields; LDS stride per instant
struct FsBlock {
  int32_t ee, n_inst, t0, r0;   // endeffector, instants, first instant's time index (fs_t), first row
  int32_t v0, nv, L, tmpl;      // CSR range [v0, v0 + nv), row length, template offset (fs_tmpl)
  int32_t js0, ns1, wsoff, pad;
};
static_assert(sizeof(FsBlock) % 4 == 0, "FsBlock is staged to LDS as int32 words");

// Streaming RangeOfMotion and Dynamic under phase-duration optimisation (gstream.hip), the FsBlock
// scheme generalised to rows whose columns differ by row type. Two launches per class:
//   record:  one block per problem, one lane per instant (Dynamic: per instant, per base-angular axis,
//            per (instant, endeffector)) evaluates the instant once and stores what every Jacobian
//            entry of its rows is a function of (the record, field-major in the handle's scratch);
//   compose: one block per (problem, GsBlock) streams the block's whole CSR range with 16-byte
//            stores, each unit written once, forming every entry from its instant's record and the
//            entry's position.
// Row r of an instant (its row type) is [base prefix | template]: the prefix holds the base-linear and
// base-angular columns of the instant's active base polynomials, coded per (instant, row) as
// blk << 4 | dim << 2 | basis (gs_pcode; the base node sets hold the smallest columns); the template is
// the same for every instant (checked) and codes each remaining column (gs_tmpl):
//   bit 31 set: schedule column, bits 16-18 endeffector, bits 0-15 column within its PhaseDurations;
//   else: a PhaseSpline column, bits 28-29 spline kind (0 motion, 1 force, 2 torque), 25-27
//   endeffector, 22-23 dimension, 0-21 PhaseCol index within that dimension's list.
// A PhaseSpline column is non-zero only in its instant's active window, at most kGsAct PhaseCols per
// dimension from the polynomial's first (pact); the composer's prologue forms their basis sums.
enum GsClass { GS_ROM = 0, GS_DYN = 1, GS_TQ = 2, GS_COUNT = 3 };   // GS_TQ: TorqueConstraintDiscretized (no base prefix)
constexpr int kGsRowTypes = 6;
constexpr int kGsAct = 4;
static_assert(kFsS == kGsAct, "the FDISC record's window sums are one active window");
// The composer launch (gstream.hip towr_gait_compose_kernel): the ForceConstraintDiscretized,
// RangeOfMotion and Dynamic compose blocks of every problem in one grid, kComposeBlock threads each.
// (experiment builds: -DTOWR_COMPOSE_BLOCK / -DTOWR_COMPOSE_BLOCK_RD. Round 5, ANYmal gait, B = 1024, one box, ms per step
// gait / + Torque: 512 / 256 0.606-0.619 / 1.163-1.174; FDISC composer 1024: 0.624-0.635 / 1.29; 256: 0.667-0.682 / 1.28;
// RangeOfMotion / Dynamic composer 512: 0.660-0.664 / 1.23; 128: 0.654-0.659 / 1.19)
#ifndef TOWR_COMPOSE_BLOCK
#define TOWR_COMPOSE_BLOCK 512
#endif
#ifndef TOWR_COMPOSE_BLOCK_RD
#define TOWR_COMPOSE_BLOCK_RD 256
#endif
constexpr int kComposeBlock = TOWR_COMPOSE_BLOCK;
constexpr int kComposeBlockRD = TOWR_COMPOSE_BLOCK_RD;   // a launch without FDISC blocks
inline int compose_block(int mask) { return (mask & 25) ? kComposeBlock : kComposeBlockRD; }
constexpr int kGsInstRom = 16;   // instants per compose block
constexpr int kGsInstTq = 16;
constexpr int kGsInstDyn = 2;   // measured on MI355X (ANYmal gait, B = 1024, grouped composer): 2 -> 0.201 ms, 4 -> 0.230, 8 -> 0.219
// A row type is cut into segments: its base prefix, each maximal run of template columns of one
// (spline kind, endeffector) or of one endeffector's schedule. Per instant a segment owns W values
// (GsSeg::vbase): the prefix and schedule segments all their positions, a PhaseSpline segment the
// window of W positions starting at ws(poly) (gs_ws[wsoff + poly], the active polynomial's first
// position in the segment); positions outside it are 0. The composer computes an instant's values once
// (one lane each), then every entry of the CSR range is one lookup: segment (gs_tseg, by position in
// the instant), window start, value.
// p0: first position in the instant; toff: gs_tmpl index = toff + position (prefix: gs_pcode index within the
// instant's codes = toff + position)
struct GsSeg { int8_t r, type, kind, ee; int16_t p0, len, W, vbase; int32_t wsoff, toff; };   // type 0 prefix, 1 window, 2 schedule
struct GsGeo {
  int32_t cls, ee, nrt, Li;   // class, endeffector (RangeOfMotion), row types, values per instant
  int32_t L[kGsRowTypes], P[kGsRowTypes], T[kGsRowTypes], poff[kGsRowTypes];   // per row type: length, prefix, template offset, prefix codes offset
  int32_t Psum, pc0, rec0, r0;   // prefix codes per instant, gs_pcode offset of instant 0, first record index, first row
  int32_t ns, seg0, vt, ts0;     // segments (gs_segs[seg0..]), values per instant, gs_tseg offset (Li bytes)
  int32_t vm0, K, blob0, blob_n16;   // gs_vmap offset (vt entries: segment << 16 | value index), instants,
                                     // the composer blob (gs_blob[blob0 ..], 16-byte units)
  int32_t o_vmap, o_tmpl, o_tseg, o_pcode, o_ws, reserved[3];   // byte offsets of its sections (segments at 0)
};
struct GsBlock { int32_t geo, k0, n_inst, v0, nv, reserved[3]; };   // instants [k0, k0 + n_inst) of the geometry
// a record lane's instant; kk / nb: its index in its GsBlock and the block's instants (the record chunk)
// p0: TorqueConstraintDiscretized's k_friction (ItemDesc::p0)
struct GsInst { double t; int32_t seg, row0; int16_t ee, kk, nb, reserved; double p0; };
// Records (gstream.hip gs_records): per instant RS fields, the composer's view of the instant —
// ND doubles then NI doubles of ints, two 32-bit ints per double (gs_int2; int j is dword j of that area) — so that a composer block's prologue is one contiguous
// copy. The fields of the GsBlock of instants [k0, k0 + n) form one chunk at RS * k0 (class-global
// instant index), field-major inside it (field f of instant k0 + kk at RS * k0 + f * n + kk).
//   RangeOfMotion: R[9] | HL[4] | Ag[axis][r] (9) | HA[4] | Jx.dx[3] v[3] | sums[dim][4] (12);
//                  ints cur | qa[dim] (3) | poly (3 doubles)
//   Dynamic:       fs[3] | Lp[3] | HpL[4] | HaL[4] | A[axis][p v a][r] (27) | HpA HvA HaA (12), then per
//                  endeffector Fp[3] | rv[3] | Jf.dx v[6] | Jx.dx v[6] | motion sums[dim][4] (12) | force sums[4] |
//                  torque sums[4]; ints per endeffector (6 doubles, each pair written by one record lane): curX | qaX[3] |
//                  polyX | - | curF | qaF | polyF | - | qaT | polyT (the force and torque windows start at one PhaseCol
//                  index in every dimension, spline_dims_coincide; round 5: 14 ints in 14 doubles). The force
//                  and torque sums are one set for the three dimensions, as TQDISC's below (the layout streams Dynamic
//                  only when they coincide, spline_dims_coincide): 38 doubles per endeffector instead of round 5's 54
//   TorqueConstraintDiscretized: t1[3] | t2[3] | n[3] | b[3] (= -k mu n) | Jt.dx v[6] | Jf.dx v[6] |
//                  torque sums[4] | force sums[4]; ints cur | qaT | qaF | polyT | polyF (3 doubles). The sums and qa are
//                  the same for the three dimensions (the layout streams TQDISC only when the torque and force
//                  splines' active windows hold PhaseCols of one structure in every dimension, spline_dims_coincide),
//                  so one set of 4 per spline: 35 fields instead of round 5's 57
//                  (torque_constraint_discretized.cc:139-235 without the motion block: a terrain
//                  without curvature, where every motion scale is exactly 0.0 and the block is skipped, :57)
// (kind 0 motion, 1 force, 2 torque; sums / qa: the active-window basis sums of the PhaseSpline, the
// first active PhaseCol of each dimension and the basis sums of up to kGsAct PhaseCols from it)
constexpr int kRomND = 44, kRomNI = 3;
constexpr int kDynBaseND = 53, kDynEeND = 38, kDynEeNI = 6;
// field of the window sum q of kind (0 motion, 1 force, 2 torque) and dimension e in a Dynamic record's endeffector part
TG_HD constexpr int dyn_sum_field(int kind, int e, int q) { return kind == 0 ? 18 + e * kGsAct + q : 26 + kind * kGsAct + q; }
constexpr int kTqND = 32, kTqNI = 3;
TG_HD constexpr int gs_rec_nd(int cls, int E) { return cls == GS_ROM ? kRomND : cls == GS_TQ ? kTqND : kDynBaseND + kDynEeND * E; }
TG_HD constexpr int gs_rec_ni(int cls, int E) { return cls == GS_ROM ? kRomNI : cls == GS_TQ ? kTqNI : kDynEeNI * E; }
TG_HD constexpr int gs_rec_fields(int cls, int E) { return gs_rec_nd(cls, E) + gs_rec_ni(cls, E); }
#ifndef TOWR_GS_GROUP   // (experiment builds: -DTOWR_GS_GROUP; round 5, one box, gait / + Torque / headline ms: 2 0.592-0.595 /
                        // 1.161-1.165 / 0.2365-0.2375; 1 0.620-0.629 / 1.276; 4 0.589-0.599 / 1.160-1.166 / 0.2364-0.2372;
                        // with the FDISC composer at 4 (towr_gpu.hip kFsGroup), the others at 4: 0.589-0.594 / 1.146-1.150
                        // vs 0.584-0.599 / 1.141-1.144, at 1: 0.600-0.601 / 1.160-1.166)
#define TOWR_GS_GROUP 2
#endif
constexpr int kGsGroup = TOWR_GS_GROUP;   // problems per composer block (gstream and fstream; 1 -> 0.333 ms, 2 -> 0.321, 8+ slower: a block
                              // waits for its stores to drain before the next problem's records land)
constexpr int kGsChunkMax = 2048;   // record doubles of a compose block (prefetched into registers: kGsChunkMax / kComposeBlock per thread)
// the RangeOfMotion / Dynamic records' arguments (gs_records)
struct GsRecArgs {
  double* rec;                 // per problem: RangeOfMotion records at 0, Dynamic records at dyn_off
  int64_t ldr, dyn_off;
  const GsInst* inst[GS_COUNT];
  int32_t K[GS_COUNT];         // instants per class (0: the class is not streamed)
  int32_t st_off, scr_off;     // LDS (doubles): the Dynamic states, the scratch (9 per instant, 9 per (ee, instant))
};

// Pattern watch (curved terrain): ForceConstraintDiscretized / TorqueConstraintDiscretized add their
// motion block of row i, dimension dim only where its scale is non-zero (force_constraint_discretized.cc:58,
// torque_constraint_discretized.cc:57), so the reference's pattern moves with x while IPOPT's structure
// (and the engine's CSR) is frozen at x0. One WatchItem per such instant: the x0 presence of each
// (dim, row) block and the entries a block holds; towr_gpu_pattern_outside counts, at any x, the
// reference entries outside the frozen pattern (blocks present at x, absent at x0), on the host.
struct WatchItem {
  double t, kf;           // instant; TorqueConstraintDiscretized's k_friction
  int32_t seg, type;      // segment-table row, IT_FDISC / IT_TQDISC
  int32_t ee, mask;       // endeffector; bit dim * rows + row: block present at x0
  int32_t cnt[2];         // entries of a block of dimension 0 / 1 (the motion spline's Jacobian row)
};

// a Dynamic instant of the RotVec coefficient pre-pass (fixed gait): its time and segment-table row
struct RvInst { double t; int32_t seg, reserved; };
constexpr int kRvCoef = 30;   // per instant: per component e, Mp[3] | Mv[3] | Ma[3] (dyn_rv_column); then the base terms ab[3]
constexpr int kRvAb = 27;     // (dyn_base_ab, read by the instant's group-0 lane)
// Scratch layout of the pre-pass: blocks of 64 (problem, instant) pairs pr = b K + q, field-major inside a block, so
// a wave's store of one field is 512 contiguous bytes and the kRvCoef fields of one pair sit in one 15 kB block
// (field-major over the whole batch put them 1.8 MB apart at B = 4096); field f of pair pr at rv_at(pr) + 64 f
__host__ __device__ constexpr int64_t rv_at(int64_t pr) { return (pr >> 6) * (int64_t)kRvCoef * 64 + (pr & 63); }

struct VarSetInfo { int kind, ee, col0, n; };
struct ConsInfo { int kind, ee, row0, rows; };

struct Layout {
  int n = 0, m = 0;
  int64_t nnz = 0;
  std::vector<VarSetInfo> varsets;
  std::vector<ConsInfo> cons;
  std::vector<SplineMeta> spl;
  std::vector<int32_t> nodecol;
  std::vector<double> dur;
  std::vector<SegRec> segs;     // (2 + 4 n_ee) records per time instant
  bool gait = false;            // phase-duration optimisation (PhaseSplines, schedule variables)
  bool rotvec = false;          // Parameters::RotationVector base orientation (RotVecConverter)
  std::vector<PolyPhase> pinfo; // PhaseSpline polynomial phases
  std::vector<PhaseCol> pcols;  // PhaseSpline full-pattern columns
  std::vector<int32_t> pact;    // PhaseSpline active PhaseCol ranges (SplineMeta::pact_off)
  std::vector<SchedInfo> sched; // per endeffector (col0 = -1 without schedule variables)
  std::vector<EELinDef> eelin;  // EELinearConstraint definitions (ItemDesc::a0 indexes them)
  std::vector<LinNz> lin;       // LinearEqualityConstraint rows (IT_LINEQ: ItemDesc::a0 / a1)
  std::vector<ItemDesc> items;
  std::vector<int32_t> slots;     // build-time: candidate -> global CSR position (or -1)
  std::vector<SlotGroup> slot_groups;   // device slot table (see SlotGroup); item.slot indexes it
  std::vector<ItemDirect> idirect;      // gait: per item (lane), direct-position ranges (ItemDirect)
  std::vector<int64_t> row_ptr;
  std::vector<int32_t> col;
  std::vector<TileDesc> tiles;
  std::vector<double> x0;
  RobotC rb{};
  towr_terrain_t terrain{};
  int32_t fdisc_motion = 0;
  towr_problem_desc_t desc{};
  // tiles are grouped by item type: tiles [type_tile0[t], type_tile0[t+1]) run in one launch of
  // the type's kernel with type_block[t] threads and type_lds[t] doubles of dynamic LDS
  int32_t type_tile0[IT_COUNT + 1] = {};
  int32_t type_block[IT_COUNT] = {};
  int32_t type_lds[IT_COUNT] = {};
  int32_t type_lds_rows_off[IT_COUNT] = {};   // start of the g buffer inside the type's LDS
  int32_t type_lds_dummy_off[IT_COUNT] = {};  // per-lane dummy slots for absent candidates
  int32_t dyn_scr_off = 0;                    // DYN LDS: endeffector sum terms after the g rows
  // fixed gait, RotVec: the Dynamic instants whose base-angular coefficients the pre-pass forms
  // (tiles.hip towr_rv_coef_kernel; a RotVec group-1 item's a0 indexes them)
  std::vector<RvInst> rv_inst;
  // algorithmic bytes per problem of each type's launch: CSR values + g rows written, distinct
  // x columns read (= the columns of its Jacobian rows)
  int64_t type_bytes[IT_COUNT] = {};
  // small kinds (is_misc_kind) run in one launch: kMiscWaves tiles per block, one per wave
  std::vector<int32_t> misc_tiles;   // groups of kMiscWaves tile indices (-1 = empty wave)
  std::vector<int32_t> misc_lds;     // per (group, wave): LDS offset of the wave's tile, its g-row offset (doubles)
  std::vector<int32_t> misc_xspan;   // x spans the small-kind blocks stage: (first 16-B unit, units) pairs; empty = all of x
  int32_t misc_region = 0;           // LDS of the largest group (doubles)
  int64_t misc_bytes = 0;
  // streaming ForceConstraintDiscretized (FsBlock): enabled under phase-duration optimisation on
  // terrains without curvature when every row of each constraint holds the same columns
  bool fstream = false;
  std::vector<FsBlock> fs_blocks;
  std::vector<double> fs_t;
  std::vector<int32_t> fs_tmpl;
  std::vector<int32_t> fs_ws;        // per (constraint, force polynomial): window start, window dimension codes
  std::vector<int32_t> fs_iee, fs_irow, fs_iblk;   // per instant (fs_t order): endeffector, first row, FsBlock
  int32_t fs_tmpl_max = 0;
  // streaming RangeOfMotion / Dynamic (GsGeo): per class enabled when every constraint of the class fits
  bool gstream[GS_COUNT] = {};
  std::vector<GsGeo> gs_geo;
  std::vector<GsBlock> gs_blocks[GS_COUNT];
  std::vector<GsInst> gs_inst[GS_COUNT];   // record lanes' instants (Dynamic: one per instant)
  std::vector<int32_t> gs_tmpl;
  std::vector<uint8_t> gs_pcode;
  std::vector<GsSeg> gs_segs;
  std::vector<uint8_t> gs_tseg;
  std::vector<uint32_t> gs_vmap;
  std::vector<int16_t> gs_ws;
  // per geometry, the composer's static tables in one blob staged to LDS in one pass:
  // [segments | value map | template | position -> segment | prefix codes of every instant | window starts]
  // (GsSeg::toff of a template segment indexes the blob's template, GsSeg::wsoff its window starts)
  std::vector<uint4> gs_blob;
  std::vector<WatchItem> watch;     // pattern watch (curved terrain only)
  int32_t gs_geo_max[GS_COUNT][4] = {};  // largest geometry of the class: Li, segments, values per instant, blob bytes
  int32_t gs_tmpl_max[GS_COUNT] = {};      // template ints of the largest geometry (compose LDS)
  int32_t gs_pcode_max[GS_COUNT] = {};     // prefix codes per instant, largest geometry
  int32_t gs_nmax[GS_COUNT] = {};          // instants of the largest compose block
  // cost terms (eval_f / eval_grad_f): work items sorted by CostType, one block per problem
  std::vector<CostItem> cost_items;
  std::vector<double> cost_q;        // CT_ENERGYQ Gram matrices, 16 doubles per item (CostItem::q)
  // Deterministic gradient (fixed phase durations): every present gradient entry of every cost item has an
  // LDS contribution slot, ordered by column (layout.hip build_cost_slots): entry k of item i goes to slot
  // cost_cslot[CostItem::cslot + k], and column j sums slots [cost_cptr[j], cost_cptr[j + 1]) in order.
  // cost_nslot = 0: fixed-point limbs instead (phase-duration optimisation, where the PhaseSpline windows
  // move with x, or more slots than kCostSlotMax).
  int32_t cost_nslot = 0;
  std::vector<uint16_t> cost_cptr;
  std::vector<uint16_t> cost_cslot;
  // SoftConstraint terms (TOWR_COST_SOFT), in cost order: the cost index and the wrapped constraint.
  // The wrapped sets are evaluated by a second layout (the handle's soft child) whose constraint
  // list is exactly these sets in this order (soft_desc).
  std::vector<std::pair<int32_t, int32_t>> soft;
};

#ifndef TOWR_COST_SLOT_MAX   // (experiment builds: -DTOWR_COST_SLOT_MAX=0, the limbs everywhere)
#define TOWR_COST_SLOT_MAX 8192
#endif
constexpr int kCostSlotMax = TOWR_COST_SLOT_MAX;   // contribution slots of the cost kernel's LDS (64 KB)
constexpr int kCostLanes = 256;   // threads of the cost kernel's blocks (kCostBlock, its wave schedule)
constexpr int kMiscWaves = 4;   // one-wave small-kind tiles per group (block)
constexpr int kSlotSpare = 4;   // spare slot groups per lane: the kernels prefetch up to this many ahead
constexpr bool is_misc_kind(int t) { return t != IT_DYN && t != IT_ROM && t != IT_FDISC && t != IT_TQDISC; }

// launch classes: the heavy kinds have their own kernels, the small kinds share one
enum LaunchClass { LC_DYN = 0, LC_ROM = 1, LC_FDISC = 2, LC_TQDISC = 3, LC_MISC = 4, LC_COUNT = 5 };
constexpr int class_type(int lc) { return lc == LC_TQDISC ? IT_TQDISC : lc; }   // tile classes

// LDS tile caps (doubles of CSR values / rows per tile)
constexpr int kTileValueCap = 8192;
constexpr int kTileRowCap = 2048;
constexpr int kMiscValueCap = 3072;   // small-kind tiles: 4 share one block's LDS
constexpr int kMiscRowCap = 512;

// Tile value cap under phase-duration optimisation: the tile classes have no LDS tile there (they
// store straight into a zero-filled V, TileEmit DIRECT), so a tile is bounded only by its lanes and
// the uint16 slot positions (values + 64 dummy slots < kSlotAbsent)
constexpr int kTileValueCapGait = 65536 - 2 - 64 - 2;

// Row-split items (phase-duration optimisation only). A PhaseSpline item emits its full-pattern
// windows and schedule columns one candidate at a time, a chain of dependent slot-table and
// PhaseCol loads; one item per instant would leave a tile of ~20 instants on 20 lanes of a 192-lane
// block. Such items are split over lanes by rows (ItemDesc::rsel, split_part_rows): every lane
// evaluates the instant, only its rows' candidates are emitted. Returns the lanes per item (1 = not split).
int split_rows(int type, int group, bool gait);

// Block size of the tile classes. Under phase-duration optimisation every wave holds one row of
// the split items (lanes = instants), so that a wave's lanes take the same branches: a wave mixing
// the rows of an item would execute every row's emission path one after the other.
//   DYN: g0 | g1 | row 0 .. 5 of the endeffector groups (lanes = ee x instant);
//   ROM: two halves of 64 instants, each g0 | g1 | row 0 | 1 | 2 of the motion group;
//   FDISC: two halves of 64 instants, each row 0 | 1 | 2 | 3 | 4;  TQDISC: rows 0 .. 3.
// A 5-wave block is placed as if it took 2 waves on every SIMD (hipOccupancy... and the measured
// residency: 1 block per CU at 168 VGPRs), and a 4-wave block with FDISC rows (0, 1) on one wave
// waits for that wave (1.5x the others): 10-wave blocks are balanced and fill 10 of the 12 wave slots.
constexpr int kDynGaitRowParts = 6;
constexpr int tile_block(int type, bool gait) {
  return type == IT_DYN ? (gait ? 64 * (2 + kDynGaitRowParts) : 256) : type == IT_ROM ? (gait ? 640 : 192) : type == IT_FDISC ? (gait ? 640 : 192)
       : type == IT_TQDISC ? (gait ? 256 : 192) : 64;
}

// Launch geometry of each item type (wave-uniform: each wave of a block runs one code path)
struct TypeSpec { int block; int max_inst; };
TypeSpec type_spec(int type, int n_ee, bool gait, bool rotvec = false);
// thread (lane) of the block that evaluates row-part `sub` (0 .. split_rows - 1) of group `g` of
// the k-th of n instances in a tile
int type_lane(int type, int group, int k, int n, int n_ee, bool gait, int sub);

inline int64_t fs_record_doubles() { return kFsRS; }   // FDISC record doubles per instant

// The streaming kernels (gstream.hip): compose LDS (bytes), record doubles per problem of one class,
// entry points. The record kernel uses fs_inst_lds_bytes' LDS layout, then its Dynamic states and
// scratch (gs_rec_lds).
size_t gs_stream_lds(const Layout& L, int cls);
size_t fs_compose_lds(const Layout& L);   // the ForceConstraintDiscretized compose block (bytes)
int64_t gs_record_doubles(const Layout& L, int cls);
const void* gait_rec_kernel(bool rotvec, int roles);   // instantiation: bit 0 the FDISC part, 1 the RangeOfMotion / Dynamic parts, 2 the TQDISC part
const void* gait_compose_kernel(int mask);   // roles: bit 0 FDISC, 1 RangeOfMotion, 2 Dynamic, 3 small kinds, 4 TQDISC
constexpr int kComposeMasks[] = {1, 2, 4, 6, 7, 15, 16, 17, 23, 31};   // the instantiated role sets
// the composer launch's arguments: the record arrays (per problem, leading dimensions; the
// TorqueConstraintDiscretized records sit in the FDISC record array at tq_off) and, per role (0 FDISC,
// 1 RangeOfMotion, 2 Dynamic, 3 small-kind groups, 4 TorqueConstraintDiscretized), its blocks per problem
// group (0: not in this launch). A problem group's units: [FDISC | TQDISC | RangeOfMotion | Dynamic | small kinds]
struct ComposeArgs {
  const double* frec; int64_t fldr, tq_off;
  const double* grec; int64_t gldr, gdyn_off;
  const GsBlock* blk[GS_COUNT];
  int32_t nt[5];
  int32_t ng;          // problem groups: a block composes problems g, g + ng, ... (kGsGroup per block)
  int32_t misc_x_off;  // small kinds: the staged x's LDS offset (doubles)
};
// the record launch's arguments (towr_gait_rec_kernel): nparts blocks per problem, block r doing part
// (parts >> 4 r) & 15 (RecPart); the FDISC records (frec, fldr, ni instants) and the
// TorqueConstraintDiscretized records (frec + tq_off, g.inst[GS_TQ]) share one array per problem
enum RecPart { kRecFdisc = 1, kRecTq = 2, kRecGs = 3, kRecGsDyn = 4, kRecGsRom = 5 };
struct RecArgs {
  GsRecArgs g;
  double* frec; int64_t fldr, tq_off;
  int32_t ni, nparts, parts;
  // the FDISC launch (gstream.hip towr_gait_frec_kernel): byte offset in LDS of the staged FsBlock / window /
  // template tables (0: the lanes read them in global memory), and their sizes in int32 words
  int32_t fs_lds, fs_nb, fs_nws, fs_ntm;
};
size_t gs_dyn_state_bytes(bool rotvec);   // the record kernel's per-Dynamic-instant LDS state
constexpr int kGsRecMaxBlock = 512;
constexpr int kFsRecBlock = 512;   // the record launch's threads when it holds FDISC records
// The frozen-pattern check (WatchItem): reference Jacobian entries at x outside the x0 pattern, evaluated
// with the structure pass's arithmetic on the host
int64_t pattern_outside_host(const Layout& L, const double* x, const towr_terrain_t& terrain);

// Returns TOWR_OK or an error code with a message in `err`. Side data (towr_gpu_create_ex): the
// LinearEqualityConstraint matrices; the SoftConstraint bounds are checked by the handle.
int build_layout(const towr_problem_desc_t& d, Layout& L, std::string& err);
int build_layout_ex(const towr_problem_desc_t& d, int n_data, const towr_data_t* data, Layout& L, std::string& err);
// the description of the soft child: the SoftConstraint terms' wrapped sets as hard constraints, no costs
towr_problem_desc_t soft_desc(const towr_problem_desc_t& d, const Layout& L);
const towr_data_t* find_data(int n_data, const towr_data_t* data, int kind, int index);

// x0 for another init/terrain on the layout built from `d` (nlp_formulation.cc:121-346).
int initial_x_for(const towr_problem_desc_t& d, const towr_init_t& init, const towr_terrain_t& ter,
                  std::vector<double>& x0, std::string& err);


}  // namespace tg
