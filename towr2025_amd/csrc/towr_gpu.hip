// towr_gpu.hip — the C-ABI (include/towr_gpu.h) and host side of the eval_g / eval_jac_g engine: handle,
// device tables, launch sequencing, host-pointer entry points. The kernels live in tiles.hip,
// gstream.hip and cost_traj.hip.
//
// One fused launch evaluates, for a batch of B problems sharing one layout, every constraint value
// g and every Jacobian nonzero of ifopt's RowMajor CSR (what IpoptAdapter::eval_g / eval_jac_g
// return). Work decomposition:
//   * block = (problem, group of LDS tiles); blocks of one problem are placed on one XCD
//     (blockIdx % 8 round-robin), so x is fetched from HBM once per problem;
//   * the problem's x (NodesVariables / PhaseDurations values) is staged in LDS;
//   * a tile = consecutive instances of one constraint set whose CSR value range fits in LDS;
//     lanes evaluate work items (node-per-lane Hermite splines, SRBD, terrain) and accumulate
//     Jacobian candidates into LDS at precomputed slots; then the tile's contiguous CSR range and
//     g range are written with 16-byte coalesced stores.
// No MFMA: there is no dense contraction; the kernel is HBM-write bound.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "engine_math.h"
#include "kernel_common.h"
#include "layout.h"

using namespace tg;


// =================================================================================================
// handle
// =================================================================================================
struct towr_gpu_handle_s {
  Layout L;
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // device tables
  ItemDesc* d_items = nullptr;
  SlotGroup* d_slots = nullptr;
  TileDesc* d_tiles = nullptr;
  int32_t* d_nodecol = nullptr;
  SplineMeta* d_spl = nullptr;
  double* d_dur = nullptr;
  void* d_segs = nullptr;      // SegSoA storage
  SegSoA sg{};
  PolyPhase* d_pinfo = nullptr;
  PhaseCol* d_pcols = nullptr;
  int32_t* d_pact = nullptr;
  SchedInfo* d_sched = nullptr;
  int32_t* d_misc = nullptr;
  int32_t* d_misc_lds = nullptr;
  MiscWave* d_misc_wave = nullptr;
  ItemDesc* d_misc_items = nullptr;
  int32_t* d_xspan = nullptr;
  EELinDef* d_eelin = nullptr;
  LinNz* d_lin = nullptr;
  uint4* d_gtab = nullptr;     // GAIT: PhaseSpline tables blob (GaitTables)
  ItemDirect* d_idir = nullptr;
  CostItem* d_citems = nullptr;
  double* d_cq = nullptr;
  FsBlock* d_fsb = nullptr;    // streaming ForceConstraintDiscretized tables (layout.h FsBlock)
  double* d_fs_t = nullptr;
  int32_t* d_fs_tmpl = nullptr;
  int32_t* d_fs_ws = nullptr;
  int32_t* d_fs_iee = nullptr;
  int32_t* d_fs_irow = nullptr;
  int32_t* d_fs_iblk = nullptr;
  double* d_fsrec = nullptr;   // per-problem instant records of the streaming path (scratch, grown on demand)
  int64_t fsrec_cap = 0;       // problems it holds
  GsGeo* d_gs_geo = nullptr;   // streaming RangeOfMotion / Dynamic tables (layout.h GsGeo)
  int32_t* d_gs_tmpl = nullptr;
  uint8_t* d_gs_pcode = nullptr;
  GsSeg* d_gs_segs = nullptr;
  uint8_t* d_gs_tseg = nullptr;
  uint32_t* d_gs_vmap = nullptr;
  int16_t* d_gs_ws = nullptr;
  uint4* d_gs_blob = nullptr;
  GsBlock* d_gs_blk[GS_COUNT] = {};
  GsInst* d_gs_inst[GS_COUNT] = {};
  double* d_rvc = nullptr;     // fixed gait, RotVec: the Dynamic base-angular coefficients of the pre-pass (scratch)
  int64_t rvc_cap = 0;
  RvInst* d_rvi = nullptr;
  double* d_gsrec = nullptr;   // their records, both classes (scratch, grown on demand)
  int64_t gsrec_cap = 0;
  // The scratch above (and the soft child's g / values, d_sg / d_sv) is shared by every call on the
  // handle: a call on another stream than the previous one waits for the previous call's work (this
  // event), and growing a buffer waits for it on the host before the old one is freed.
  hipEvent_t scr_ev = nullptr;
  hipStream_t scr_stream = nullptr;
  bool scr_used = false;
  bool sync_call = false;   // host_eval: the call synchronises its stream before returning (no event needed)
  // towr_gpu_eval_g_keep_jac: the Jacobian of kept_x waits in the device staging d_v (kept: until any other
  // host-pointer evaluation reuses the staging)
  bool kept = false;
  std::vector<double> kept_x;
  // fusion groups (TOWR_GPU_FUSE, see towr_step_kernel): classes that run in one launch
  struct FuseGroup {
    uint32_t mask = 0;        // bit lc: launch class lc belongs to the group
    int kblock = 0;
    UnitDesc* d_units = nullptr;
    int32_t n_units = 0;
    size_t lds = 0;
  };
  static constexpr int kMaxFuse = 2;
  FuseGroup fuse[kMaxFuse];
  int n_fuse = 0;
  // one problem through host pointers (eval_g / eval_jac_values / eval_g_jac): every class in ONE
  // launch (the fused kernel over all units), so the per-call latency is one kernel, not three
  FuseGroup single;
  // host entry points: caller memory page-locked by towr_gpu_register_host (DMA straight to / from
  // it), the copy stream of the chunked host batch and its per-chunk events
  struct Pinned { const char* p; size_t n; char* dev; };   // host range and its device address
  std::vector<Pinned> pinned;
  double *hd_x = nullptr, *hd_g = nullptr, *hd_v = nullptr;   // device addresses of the pinned staging
  hipStream_t copy_stream = nullptr;
  std::vector<hipEvent_t> ev_c, ev_d;
  std::string fuse_name[kMaxFuse];   // towr_gpu_kernel_info
  // fork-join of the per-kind launches (TOWR_GPU_STREAMS = total streams incl. the caller's, 1..4)
  static constexpr int kMaxSide = 3;
  int n_side = 0;
  hipStream_t side[kMaxSide] = {};
  hipEvent_t fork = nullptr, join[kMaxSide] = {};
  bool rv_overlap = false;   // RotVec without fusion groups: Dynamic and the small kinds on side stream 0 (launch_classes)
  towr_terrain_t* d_terrain = nullptr;      // base terrain (1 entry)
  towr_terrain_t* d_bterrain = nullptr;     // per-problem batch terrains
  int32_t bterrain_n = 0;
  std::vector<towr_terrain_t> bterrain_h;   // their host copy (the frozen-pattern check)
  // staging for host-pointer entry points
  double *d_x = nullptr, *d_g = nullptr, *d_v = nullptr;
  double *h_x = nullptr, *h_g = nullptr, *h_v = nullptr;
  int32_t stage_B = 0;
  double *d_f = nullptr, *d_grad = nullptr;   // host-pointer objective entry points (one problem)
  // trajectory export: fixed phase table and the sample times of the last dt
  double* d_traj_pd = nullptr;
  int32_t* d_traj_n = nullptr;
  int32_t* d_traj_c0 = nullptr;
  double* d_traj_t = nullptr;
  double traj_dt = 0.0;
  int32_t traj_ns = 0;
  // SoftConstraint terms: a second handle over the wrapped sets (soft_desc), its CSR pattern, the
  // bounds' mid-points b (rows in its order) and its per-batch g / values scratch
  towr_gpu_handle_s* soft = nullptr;
  std::vector<double> soft_b;
  double* d_soft_b = nullptr;
  int32_t* d_soft_cptr = nullptr;   // the soft pattern by column (KParams::s_cptr / s_cent)
  int2* d_soft_cent = nullptr;
  uint16_t* d_c_cptr = nullptr;     // the cost gradient's slot lists (Layout::cost_cptr / cost_cslot)
  uint16_t* d_c_cslot = nullptr;
  int cost_grid[3] = {1, 1, 1};     // the cost kernel's persistent grid per accumulation (launch_cost)
  double *d_sg = nullptr, *d_sv = nullptr;
  int64_t soft_cap_g = 0, soft_cap_v = 0;   // problems the scratch holds
};

namespace {
std::mutex g_err_mu;
std::string g_last_error;

int fail(towr_gpu_handle h, int code, const std::string& msg) {
  if (h) h->err = msg;
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_last_error = msg;
  return code;
}

#define HIPCHK(h, expr)                                                                         \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return fail((h), TOWR_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
  } while (0)

// Every kernel launch of the engine. With TOWR_GPU_LAUNCH_LOG set (read once), the first launch of each (kernel, block,
// dynamic LDS) is written to stderr as "towr-launch <symbol> block <threads> lds <bytes> grid <blocks>": the dynamic
// LDS is a host-side choice the code object does not record, so tools/kernel_resources.py joins these lines with the
// code objects' register / scratch metadata into profiles/kernel_resources.txt (occupancy per launch).
#ifdef TOWR_STAMPS
// experiment build (tools/stamps.py): launch i after towr_gpu_debug_stamps(buf) stores its TG_STAMP slots in region i
// of buf (kStampRegion slots each, kStampRegions regions); the kernel of each region is kept for the tool
constexpr size_t kStampRegion = size_t(1) << 21;
constexpr int kStampRegions = 12;
unsigned long long* g_stamps = nullptr;
int g_stamp_n = 0;
const void* g_stamp_fn[kStampRegions];
#endif
bool launch_log_on() { static const bool log = std::getenv("TOWR_GPU_LAUNCH_LOG") != nullptr; return log; }
hipError_t launch_kernel(const void* fn, dim3 grid, dim3 block, void** args, size_t lds, hipStream_t s) {
#ifdef TOWR_STAMPS
  if (g_stamps && g_stamp_n < kStampRegions && (size_t)grid.x * 64 <= kStampRegion) {
    static_cast<KParams*>(args[0])->stamps = g_stamps + kStampRegion * g_stamp_n;   // every kernel's first argument
    g_stamp_fn[g_stamp_n++] = fn;
  }
#endif
  if (launch_log_on()) {
    static std::mutex mu;
    static std::vector<std::pair<const void*, std::pair<unsigned, size_t>>> seen;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(fn, std::make_pair(block.x, lds));
    if (std::find(seen.begin(), seen.end(), key) == seen.end()) {
      seen.push_back(key);
      const char* nm = hipKernelNameRefByPtr(fn, s);
      std::fprintf(stderr, "towr-launch %s block %u lds %zu grid %u\n", nm ? nm : "?", block.x, lds, grid.x);
    }
  }
  return hipLaunchKernel(fn, grid, block, args, lds, s);
}

template <class T>
int upload(towr_gpu_handle h, T** dst, const std::vector<T>& src) {
  const size_t bytes = sizeof(T) * (src.empty() ? 1 : src.size());
  HIPCHK(h, hipMalloc(reinterpret_cast<void**>(dst), bytes));
  if (!src.empty()) HIPCHK(h, hipMemcpy(*dst, src.data(), sizeof(T) * src.size(), hipMemcpyHostToDevice));
  return TOWR_OK;
}

// a copy padded to whole 16-byte units (k elements), for a kernel that stages it with 16-byte loads
template <class T>
std::vector<T> padded(const std::vector<T>& v, size_t k) {
  std::vector<T> out(v);
  out.resize((v.size() + k - 1) / k * k, T{});
  return out;
}

// the cost kernel's slot-id table as it stages it: cost_nslot entries (padding included) in 16-byte units
std::vector<uint16_t> cost_slot_table(const Layout& L) {
  std::vector<uint16_t> t(L.cost_cslot);
  t.resize(std::max(t.size(), (size_t)L.cost_nslot), 0);
  return padded(t, 8);
}

// every evaluation entry point: refuse layout-only handles, make the handle's device current
int bind(towr_gpu_handle h) {
  if (h->device < 0) return fail(h, TOWR_ERR_NO_DEVICE, "layout-only handle (created with device < 0) cannot evaluate");
  if (hipSetDevice(h->device) != hipSuccess) return fail(h, TOWR_ERR_HIP, "hipSetDevice failed");
  return TOWR_OK;
}

// Handle scratch ordering (see towr_gpu_handle_s::scr_ev): acquire before a call's first use on stream s,
// release after its last; grow() reallocates a per-problem buffer once every earlier use has finished.
int scratch_acquire(towr_gpu_handle h, hipStream_t s) {
  if (h->scr_used && h->scr_stream != s) HIPCHK(h, hipStreamWaitEvent(s, h->scr_ev, 0));
  return TOWR_OK;
}
int scratch_release(towr_gpu_handle h, hipStream_t s) {
  if (h->sync_call) {   // synchronised before the entry point returns: no later call needs to wait for it
    h->scr_used = false;
    return TOWR_OK;
  }
  HIPCHK(h, hipEventRecord(h->scr_ev, s));
  h->scr_stream = s;
  h->scr_used = true;
  return TOWR_OK;
}
int scratch_grow(towr_gpu_handle h, double** buf, int64_t* cap, int64_t problems, int64_t doubles_per_problem) {
  if (*cap >= problems) return TOWR_OK;
  if (*buf) {
    if (h->scr_used) HIPCHK(h, hipEventSynchronize(h->scr_ev));
    (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
  }
  HIPCHK(h, hipMalloc(buf, sizeof(double) * (size_t)problems * (size_t)std::max<int64_t>(1, doubles_per_problem)));
  *cap = problems;
  return TOWR_OK;
}

// The PhaseSpline tables a tile block stages in LDS under phase-duration optimisation, as one blob of
// 16-byte aligned sections [SplineMeta | SchedInfo | PolyPhase | pact | PhaseCol] (~18 KB for ANYmal):
// the device-side duration searches (phase_spline_locate, sched_jac) and the full-pattern window
// emission (emit_dim) walk them in dependent loads, ~10x cheaper from LDS than from L2.
// Behind the tables, each block computes the x-dependent timings of Ctx::pdur / pend / phend
// (n_time doubles: 2 per PolyPhase entry + ph_stride per endeffector).
struct GaitTables { int32_t off[5]; int32_t n16; int32_t n_time, ph_stride; };
GaitTables gait_tables(const Layout& L) {
  GaitTables g{};
  for (const SchedInfo& si : L.sched) g.ph_stride = std::max(g.ph_stride, (int32_t)si.n_phases);
  g.n_time = L.gait ? (int32_t)(2 * L.pinfo.size() + L.sched.size() * g.ph_stride) : 0;
  const size_t sz[5] = {sizeof(SplineMeta) * L.spl.size(), sizeof(SchedInfo) * L.sched.size(), sizeof(PolyPhase) * L.pinfo.size(),
                        sizeof(int32_t) * L.pact.size(), sizeof(PhaseCol) * L.pcols.size()};
  size_t o = 0;
  for (int k = 0; k < 5; ++k) { g.off[k] = (int32_t)o; o += (sz[k] + 15) & ~(size_t)15; }
  g.n16 = L.gait ? (int32_t)(o / 16) : 0;
  return g;
}
std::vector<uint4> gait_blob(const Layout& L) {
  const GaitTables g = gait_tables(L);
  std::vector<uint4> b((size_t)std::max(1, g.n16));
  std::memset(b.data(), 0, b.size() * sizeof(uint4));
  char* p = reinterpret_cast<char*>(b.data());
  if (g.n16 == 0) return b;
  std::memcpy(p + g.off[0], L.spl.data(), sizeof(SplineMeta) * L.spl.size());
  std::memcpy(p + g.off[1], L.sched.data(), sizeof(SchedInfo) * L.sched.size());
  std::memcpy(p + g.off[2], L.pinfo.data(), sizeof(PolyPhase) * L.pinfo.size());
  std::memcpy(p + g.off[3], L.pact.data(), sizeof(int32_t) * L.pact.size());
  std::memcpy(p + g.off[4], L.pcols.data(), sizeof(PhaseCol) * L.pcols.size());
  return b;
}

const void* kernel_for_class(int lc, bool gait, bool rotvec, bool streamed = false) {
  if (streamed) return gait_compose_kernel(15);   // the composer launch; the record kernel: gait_rec_kernel
  if (lc == LC_MISC) return misc_kernel_for(gait);
  return tile_kernel_for(class_type(lc), gait, rotvec);
}

// LDS of a launch class: [tile region(s) | x + zero slot | node table | GAIT: PhaseSpline tables]
// (the streaming ForceConstraintDiscretized path: its per-instant records and row template first)
bool fstream_class(const Layout& L, int lc) { return lc == LC_FDISC && L.fstream; }
int gstream_cls(const Layout& L, int lc) {   // the streaming class of launch class lc, or -1
  if (lc == LC_ROM && L.gstream[GS_ROM]) return GS_ROM;
  if (lc == LC_DYN && L.gstream[GS_DYN]) return GS_DYN;
  if (lc == LC_TQDISC && L.gstream[GS_TQ]) return GS_TQ;
  return -1;
}
bool streamed_class(const Layout& L, int lc) { return fstream_class(L, lc) || gstream_cls(L, lc) >= 0; }
// LDS of the composer launch: its largest compose block
size_t lds_bytes(const Layout& L, int lc);
int class_units(const Layout& L, int lc);
size_t compose_lds(const Layout& L, bool f = true, bool r = true, bool d = true, bool misc = true, bool t = true) {
  size_t b = L.fstream && f ? fs_compose_lds(L) : 0;
  if (L.gstream[GS_ROM] && r) b = std::max(b, gs_stream_lds(L, GS_ROM));
  if (L.gstream[GS_DYN] && d) b = std::max(b, gs_stream_lds(L, GS_DYN));
  if (L.gstream[GS_TQ] && t) b = std::max(b, gs_stream_lds(L, GS_TQ));
  if (misc && class_units(L, LC_MISC) > 0) b = std::max(b, lds_bytes(L, LC_MISC));   // small-kind groups (small batches)
  return b;
}
size_t lds_region(const Layout& L, int lc) {
  if (streamed_class(L, lc)) return compose_lds(L, true, true, true, false) / sizeof(double);
  return lc == LC_MISC ? (size_t)((L.misc_region + 1) & ~1) : (size_t)L.type_lds[class_type(lc)];
}
int class_block(const Layout& L, int lc) {
  if (streamed_class(L, lc)) return kComposeBlock;
  return lc == LC_MISC ? 64 * kMiscWaves : L.type_block[class_type(lc)];
}
size_t lds_bytes(const Layout& L, int lc) {
  if (streamed_class(L, lc)) return compose_lds(L);   // the composer (its small-kind groups stage x)
  size_t d = lds_region(L, lc);
  d += (size_t)((L.n + 2) & ~1);                                                                  // x + zero slot
  if (lc == LC_MISC || stages_nodes(class_type(lc), L.gait)) d += (L.nodecol.size() + 3) / 4 * 2;  // node table (16-B units)
  if (lc != LC_MISC && L.gait)   // PhaseSpline tables, timings, terrain
    d += (size_t)gait_tables(L).n16 * 2 + gait_tables(L).n_time + (sizeof(towr_terrain_t) + 15) / 16 * 2;
  return sizeof(double) * d;
}
int class_units(const Layout& L, int lc) {   // tiles (or misc groups, or FsBlocks) per problem
  if (lc == LC_MISC) return (int)(L.misc_tiles.size() / kMiscWaves);
  if (fstream_class(L, lc)) return (int)L.fs_blocks.size();
  if (gstream_cls(L, lc) >= 0) return (int)L.gs_blocks[gstream_cls(L, lc)].size();
  const int t = class_type(lc);
  return L.type_tile0[t + 1] - L.type_tile0[t];
}
int64_t class_bytes(const Layout& L, int lc) { return lc == LC_MISC ? L.misc_bytes : L.type_bytes[class_type(lc)]; }
// the streaming path's instant kernel (A): [x + zero slot | node table | PhaseSpline tables | timings | terrain]
size_t fs_inst_lds_bytes(const Layout& L) {
  return sizeof(double) * ((size_t)((L.n + 2) & ~1) + (L.nodecol.size() + 3) / 4 * 2 + (size_t)gait_tables(L).n16 * 2 +
                           gait_tables(L).n_time + (sizeof(towr_terrain_t) + 15) / 16 * 2);
}

// RangeOfMotion + ForceConstraintDiscretized in one launch (both 192-lane, their registers and LDS
// allow 3 blocks per CU either way). Measured on MI355X (ANYmal, B = 4096, 3 alternating runs each):
// per-class 0.269-0.275 ms per step, "rf" 0.263-0.268 ms; adding Dynamic + small kinds as a second
// group ("rf,dm") 0.285 ms, the small kinds into the first ("rfm") 0.308 ms, everything ("drftm")
// 0.317 ms: a group inherits its largest class's registers, and Dynamic's 242 VGPRs or a 256-lane
// block cost the others their residency.
constexpr const char* kDefaultFuse = "rf";

// algorithmic bytes per problem of the classes in `mask` launched together: CSR values and g rows
// written + the union of the x columns their Jacobian rows read
int64_t mask_bytes(const Layout& L, uint32_t mask) {
  std::vector<uint8_t> used((size_t)L.n, 0);
  int64_t nv = 0, nr = 0;
  auto add = [&](const TileDesc& td) {
    nv += td.v1 - td.v0; nr += td.r1 - td.r0;
    for (int32_t k = td.v0; k < td.v1; ++k) used[L.col[k]] = 1;
  };
  for (int lc = 0; lc < LC_COUNT; ++lc) {
    if (!((mask >> lc) & 1)) continue;
    if (lc == LC_MISC) {
      for (int32_t ti : L.misc_tiles) if (ti >= 0) add(L.tiles[ti]);
    } else {
      for (int ti = L.type_tile0[class_type(lc)]; ti < L.type_tile0[class_type(lc) + 1]; ++ti) add(L.tiles[ti]);
    }
  }
  int64_t nx = 0;
  for (uint8_t u : used) nx += u;
  return 8 * (nv + nr + nx);
}

// a fusion group's unit table: one round-robin pass over its classes at a time (heaviest writer
// first), so consecutive blocks of a problem alternate latency-bound and write-bound units
std::vector<UnitDesc> fused_units(const Layout& L, uint32_t mask) {
  static const int order[] = {LC_FDISC, LC_DYN, LC_ROM, LC_TQDISC, LC_MISC};
  std::vector<UnitDesc> u;
  int left[LC_COUNT];
  for (int lc = 0; lc < LC_COUNT; ++lc) left[lc] = (mask >> lc) & 1 ? class_units(L, lc) : 0;
  for (bool any = true; any;) {
    any = false;
    for (int lc : order) {
      if (left[lc] == 0) continue;
      const int k = class_units(L, lc) - left[lc]--;
      UnitDesc d{};
      d.lc = lc;
      d.tile = lc == LC_MISC ? k : L.type_tile0[class_type(lc)] + k;
      d.lds_x_off = (int32_t)lds_region(L, lc);
      d.lds_rows_off = lc == LC_MISC ? 0 : L.type_lds_rows_off[class_type(lc)];   // small kinds: misc_lds
      if (lc != LC_MISC) d.t = L.tiles[d.tile];
      u.push_back(d);
      any = true;
    }
  }
  return u;
}

void fill_common(towr_gpu_handle h, KParams& P, int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V,
                 int64_t ldv, int want_g, int want_jac, const towr_terrain_t* terrains, int per_problem) {
  const Layout& L = h->L;
  P.X = X; P.ldx = ldx; P.G = G; P.ldg = ldg; P.V = V; P.ldv = ldv;
  P.items = h->d_items; P.slots = h->d_slots; P.tiles = h->d_tiles;
  P.nodecol = h->d_nodecol; P.spl = h->d_spl; P.dur = h->d_dur;
  P.sg = h->sg; P.n_spl = (int32_t)L.spl.size();
  P.pinfo = h->d_pinfo; P.pcols = h->d_pcols; P.pact = h->d_pact; P.sched = h->d_sched; P.eelin = h->d_eelin; P.lin = h->d_lin;
  P.terrains = terrains; P.terrain_per_problem = per_problem;
  P.B = B;
  P.n = L.n; P.n_pad = (L.n + 2) & ~1; P.n_nodecol = (int32_t)L.nodecol.size();
  P.want_g = want_g; P.want_jac = want_jac; P.fdisc_motion = L.fdisc_motion;
  P.rb = L.rb;
  P.misc_tiles = h->d_misc; P.misc_lds = h->d_misc_lds; P.misc_wave = h->d_misc_wave; P.misc_items = h->d_misc_items;
  P.xspan = h->d_xspan; P.n_xspan = (int32_t)(L.misc_xspan.size() / 2);
  P.lds_scr_off = L.dyn_scr_off;
  P.rvc = h->d_rvc; P.rvi = h->d_rvi; P.n_rvi = (int32_t)L.rv_inst.size();
  const GaitTables gt = gait_tables(L);
  P.gtab = h->d_gtab;
  P.idir = h->d_idir;
  for (int k = 0; k < 5; ++k) P.gt_off[k] = gt.off[k];
  P.gt_n16 = gt.n16;
  P.n_pinfo = (int32_t)L.pinfo.size();
  P.ph_stride = gt.ph_stride;
  P.gt_ntime = gt.n_time;
  P.fsb = h->d_fsb; P.fs_t = h->d_fs_t; P.fs_tmpl = h->d_fs_tmpl; P.fs_ws = h->d_fs_ws;
  P.fs_iee = h->d_fs_iee; P.fs_irow = h->d_fs_irow; P.fs_iblk = h->d_fs_iblk;
  P.gs_geo = h->d_gs_geo; P.gs_tmpl = h->d_gs_tmpl; P.gs_pcode = h->d_gs_pcode;
  P.gs_segs = h->d_gs_segs; P.gs_tseg = h->d_gs_tseg; P.gs_vmap = h->d_gs_vmap; P.gs_ws = h->d_gs_ws; P.gs_blob = h->d_gs_blob;
}

// Fixed gait, RotVec: the pre-pass of the Dynamic base-angular coefficients (tiles.hip towr_rv_coef_kernel)
// into the handle's scratch, on the stream of the Dynamic launch that follows it (every launch holding the
// Dynamic class: its tile kernel, a fusion group, the single-problem group). Without the Jacobian only the
// base terms of the g rows (kRvAb).
int launch_rv_prepass(towr_gpu_handle h, int B, const double* X, int64_t ldx, int want_jac, hipStream_t s) {
  const Layout& L = h->L;
  const int64_t K = (int64_t)L.rv_inst.size();
  if (K == 0 || B <= 0) return TOWR_OK;
  if (int rc = scratch_grow(h, &h->d_rvc, &h->rvc_cap, B + 64, kRvCoef * K)) return rc;   // whole 64-pair blocks (rv_at)
  KParams P{};
  P.X = X; P.ldx = ldx; P.B = B;
  P.nodecol = h->d_nodecol; P.spl = h->d_spl; P.dur = h->d_dur; P.sg = h->sg; P.terrains = h->d_terrain;
  P.rb = L.rb; P.rvc = h->d_rvc; P.rvi = h->d_rvi; P.n_rvi = (int32_t)K; P.want_jac = want_jac;
  const int64_t waves = 3 * (((int64_t)B * K + 63) / 64), grid = (waves + kRvCoefBlock / 64 - 1) / (kRvCoefBlock / 64);
  if (grid > INT32_MAX) return fail(h, TOWR_ERR_INVALID, "batch too large");
  void* args[] = {&P};
  HIPCHK(h, launch_kernel(rv_coef_kernel(), dim3((unsigned)grid), dim3(kRvCoefBlock), args, 0, s));
  return TOWR_OK;
}

int launch_fused(towr_gpu_handle h, const towr_gpu_handle_s::FuseGroup& fg, int B, const double* X, int64_t ldx, double* G,
                 int64_t ldg, double* V, int64_t ldv, int want_g, int want_jac, hipStream_t s,
                 const towr_terrain_t* terrains, int per_problem) {
  const Layout& L = h->L;
  if ((fg.mask >> LC_DYN) & 1)
    if (int rc = launch_rv_prepass(h, B, X, ldx, want_jac, s)) return rc;
  KParams P{};
  fill_common(h, P, B, X, ldx, G, ldg, V, ldv, want_g, want_jac, terrains, per_problem);
  P.units = fg.d_units; P.n_units = fg.n_units;
  const int64_t total = (int64_t)B * fg.n_units;
  const int64_t grid = ((total + 7) / 8) * 8;
  if (grid > INT32_MAX) return fail(h, TOWR_ERR_INVALID, "batch too large");
  void* args[] = {&P};
  HIPCHK(h, launch_kernel(step_kernel_for(L.gait, L.rotvec, fg.kblock), dim3((unsigned)grid), dim3((unsigned)fg.kblock),
                            args, fg.lds, s));
  return TOWR_OK;
}

// The record kernel (both RangeOfMotion / Dynamic, one block per problem): its LDS is the staging of
// fs_inst_lds_bytes, one base-angular converter state per Dynamic instant, then the Dynamic scratch
// (9 doubles per instant and per (endeffector, instant)); its lanes, whole waves per kind (gstream.hip).
int64_t gs_kd(const Layout& L) { return L.gstream[GS_DYN] ? (int64_t)L.gs_inst[GS_DYN].size() : 0; }
size_t gs_state_stride(const Layout& L) { return (gs_dyn_state_bytes(L.rotvec) + 15) & ~(size_t)15; }
size_t gs_rec_lds(const Layout& L) {
  const size_t Kd = (size_t)gs_kd(L);
  return fs_inst_lds_bytes(L) + Kd * gs_state_stride(L) + sizeof(double) * 9 * Kd * (1 + (size_t)L.rb.n_ee);
}
// LDS of one record launch (bytes), used at the launch and at handle creation: the staging (fs_inst_lds_bytes), with
// a Dynamic part also its states and scratch (gs_rec_lds). A launch with the FDISC part and no RangeOfMotion /
// Dynamic part stages the FDISC tables (FsBlock, window, template) after that region when they fit in 160 kB
// (*fs_lds: their byte offset), else its lanes read them in global memory (*fs_lds = 0).
constexpr size_t kLdsMax = 160 * 1024;
size_t rec_launch_lds(const Layout& L, bool dyn, bool fdisc_only, int32_t* fs_lds) {
  const size_t base = dyn ? gs_rec_lds(L) : fs_inst_lds_bytes(L);
  if (fs_lds) *fs_lds = 0;
  if (!fdisc_only) return base;
  const size_t off = (base + 15) & ~(size_t)15;
  const size_t tabs = 4 * (L.fs_blocks.size() * (sizeof(FsBlock) / 4) + L.fs_ws.size() + L.fs_tmpl.size());
  if (off + tabs > kLdsMax) return base;
  if (fs_lds) *fs_lds = (int32_t)off;
  return off + tabs;
}
int gs_rec_threads(const Layout& L, int64_t Kd, int64_t Kr) {   // the record lanes of Kd Dynamic and Kr RangeOfMotion instants
  const int64_t ee0 = (Kd + 63) & ~63, r0 = (ee0 + 3 * L.rb.n_ee * Kd + 63) & ~63;
  const int64_t lanes = std::max<int64_t>(r0 + Kr, 4 * ((Kd + 63) & ~63));
  return (int)std::min<int64_t>(kGsRecMaxBlock, std::max<int64_t>(64, (lanes + 63) & ~63));
}

// The streaming path under phase-duration optimisation (gstream.hip) for the streamed classes in
// `mask` (bits LC_FDISC, LC_TQDISC, LC_ROM, LC_DYN; LC_MISC: the small kinds may join the composer launch):
//   records: the FDISC / TQDISC records and the RangeOfMotion / Dynamic records (towr_gait_rec_kernel, one
//            block per problem and record part, RecPart) into the handle's record scratch; they write g;
//   compose: the compose blocks of the classes (towr_gait_compose_kernel), each CSR range written once.
// Only the classes in `mask` are recorded (a single-class launch records nothing else).
// A batch of kSplitBatch problems or more runs as two chains (one after the other without a side stream,
// TOWR_GPU_STREAMS=1): FDISC + TQDISC records + their compose launch on the high-priority side stream 0 beside
// the RangeOfMotion / Dynamic records + the Dynamic and RangeOfMotion compose launches on the caller's stream, so
// that the write-bound FDISC compose overlaps the latency-bound record work (MI355X, ANYmal gait, B = 1024, one
// box, round 3: 0.600-0.608 ms per step; one chain 0.663, records in 256-problem chunks pipelined against the
// compose 0.737, Dynamic + RangeOfMotion in one compose launch 0.640). With TQDISC and a second side stream it is
// a third chain (below). The caller joins the side streams after its other launches (*forked). A smaller
// batch (B = 1: IPOPT's callbacks) is two launches on the caller's stream: every record part in one, every compose role and the
// small-kind groups in the other (*misc_done) — at B = 1 a launch boundary or a cross-stream event costs
// more than any overlap gains (MI355X, ANYmal gait: 97 us for the per-class chains, 70 us for four launches
// on one stream).
constexpr int kSplitBatch = 64;
#ifndef TOWR_FS_GROUP   // (experiment builds: -DTOWR_FS_GROUP / -DTOWR_TQ_GROUP)
#define TOWR_FS_GROUP 4
#endif
#ifndef TOWR_TQ_GROUP
#define TOWR_TQ_GROUP kGsGroup
#endif
constexpr int kFsGroup = TOWR_FS_GROUP, kTqGroup = TOWR_TQ_GROUP;
bool compose_lds_attr(size_t lds) {   // every composer instantiation may take `lds` bytes of LDS
  for (int m = 1; m < 32; ++m)
    if (hipFuncSetAttribute(gait_compose_kernel(m), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return false;
  return true;
}
// per-problem record doubles: [FDISC instants | TQDISC records] and [RangeOfMotion | Dynamic]
int64_t fs_rec_doubles(const Layout& L) { return fs_record_doubles() * (int64_t)L.fs_t.size(); }
int64_t frec_ld(const Layout& L) { return fs_rec_doubles(L) + (L.gstream[GS_TQ] ? gs_record_doubles(L, GS_TQ) : 0); }
int launch_stream_path(towr_gpu_handle h, KParams P, uint32_t mask, hipStream_t st, bool* forked, bool* misc_done) {
  const Layout& L = h->L;
  const int B = P.B;
  const bool fs = L.fstream && ((mask >> LC_FDISC) & 1), tq = L.gstream[GS_TQ] && ((mask >> LC_TQDISC) & 1);
  const bool gr = L.gstream[GS_ROM] && ((mask >> LC_ROM) & 1), gd = L.gstream[GS_DYN] && ((mask >> LC_DYN) & 1);
  const int32_t ni = (int32_t)L.fs_t.size();
  const int64_t fldr = frec_ld(L), tq_off = fs_rec_doubles(L);
  const int64_t lr = L.gstream[GS_ROM] ? gs_record_doubles(L, GS_ROM) : 0, ld = L.gstream[GS_DYN] ? gs_record_doubles(L, GS_DYN) : 0;
  if (fs || tq)
    if (int rc = scratch_grow(h, &h->d_fsrec, &h->fsrec_cap, B, fldr)) return rc;
  if (gr || gd)
    if (int rc = scratch_grow(h, &h->d_gsrec, &h->gsrec_cap, B, lr + ld)) return rc;
  const bool big = B >= kSplitBatch;
  const bool split = (fs || tq) && (gr || gd) && h->n_side > 0 && big;
  const bool misc = !big && ((mask >> LC_MISC) & 1) && class_units(L, LC_MISC) > 0;
  // two chains: the FDISC / TQDISC chain (the longer one, and its compose cannot start before its records) on
  // the high-priority side stream 0, the RangeOfMotion / Dynamic chain and what follows on the caller's stream.
  // At equal priority the FDISC record blocks waited for CU slots behind the other chain's blocks: the record
  // launch took 299 us instead of 75 us (rocprofv3 kernel trace, ANYmal gait, B = 1024) and the FDISC compose
  // started only after the other chain had finished.
  // (round 5: the chains swapped, FDISC on the caller's stream so that the step's last launch and the next step's first
  // share a stream, the RangeOfMotion / Dynamic chain on side 0 at the default / least priority (HIP range 1 .. -1):
  // ANYmal gait, B = 1024, one box, 4 runs: 0.623-0.648 / 0.656-0.659 vs 0.611-0.614 ms, + Torque 1.227-1.233 /
  // 1.223-1.227 vs 1.163-1.171; gpurun_out/r05r_ab.log)
  const hipStream_t fst = split ? h->side[0] : st;   // the FDISC / TQDISC chain
  const hipStream_t gst = st;                        // the RangeOfMotion / Dynamic chain
  // with a second side stream, TQDISC (records + compose) is a third chain: its compose is as long as FDISC's
  // (ANYmal gait + Torque, B = 1024: 1.7 GB vs 1.46 GB of values), and behind FDISC's in one chain it was the step
  // (measured: ANYmal gait + Torque, B = 1024, one box: 1.206 ms per step with three chains, 1.233 with TQDISC
  // behind FDISC in one chain)
  const bool tq3 = split && tq && fs && h->n_side > 1;
  const hipStream_t tst = tq3 ? h->side[1] : fst;
  // (round 6, ANYmal gait, B = 1024, one box, 3 runs each: a second side stream for the non-Torque gait, carrying the
  // small kinds beside the records, or the RangeOfMotion composer beside the Dynamic composer, or the RangeOfMotion /
  // Dynamic records at the greatest priority: 0.590-0.613 ms per step, all within the product's 0.589-0.606. The kernel
  // trace shows why: the RangeOfMotion / Dynamic records finish at 144 us in one step and at 413 us in the next, behind
  // the FDISC composer's blocks, and the composers that follow are bandwidth-bound together whichever way they overlap.)
  if (split) {
    HIPCHK(h, hipEventRecord(h->fork, st));
    HIPCHK(h, hipStreamWaitEvent(fst, h->fork, 0));
    if (tq3) HIPCHK(h, hipStreamWaitEvent(tst, h->fork, 0));
  }
  RecArgs R{};
  R.frec = h->d_fsrec; R.fldr = fldr; R.tq_off = tq_off; R.ni = fs ? ni : 0;
  R.g.rec = h->d_gsrec; R.g.ldr = lr + ld; R.g.dyn_off = lr;
  for (int c = 0; c < GS_COUNT; ++c) R.g.inst[c] = h->d_gs_inst[c];
  R.g.K[GS_ROM] = gr ? (int32_t)L.gs_inst[GS_ROM].size() : 0;
  R.g.K[GS_DYN] = gd ? (int32_t)L.gs_inst[GS_DYN].size() : 0;
  R.g.K[GS_TQ] = tq ? (int32_t)L.gs_inst[GS_TQ].size() : 0;
  R.g.st_off = (int32_t)(fs_inst_lds_bytes(L) / sizeof(double));
  R.g.scr_off = R.g.st_off + (int32_t)(gs_kd(L) * gs_state_stride(L) / sizeof(double));
  // one block per (problem, part); threads: the parts' lanes in whole waves (FDISC / TQDISC one per instant,
  // the RangeOfMotion / Dynamic parts gs_rec_threads), at most kGsRecMaxBlock; LDS: the staging
  // (fs_inst_lds_bytes), with a RangeOfMotion / Dynamic part also its states and scratch (gs_rec_lds)
  auto records = [&](std::initializer_list<int> parts, hipStream_t s) -> int {
    R.nparts = 0; R.parts = 0;
    int roles = 0;
    int64_t lanes = 64;
    bool dyn = false;   // a part with Dynamic lanes: the converter states and sums in LDS (gs_rec_lds)
    for (int p : parts) {
      if (p == 0) continue;
      R.parts |= p << (4 * R.nparts++);
      roles |= p == kRecFdisc ? 1 : p == kRecTq ? 4 : 2;
      dyn = dyn || ((p == kRecGs || p == kRecGsDyn) && R.g.K[GS_DYN] > 0);
      lanes = std::max<int64_t>(lanes, p == kRecFdisc ? R.ni : p == kRecTq ? R.g.K[GS_TQ] : gs_rec_threads(L, R.g.K[GS_DYN], R.g.K[GS_ROM]));
    }
    if (R.nparts == 0) return TOWR_OK;
    const int threads = (int)std::min<int64_t>(kGsRecMaxBlock, (lanes + 63) & ~63);
    // the FDISC launch (no RangeOfMotion / Dynamic part) stages the FDISC tables after its staging region when they
    // fit, so its lanes' table reads after the instant (block, window start, template) are LDS reads
    const size_t lds = rec_launch_lds(L, dyn, (roles & 1) && !(roles & 2), &R.fs_lds);
    R.fs_nb = (int32_t)(L.fs_blocks.size() * (sizeof(FsBlock) / 4));
    R.fs_nws = (int32_t)L.fs_ws.size();
    R.fs_ntm = (int32_t)L.fs_tmpl.size();
    void* aa[] = {&P, &R};
    HIPCHK(h, launch_kernel(gait_rec_kernel(L.rotvec, roles), dim3((unsigned)(B * R.nparts)), dim3((unsigned)threads), aa, lds, s));
    return TOWR_OK;
  };
  ComposeArgs C{};
  C.frec = h->d_fsrec; C.fldr = fldr; C.tq_off = tq_off;
  C.grec = h->d_gsrec; C.gldr = lr + ld; C.gdyn_off = lr;
  for (int c = 0; c < GS_COUNT; ++c) C.blk[c] = h->d_gs_blk[c];
  C.ng = (B + kGsGroup - 1) / kGsGroup;
  C.misc_x_off = (int32_t)lds_region(L, LC_MISC);
  auto compose = [&](bool f, bool t, bool r, bool d, bool m, hipStream_t s) -> int {
    const bool j = P.want_jac != 0;   // without the Jacobian only the small kinds (their g rows)
    C.nt[0] = f && j ? (int32_t)L.fs_blocks.size() : 0;
    C.nt[1] = r && j ? (int32_t)L.gs_blocks[GS_ROM].size() : 0;
    C.nt[2] = d && j ? (int32_t)L.gs_blocks[GS_DYN].size() : 0;
    C.nt[3] = m ? class_units(L, LC_MISC) : 0;
    C.nt[4] = t && j ? (int32_t)L.gs_blocks[GS_TQ].size() : 0;
    // problems per block: kGsGroup; a launch of FDISC blocks only: kFsGroup (the next problem's records prefetched while
    // one streams, so a block with more problems keeps its trips going longer; MI355X, ANYmal gait, B = 1024, one box,
    // 3 runs, gait / + Torque ms: 2 0.596-0.598 / 1.163-1.167; 4 0.587-0.592 / 1.146-1.149; 8 0.585-0.593 / 1.151-1.157)
    // and of TQDISC blocks only: kTqGroup (4: + Torque 1.161-1.163 vs 1.145-1.150; 1: 1.185-1.193)
    const bool fonly = C.nt[0] > 0 && C.nt[1] + C.nt[2] + C.nt[3] + C.nt[4] == 0;
    const bool tonly = C.nt[4] > 0 && C.nt[0] + C.nt[1] + C.nt[2] + C.nt[3] == 0;
    const int grp = fonly ? kFsGroup : tonly ? kTqGroup : kGsGroup;
    C.ng = (B + grp - 1) / grp;
    const int64_t units = (int64_t)C.nt[0] + C.nt[1] + C.nt[2] + C.nt[3] + C.nt[4];
    const int64_t grid = ((int64_t)C.ng * units + 7) / 8 * 8;   // whole rounds of 8 (XCD-aware mapping)
    if (grid == 0) return TOWR_OK;
    if (grid > INT32_MAX) return fail(h, TOWR_ERR_INVALID, "batch too large");
    void* ab[] = {&P, &C};
    // the launch's own roles: their instantiation (registers) and LDS; without FDISC, TQDISC or small kinds 256 threads
    const int roles = (C.nt[0] ? 1 : 0) | (C.nt[1] ? 2 : 0) | (C.nt[2] ? 4 : 0) | (C.nt[3] ? 8 : 0) | (C.nt[4] ? 16 : 0);
    HIPCHK(h, launch_kernel(gait_compose_kernel(roles), dim3((unsigned)grid), dim3(compose_block(roles)), ab,
                              compose_lds(L, C.nt[0] > 0, C.nt[1] > 0, C.nt[2] > 0, C.nt[3] > 0, C.nt[4] > 0), s));
    return TOWR_OK;
  };
  const int fpart = fs ? kRecFdisc : 0;
  if (big) {   // (without a side stream the two chains run one after the other on the caller's stream)
    if (tq3) {
      if (int rc = records({kRecTq}, tst)) return rc;
      if (int rc = compose(false, true, false, false, false, tst)) return rc;
    }
    const bool tqf = tq && !tq3;   // TQDISC in the FDISC chain
    if (fs || tqf) {
      // (the FDISC records in two blocks per problem, each half the instants: 0.638 vs 0.629 ms, not kept)
      if (int rc = records({fpart, tqf ? kRecTq : 0}, fst)) return rc;
      if (int rc = compose(fs, tqf, false, false, false, fst)) return rc;
    }
    if (gr || gd) {
      // one block per problem: two blocks (Dynamic | RangeOfMotion lanes) in one launch or in two launches
      // measured slower (ANYmal gait, B = 1024, one box: 0.676 / 0.675 vs 0.645 / 0.660 ms per step)
      if (int rc = records({kRecGs}, gst)) return rc;
      if (int rc = compose(false, false, false, gd, false, gst)) return rc;
      if (int rc = compose(false, false, gr, false, false, gst)) return rc;
    }
  } else {   // every record part in one launch (RangeOfMotion and Dynamic in two blocks beside FDISC: shorter chains per CU)
    const bool two = gr && gd && (fs || tq);
    if (int rc = records({fpart, tq ? kRecTq : 0, two ? kRecGsDyn : (gr || gd) ? kRecGs : 0, two ? kRecGsRom : 0}, st)) return rc;
    if (int rc = compose(fs, tq, gr, gd, misc, st)) return rc;
  }
  *forked = split;   // the caller joins side stream 0 (and 1) after its other launches (which follow on its own stream)
  *misc_done = misc;
  return TOWR_OK;
}

bool gait_streamed(const Layout& L) { return L.fstream || L.gstream[GS_ROM] || L.gstream[GS_DYN] || L.gstream[GS_TQ]; }
bool uses_scratch(const Layout& L) { return gait_streamed(L) || !L.rv_inst.empty(); }

int launch_classes(towr_gpu_handle h, int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V, int64_t ldv,
                   int want_g, int want_jac, hipStream_t s, const towr_terrain_t* terrains, int per_problem, int only_class);
int launch(towr_gpu_handle h, int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V, int64_t ldv,
           int want_g, int want_jac, hipStream_t s, const towr_terrain_t* terrains, int per_problem, int only_class) {
  if (B <= 0) return TOWR_OK;
  const bool scr = uses_scratch(h->L);
  if (scr)
    if (int rc = scratch_acquire(h, s)) return rc;
  if (int rc = launch_classes(h, B, X, ldx, G, ldg, V, ldv, want_g, want_jac, s, terrains, per_problem, only_class)) {
    // a failure after the streaming path forked its side stream: join every side stream into s and still
    // order the scratch, so that later calls (and scratch_grow's hipFree) wait for the kernels already queued
    for (int i = 0; i < h->n_side; ++i)
      if (hipEventRecord(h->join[i], h->side[i]) == hipSuccess) (void)hipStreamWaitEvent(s, h->join[i], 0);
    if (scr) (void)scratch_release(h, s);
    return rc;
  }
  return scr ? scratch_release(h, s) : TOWR_OK;
}

int launch_classes(towr_gpu_handle h, int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V, int64_t ldv,
                   int want_g, int want_jac, hipStream_t s, const towr_terrain_t* terrains, int per_problem, int only_class) {
  const Layout& L = h->L;
  uint32_t fused_mask = 0;
  // a batch with fusion groups: the other classes on the side streams beside the fused launches (forked before
  // them: the fused launch on the caller's stream, Dynamic then the small kinds on side stream 0); at small B the
  // fork and join cost more than the overlap gains
  // RotVec layouts (per-class launches, no fusion group): RangeOfMotion and FDISC on the caller's stream, the coefficient
  // pre-pass, Dynamic and the small kinds on side stream 0 beside them (h->rv_overlap)
  const bool rv_side = h->rv_overlap && h->n_fuse == 0;
  const bool overlap = only_class < 0 && h->n_side > 0 && (h->n_fuse > 0 || rv_side) && !gait_streamed(L) && B >= kSplitBatch;
  if (overlap) {
    HIPCHK(h, hipEventRecord(h->fork, s));
    for (int i = 0; i < h->n_side; ++i) HIPCHK(h, hipStreamWaitEvent(h->side[i], h->fork, 0));
  }
  if (only_class < 0)
    for (int g = 0; g < h->n_fuse; ++g) {
      if (int rc = launch_fused(h, h->fuse[g], B, X, ldx, G, ldg, V, ldv, want_g, want_jac, s, terrains, per_problem)) return rc;
      fused_mask |= h->fuse[g].mask;
    }
  // The launch classes are independent (disjoint rows and CSR ranges): they may run on the handle's side
  // streams (above, or TOWR_GPU_STREAMS without fusion groups) and join back into the caller's stream. Heaviest first.
  int order[LC_COUNT], nk = 0;
  for (int lc = 0; lc < LC_COUNT; ++lc)
    if (class_units(L, lc) > 0 && !((fused_mask >> lc) & 1) && (only_class < 0 || lc == only_class)) order[nk++] = lc;
  std::sort(order, order + nk, [&](int a, int b) { return class_bytes(L, a) > class_bytes(L, b); });
  // the small kinds last (round 5, ANYmal, B = 4096, one box: before Dynamic on the side stream 0.2365-0.2377 ms per step,
  // after it 0.2359-0.2374)
  std::stable_partition(order, order + nk, [](int lc) { return lc != LC_MISC; });
  // (the streaming path forks its own side stream, see launch_stream_path; the other classes follow it on
  // the caller's stream; a small batch with fusion groups runs serially)
  const int nside = overlap ? h->n_side : (only_class < 0 && nk > 1 && !uses_scratch(L) && h->n_fuse == 0) ? std::min(h->n_side, nk - 1) : 0;
  if (nside > 0 && !overlap) {
    HIPCHK(h, hipEventRecord(h->fork, s));
    for (int i = 0; i < nside; ++i) HIPCHK(h, hipStreamWaitEvent(h->side[i], h->fork, 0));
  }
  bool stream_done = false, stream_forked = false, misc_done = false;
  // one launch of a class that is not streamed (a tile class or the small kinds) on stream st
  auto launch_one = [&](int lc, hipStream_t st) -> int {
    KParams P{};
    fill_common(h, P, B, X, ldx, G, ldg, V, ldv, want_g, want_jac, terrains, per_problem);
    const int nt = class_units(L, lc);
    P.ntiles = nt;
    if (lc == LC_MISC) {
      P.tile0 = 0;
      P.misc_tiles = h->d_misc; P.misc_lds = h->d_misc_lds; P.misc_wave = h->d_misc_wave; P.misc_items = h->d_misc_items;
    } else {
      P.tile0 = L.type_tile0[class_type(lc)];
      P.lds_rows_off = L.type_lds_rows_off[class_type(lc)];
      P.lds_scr_off = L.dyn_scr_off;
    }
    P.n = L.n; P.n_pad = (L.n + 2) & ~1; P.n_nodecol = (int32_t)L.nodecol.size();
    P.lds_x_off = (int32_t)lds_region(L, lc);
    P.want_g = want_g; P.want_jac = want_jac; P.fdisc_motion = L.fdisc_motion;
    P.rb = L.rb;
    const int64_t total = (int64_t)B * nt;
    const int64_t grid = ((total + 7) / 8) * 8;
    if (grid > INT32_MAX) return fail(h, TOWR_ERR_INVALID, "batch too large");
    if (lc == LC_DYN) {
      if (int rc = launch_rv_prepass(h, B, X, ldx, want_jac, st)) return rc;
      P.rvc = h->d_rvc;   // (grown by the pre-pass)
    }
    const int block = class_block(L, lc);
    void* args[] = {&P};
    HIPCHK(h, launch_kernel(kernel_for_class(lc, L.gait, L.rotvec), dim3((unsigned)grid), dim3((unsigned)block), args,
                              lds_bytes(L, lc), st));
    return TOWR_OK;
  };
  for (int q = 0; q < nk; ++q) {
    const int lc = order[q];
    if (lc == LC_MISC && misc_done) continue;   // in the streaming path's composer launch
    const hipStream_t st = stream_forked ? s
                         : overlap ? ((rv_side && lc != LC_DYN && lc != LC_MISC) ? s : h->side[q % nside])
                         : (nside > 0 && q % (nside + 1) != 0) ? h->side[q % (nside + 1) - 1] : s;
    if (streamed_class(L, lc)) {   // every streamed class at the first one: its records and one composer launch
      if (stream_done) continue;
      stream_done = true;
      uint32_t mask = 0;
      for (int k = 0; k < nk; ++k)
        if (streamed_class(L, order[k]) || order[k] == LC_MISC) mask |= 1u << order[k];   // (the small kinds are last)
      KParams P{};
      fill_common(h, P, B, X, ldx, G, ldg, V, ldv, want_g, want_jac, terrains, per_problem);
      P.ntiles = class_units(L, lc);
      if (int rc = launch_stream_path(h, P, mask, s, &stream_forked, &misc_done)) return rc;
      continue;
    }
    if (int rc = launch_one(lc, st)) return rc;
  }
  for (int i = 0; i < (stream_forked ? std::min(h->n_side, 2) : nside); ++i) {
    HIPCHK(h, hipEventRecord(h->join[i], h->side[i]));
    HIPCHK(h, hipStreamWaitEvent(s, h->join[i], 0));
  }
  return TOWR_OK;
}

// LDS of the cost launch (doubles): [accumulators | x + zero slot | node table | wave partials, error flag].
// The accumulators (cost_traj.hip): acc 1 = one slot per present gradient entry (Layout::cost_nslot), acc 2 =
// three 64-bit limbs per column, acc 0 (f only) = none.
int cost_acc(const Layout& L, bool grad) { return !grad ? 0 : L.cost_nslot > 0 ? 1 : 2; }
size_t cost_x_off(const Layout& L, int acc) {
  const size_t n_pad = (size_t)((L.n + 2) & ~1);
  return acc == 1 ? (size_t)((L.cost_nslot + 1) & ~1) : acc == 2 ? 3 * n_pad : 0;
}
size_t cost_red_off(const Layout& L, int acc) {   // ... after x and the node table: acc 1's slot tables (16-byte units)
  const size_t tabs = acc == 1 ? 2 * ((size_t)(L.cost_nslot + 7) / 8 + (size_t)(L.n + 8) / 8) : 0;
  return cost_x_off(L, acc) + (size_t)((L.n + 2) & ~1) + (L.nodecol.size() + 3) / 4 * 2 + tabs;
}
size_t cost_lds_bytes(const Layout& L, int acc) { return sizeof(double) * (cost_red_off(L, acc) + kCostBlock / 64 + 2); }

int launch(towr_gpu_handle h, int B, const double* X, int64_t ldx, double* G, int64_t ldg, double* V, int64_t ldv,
           int want_g, int want_jac, hipStream_t s, const towr_terrain_t* terrains, int per_problem, int only_class);

// SoftConstraint terms: the soft child evaluates the wrapped sets' g (and, for the gradient, their
// Jacobian values) of the batch into the handle's scratch, on the same stream, before the cost launch
int launch_soft(towr_gpu_handle h, int B, const double* X, int64_t ldx, bool grad, hipStream_t s,
                const towr_terrain_t* terrains, int per_problem, KParams& P) {
  towr_gpu_handle c = h->soft;
  const int64_t ms = std::max(1, c->L.m), nzs = std::max<int64_t>(1, c->L.nnz);
  if (int rc = scratch_grow(h, &h->d_sg, &h->soft_cap_g, B, ms)) return rc;
  if (grad)
    if (int rc = scratch_grow(h, &h->d_sv, &h->soft_cap_v, B, nzs)) return rc;
  if (int rc = launch(c, B, X, ldx, h->d_sg, ms, grad ? h->d_sv : nullptr, nzs, 1, grad ? 1 : 0, s, terrains, per_problem, -1))
    return fail(h, rc, "SoftConstraint sets: " + c->err);
  P.sG = h->d_sg; P.s_ldg = ms; P.sV = h->d_sv; P.s_ldv = nzs;
  P.s_cptr = h->d_soft_cptr; P.s_cent = h->d_soft_cent; P.s_b = h->d_soft_b; P.s_m = c->L.m;
  return TOWR_OK;
}

int launch_cost(towr_gpu_handle h, int B, const double* X, int64_t ldx, double* F, double* GR, int64_t ldgr,
                hipStream_t s, const towr_terrain_t* terrains, int per_problem) {
  if (B <= 0) return TOWR_OK;
  const Layout& L = h->L;
  KParams P{};
  if (h->soft) {
    if (int rc = scratch_acquire(h, s)) return rc;
    if (int rc = launch_soft(h, B, X, ldx, GR != nullptr, s, terrains, per_problem, P)) return rc;
  }
  P.X = X; P.ldx = ldx;
  P.nodecol = h->d_nodecol; P.spl = h->d_spl; P.dur = h->d_dur;
  P.sg = h->sg; P.n_spl = (int32_t)L.spl.size();
  P.pinfo = h->d_pinfo; P.pcols = h->d_pcols; P.pact = h->d_pact; P.sched = h->d_sched; P.eelin = h->d_eelin; P.lin = h->d_lin;
  P.terrains = terrains; P.terrain_per_problem = per_problem;
  P.B = B;
  P.n = L.n; P.n_pad = (L.n + 2) & ~1; P.n_nodecol = (int32_t)L.nodecol.size();
  P.fdisc_motion = L.fdisc_motion; P.rb = L.rb;
  P.citems = h->d_citems; P.n_citems = (int32_t)L.cost_items.size(); P.cq = h->d_cq;
  const int acc = cost_acc(L, GR != nullptr);
  P.lds_x_off = (int32_t)cost_x_off(L, acc);
  P.lds_red_off = (int32_t)cost_red_off(L, acc);
  P.c_cptr = h->d_c_cptr; P.c_cslot = h->d_c_cslot; P.c_nslot = L.cost_nslot;
  P.F = F; P.GR = GR; P.ldgr = ldgr;
  void* args[] = {&P};
  HIPCHK(h, launch_kernel(cost_kernel_for(L.gait, acc, L.rotvec), dim3((unsigned)std::min(B, h->cost_grid[acc])),
                            dim3(kCostBlock), args, cost_lds_bytes(L, acc), s));
  return h->soft ? scratch_release(h, s) : TOWR_OK;
}

// SaveTrajectoryToCSV's sample times: t = 0, dt, ... accumulated while t <= T + 1e-9, with
// T = base_linear_->GetTotalTime() (save_data.cpp:14, 55-58)
std::vector<double> traj_times(const Layout& L, double dt) {
  double T = 0.0;
  for (int i = 0; i < L.spl[0].n_polys; ++i) T += L.dur[L.spl[0].dur_off + i];
  std::vector<double> ts;
  for (double t = 0.0; t <= T + 1e-9; t += dt) ts.push_back(t);
  return ts;
}
constexpr int64_t kTrajMaxSamples = 1 << 22;

int launch_traj(towr_gpu_handle h, int B, const double* X, int64_t ldx, double dt, double* OUT, int64_t ldo, hipStream_t s) {
  const Layout& L = h->L;
  if (!(dt > 0.0)) return fail(h, TOWR_ERR_INVALID, "sample period must be > 0");
  if (dt != h->traj_dt || !h->d_traj_t) {
    const std::vector<double> ts = traj_times(L, dt);
    if ((int64_t)ts.size() > kTrajMaxSamples) return fail(h, TOWR_ERR_INVALID, "too many trajectory samples");
    if (h->d_traj_t) { (void)hipFree(h->d_traj_t); h->d_traj_t = nullptr; }
    HIPCHK(h, hipMalloc(&h->d_traj_t, sizeof(double) * ts.size()));
    HIPCHK(h, hipMemcpy(h->d_traj_t, ts.data(), sizeof(double) * ts.size(), hipMemcpyHostToDevice));
    h->traj_dt = dt; h->traj_ns = (int32_t)ts.size();
  }
  const int ns = h->traj_ns, cols = traj_cols(L.rb.n_ee);
  if (ldo < (int64_t)ns * cols) return fail(h, TOWR_ERR_INVALID, "leading dimension smaller than n_samples * n_cols");
  if (B <= 0) return TOWR_OK;
  KParams P{};
  P.X = X; P.ldx = ldx;
  P.nodecol = h->d_nodecol; P.spl = h->d_spl; P.dur = h->d_dur;
  P.pinfo = h->d_pinfo; P.pcols = h->d_pcols; P.pact = h->d_pact; P.sched = h->d_sched; P.eelin = h->d_eelin; P.lin = h->d_lin;
  P.terrains = h->d_terrain;
  P.n = L.n; P.n_pad = (L.n + 2) & ~1; P.n_nodecol = (int32_t)L.nodecol.size();
  P.rb = L.rb;
  TrajPhases ph{h->d_traj_pd, h->d_traj_n, h->d_traj_c0};
  const int32_t xoff = ((cols * (kTrajBlock + 1)) + 1) & ~1;
  const size_t lds = sizeof(double) * ((size_t)xoff + P.n_pad + (L.nodecol.size() + 3) / 4 * 2);
  if (lds > 160 * 1024) return fail(h, TOWR_ERR_UNSUPPORTED, "trajectory rows exceed the LDS");
  if (lds > 64 * 1024) HIPCHK(h, hipFuncSetAttribute(traj_kernel_for(L.gait), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int64_t grid = (int64_t)B * ((ns + kTrajBlock - 1) / kTrajBlock);
  if (grid > INT32_MAX) return fail(h, TOWR_ERR_INVALID, "batch too large");
  const double* tp = h->d_traj_t;
  void* args[] = {&P, &tp, const_cast<int*>(&ns), &ph, &OUT, &ldo, const_cast<int32_t*>(&xoff)};
  HIPCHK(h, launch_kernel(traj_kernel_for(L.gait), dim3((unsigned)grid), dim3(kTrajBlock), args, lds, s));
  return TOWR_OK;
}

int ensure_stage(towr_gpu_handle h, int B) {
  if (B <= h->stage_B) return TOWR_OK;
  const Layout& L = h->L;
  if (h->d_x) { (void)hipFree(h->d_x); (void)hipFree(h->d_g); (void)hipFree(h->d_v); }
  if (h->h_x) { (void)hipHostFree(h->h_x); (void)hipHostFree(h->h_g); (void)hipHostFree(h->h_v); }
  h->d_x = h->d_g = h->d_v = h->h_x = h->h_g = h->h_v = nullptr;
  HIPCHK(h, hipMalloc(&h->d_x, sizeof(double) * (size_t)B * L.n));
  HIPCHK(h, hipMalloc(&h->d_g, sizeof(double) * (size_t)B * std::max(1, L.m)));
  HIPCHK(h, hipMalloc(&h->d_v, sizeof(double) * (size_t)B * std::max<int64_t>(1, L.nnz)));
  if (!h->d_f) {
    HIPCHK(h, hipMalloc(&h->d_f, sizeof(double)));
    HIPCHK(h, hipMalloc(&h->d_grad, sizeof(double) * (size_t)std::max(1, L.n)));
  }
  HIPCHK(h, hipHostMalloc(&h->h_x, sizeof(double) * (size_t)B * L.n, hipHostMallocDefault));
  HIPCHK(h, hipHostMalloc(&h->h_g, sizeof(double) * (size_t)B * std::max(1, L.m), hipHostMallocDefault));
  HIPCHK(h, hipHostMalloc(&h->h_v, sizeof(double) * (size_t)B * std::max<int64_t>(1, L.nnz), hipHostMallocDefault));
  HIPCHK(h, hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hd_x), h->h_x, 0));
  HIPCHK(h, hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hd_g), h->h_g, 0));
  HIPCHK(h, hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hd_v), h->h_v, 0));
  h->stage_B = B;
  return TOWR_OK;
}

// Terrain of a batch launch: the per-problem set (towr_gpu_set_batch_terrain) when one is set, which
// must then hold exactly B entries; else the description's terrain for every problem. `single`
// entry points (one problem through host pointers) always use the description's terrain.
int batch_terrain(towr_gpu_handle h, int B, bool single, const towr_terrain_t** ter, int* per) {
  *ter = h->d_terrain; *per = 0;
  if (single || !h->d_bterrain) return TOWR_OK;
  if (h->bterrain_n != B)
    return fail(h, TOWR_ERR_INVALID, "batch terrains are set for " + std::to_string(h->bterrain_n) + " problems, the call has " +
                                         std::to_string(B) + " (set them again, or with B = 0 to clear)");
  *ter = h->d_bterrain; *per = 1;
  return TOWR_OK;
}

// [p, p + bytes) inside caller memory registered with towr_gpu_register_host
bool is_registered(towr_gpu_handle h, const void* p, size_t bytes) {
  const char* c = static_cast<const char*>(p);
  for (const auto& r : h->pinned)
    if (c >= r.p && c + bytes <= r.p + r.n) return true;
  return false;
}
// device address of registered host memory (zero-copy access from a kernel), or nullptr
template <class T>
T* device_view(towr_gpu_handle h, T* p, size_t bytes) {
  const char* c = reinterpret_cast<const char*>(p);
  for (const auto& r : h->pinned)
    if (c >= r.p && c + bytes <= r.p + r.n) return reinterpret_cast<T*>(r.dev + (c - r.p));
  return nullptr;
}

// host memcpy over a few threads: one thread reaches ~10 GB/s on the box's EPYC cores, below what a
// PCIe Gen5 x16 DMA delivers into the pinned staging, so large copies are split
void par_copy(void* dst, const void* src, size_t bytes) {
  constexpr size_t kMinPerThread = 4u << 20;
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const int nt = (int)std::min<size_t>(std::min(8u, hw), bytes / kMinPerThread);
  if (nt <= 1) { std::memcpy(dst, src, bytes); return; }
  const size_t part = (bytes / nt + 63) & ~(size_t)63;
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) {
    const size_t o = (size_t)t * part;
    if (o >= bytes) break;
    th.emplace_back([=] { std::memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, std::min(part, bytes - o)); });
  }
  std::memcpy(dst, src, std::min(part, bytes));
  for (auto& t : th) t.join();
}

int ensure_events(towr_gpu_handle h, size_t n) {
  while (h->ev_c.size() < n) {
    hipEvent_t a = nullptr, b = nullptr;
    HIPCHK(h, hipEventCreateWithFlags(&a, hipEventDisableTiming));
    if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) { (void)hipEventDestroy(a); return fail(h, TOWR_ERR_HIP, "hipEventCreate failed"); }
    h->ev_c.push_back(a); h->ev_d.push_back(b);
  }
  return TOWR_OK;
}

// Host-pointer evaluation (IpoptAdapter-shaped entry points and the host batch).
//   * x goes H2D straight from the caller's array when it is registered (towr_gpu_register_host),
//     else through the pinned staging;
//   * B = 1 runs the single-launch group (every class in one kernel) when the layout has one, zero-copy
//     (x read and g / values written through mapped host memory, see below);
//   * B > 1 is cut into chunks of ~64 MB of output: the handle's stream evaluates chunk i while the
//     copy stream moves chunk i - 1 to the host (a PCIe DMA overlaps the next chunk's kernels), and
//     the host thread copies finished chunks out of the staging in parallel with both. Outputs in
//     registered caller memory are DMA'd in place (no host copy at all).
int host_eval(towr_gpu_handle h, int B, const double* X, double* G, double* V, bool single) {
  h->kept = false;   // (the staging below may be overwritten)
  const towr_terrain_t* ter;
  int per;
  if (int rc = batch_terrain(h, B, single, &ter, &per)) return rc;
  if (int rc = ensure_stage(h, B)) return rc;
  const Layout& L = h->L;
  const size_t xb = sizeof(double) * (size_t)B * L.n;
  const size_t gp = sizeof(double) * (size_t)L.m, vp = sizeof(double) * (size_t)L.nnz;   // per problem
  const bool xr = is_registered(h, X, xb);
  const bool gr = G && is_registered(h, G, gp * B), vr = V && is_registered(h, V, vp * B);
  double* gdst = gr ? G : h->h_g;   // D2H destinations
  double* vdst = vr ? V : h->h_v;
  if (B == 1) {
    // one problem, zero-copy: the kernels stage x from host memory and write g and the CSR values straight
    // into host memory over PCIe (the tile copy-outs and the composers store each value exactly once), so
    // the call is its launches and one synchronisation — no DMA command on either side. With fixed phase
    // durations every class runs in ONE launch (the single group); under phase-duration optimisation the
    // record kernels read x over PCIe and the composers stream the ~2 MB of values to the host.
    const double* xd = device_view(h, X, xb);
    if (!xd) { std::memcpy(h->h_x, X, xb); xd = h->hd_x; }
    double* gd = G ? device_view(h, G, gp) : nullptr;
    double* vd = V ? device_view(h, V, vp) : nullptr;
    h->sync_call = true;   // (the scratch event: this call ends with a synchronisation below)
    const bool scr = uses_scratch(L);
    if (scr && h->single.n_units > 0)
      if (int rc = scratch_acquire(h, h->stream)) { h->sync_call = false; return rc; }
    const int rc = h->single.n_units > 0
                       ? launch_fused(h, h->single, 1, xd, L.n, gd ? gd : h->hd_g, L.m, vd ? vd : h->hd_v, L.nnz, G != nullptr,
                                      V != nullptr, h->stream, ter, per)
                       : launch(h, 1, xd, L.n, gd ? gd : h->hd_g, L.m, vd ? vd : h->hd_v, L.nnz, G != nullptr, V != nullptr, h->stream,
                                ter, per, -1);
    if (scr && h->single.n_units > 0) (void)scratch_release(h, h->stream);
    h->sync_call = false;
    if (rc) {
      (void)hipStreamSynchronize(h->stream);   // whatever was launched has finished before the scratch is reused
      return rc;
    }
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (G && !gd) std::memcpy(G, h->h_g, gp);
    if (V && !vd) par_copy(V, h->h_v, vp);
    return TOWR_OK;
  }
  const double* xsrc = X;
  if (!xr) { par_copy(h->h_x, X, xb); xsrc = h->h_x; }
  HIPCHK(h, hipMemcpyAsync(h->d_x, xsrc, xb, hipMemcpyHostToDevice, h->stream));
  const size_t out_pp = (G ? gp : 0) + (V ? vp : 0) + 1;
  const int C = (int)std::max<size_t>(1, std::min<size_t>((size_t)B, (64u << 20) / out_pp));
  const int nch = (B + C - 1) / C;
  if (nch == 1) {   // one chunk: everything on the handle's stream
    if (int rc = launch(h, B, h->d_x, L.n, h->d_g, L.m, h->d_v, L.nnz, G != nullptr, V != nullptr, h->stream, ter, per, -1))
      return rc;
    if (G) HIPCHK(h, hipMemcpyAsync(gdst, h->d_g, gp * B, hipMemcpyDeviceToHost, h->stream));
    if (V) HIPCHK(h, hipMemcpyAsync(vdst, h->d_v, vp * B, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    if (G && !gr) par_copy(G, h->h_g, gp * B);
    if (V && !vr) par_copy(V, h->h_v, vp * B);
    return TOWR_OK;
  }
  if (int rc = ensure_events(h, (size_t)nch)) return rc;
  for (int i = 0; i < nch; ++i) {   // enqueue: kernels on the stream, DMA on the copy stream
    const int c0 = i * C, cb = std::min(C, B - c0);
    if (int rc = launch(h, cb, h->d_x + (size_t)c0 * L.n, L.n, h->d_g + (size_t)c0 * L.m, L.m, h->d_v + (size_t)c0 * L.nnz, L.nnz,
                        G != nullptr, V != nullptr, h->stream, per ? ter + c0 : ter, per, -1))
      return rc;
    HIPCHK(h, hipEventRecord(h->ev_c[i], h->stream));
    HIPCHK(h, hipStreamWaitEvent(h->copy_stream, h->ev_c[i], 0));
    if (G) HIPCHK(h, hipMemcpyAsync(gdst + (size_t)c0 * L.m, h->d_g + (size_t)c0 * L.m, gp * cb, hipMemcpyDeviceToHost, h->copy_stream));
    if (V) HIPCHK(h, hipMemcpyAsync(vdst + (size_t)c0 * L.nnz, h->d_v + (size_t)c0 * L.nnz, vp * cb, hipMemcpyDeviceToHost, h->copy_stream));
    HIPCHK(h, hipEventRecord(h->ev_d[i], h->copy_stream));
  }
  for (int i = 0; i < nch; ++i) {   // drain: each chunk leaves the staging while later ones move
    const int c0 = i * C, cb = std::min(C, B - c0);
    HIPCHK(h, hipEventSynchronize(h->ev_d[i]));
    if (G && !gr) par_copy(G + (size_t)c0 * L.m, h->h_g + (size_t)c0 * L.m, gp * cb);
    if (V && !vr) par_copy(V + (size_t)c0 * L.nnz, h->h_v + (size_t)c0 * L.nnz, vp * cb);
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  return TOWR_OK;
}

// Fusion groups from TOWR_GPU_FUSE (or kDefaultFuse): comma-separated groups of class letters (d
// Dynamic, r RangeOfMotion, f ForceConstraintDiscretized, t TorqueConstraintDiscretized, m small
// kinds), e.g. "rf" or "rf,dm"; "none" = per-class launches. Classes this layout lacks are dropped; a
// group needs two classes. Layout-only: the unit tables are uploaded by towr_gpu_create.
int setup_fusion(towr_gpu_handle h, std::string& err) {
  const Layout& L = h->L;
  // phase-duration optimisation: the tile classes run wave-per-row blocks of different sizes
  // (tile_block), which the fused kernel's fixed 192 / 256-lane bodies do not cover
  if (L.gait) return TOWR_OK;
  const char* fz = std::getenv("TOWR_GPU_FUSE");
  // RotVec: per-class launches (ANYmal, B = 4096, one box: 0.359-0.367 ms per step, "rf" 0.375: its
  // RangeOfMotion tiles carry the Rodrigues / left-Jacobian chain and share the CUs worse)
  const std::string spec = fz ? fz : L.rotvec ? "none" : kDefaultFuse;
  size_t p0 = 0;
  while (p0 <= spec.size() && h->n_fuse < towr_gpu_handle_s::kMaxFuse) {
    const size_t p1 = std::min(spec.find(',', p0), spec.size());
    uint32_t mask = 0;
    for (size_t k = p0; k < p1; ++k) {
      const char* letters = "drftm";
      const char* f = std::strchr(letters, spec[k]);
      if (f && *f) mask |= 1u << (f - letters);
    }
    for (int lc = 0; lc < LC_COUNT; ++lc)
      if (((mask >> lc) & 1) && class_units(L, lc) == 0) mask &= ~(1u << lc);
    for (int g = 0; g < h->n_fuse; ++g) mask &= ~h->fuse[g].mask;
    if (__builtin_popcount(mask) >= 2) {
      towr_gpu_handle_s::FuseGroup& fg = h->fuse[h->n_fuse++];
      fg.mask = mask;
      // 256 with Dynamic; 192-lane tiles otherwise, small-kind groups of 3 waves fit those blocks
      fg.kblock = (mask & (1u << LC_DYN)) || ((mask & (1u << LC_MISC)) && 64 * kMiscWaves > 192) ? 256 : 192;
      for (int lc = 0; lc < LC_COUNT; ++lc)
        if ((mask >> lc) & 1) {
          fg.lds = std::max(fg.lds, lds_bytes(L, lc));
          if (lc != LC_MISC && L.type_block[class_type(lc)] != (lc == LC_DYN ? 256 : 192)) {
            err = "internal: fused launch expects 256-lane Dynamic and 192-lane tiles"; return TOWR_ERR_INVALID;
          }
        }
      fg.n_units = (int32_t)fused_units(L, mask).size();
      if (fg.lds > 160 * 1024) { err = "tile too large for LDS"; return TOWR_ERR_UNSUPPORTED; }
    }
    p0 = p1 + 1;
  }
  // the single-problem group: every class of the layout in one launch (at B = 1 a launch is one wave
  // of latency however wide, so one launch instead of three is the whole gain)
  uint32_t all = 0;
  bool fits = true;
  for (int lc = 0; lc < LC_COUNT; ++lc)
    if (class_units(L, lc) > 0) {
      all |= 1u << lc;
      if (lc != LC_MISC && L.type_block[class_type(lc)] != (lc == LC_DYN ? 256 : 192)) fits = false;
    }
  if (fits && __builtin_popcount(all) >= 2) {
    towr_gpu_handle_s::FuseGroup& sg = h->single;
    sg.mask = all;
    sg.kblock = (all & (1u << LC_DYN)) || ((all & (1u << LC_MISC)) && 64 * kMiscWaves > 192) ? 256 : 192;
    for (int lc = 0; lc < LC_COUNT; ++lc)
      if ((all >> lc) & 1) sg.lds = std::max(sg.lds, lds_bytes(L, lc));
    sg.n_units = sg.lds <= 160 * 1024 ? (int32_t)fused_units(L, all).size() : 0;
  }
  return TOWR_OK;
}

}  // namespace

// =================================================================================================
// C-ABI
// =================================================================================================
extern "C" {

#ifdef TOWR_STAMPS
// experiment build: device buffer of kStampRegions x kStampRegion slots for the TG_STAMP timestamps (null: off);
// resets the launch count. towr_gpu_debug_stamp_kernel(i): the kernel symbol of region i (null past the last)
int towr_gpu_debug_stamps(void* buf) { g_stamps = static_cast<unsigned long long*>(buf); if (buf) g_stamp_n = 0; return TOWR_OK; }
const char* towr_gpu_debug_stamp_kernel(int i) { return i < g_stamp_n ? hipKernelNameRefByPtr(g_stamp_fn[i], nullptr) : nullptr; }
#endif

int towr_gpu_abi_version(void) { return TOWR_GPU_ABI_VERSION; }

int towr_gpu_num_kernels(void) { return LC_COUNT + towr_gpu_handle_s::kMaxFuse; }

const char* towr_gpu_last_error(towr_gpu_handle h) {
  if (h) return h->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_last_error.c_str();
}

int towr_gpu_create(const towr_problem_desc_t* desc, int device, towr_gpu_handle* out) {
  return towr_gpu_create_ex(desc, 0, nullptr, device, out);
}

int towr_gpu_create_ex(const towr_problem_desc_t* desc, int32_t n_data, const towr_data_t* data, int device, towr_gpu_handle* out) {
  if (!desc || !out || n_data < 0 || (n_data > 0 && !data)) return fail(nullptr, TOWR_ERR_INVALID, "null argument");
  *out = nullptr;
  towr_gpu_handle h = new towr_gpu_handle_s();
  std::string err;
  const int rc = build_layout_ex(*desc, n_data, data, h->L, err);
  if (rc != TOWR_OK) { fail(nullptr, rc, err); delete h; return rc; }
  if (int rf = setup_fusion(h, err)) { fail(nullptr, rf, err); delete h; return rf; }
  if (!h->L.soft.empty()) {   // SoftConstraint terms: the wrapped sets as the hard constraints of a child handle
    const towr_problem_desc_t sd = soft_desc(*desc, h->L);
    std::vector<towr_data_t> cd;   // their LinearEquality matrices, re-indexed to the child's constraint list
    for (size_t k = 0; k < h->L.soft.size(); ++k)
      if (const towr_data_t* m = find_data(n_data, data, TOWR_DATA_LINEAR_M, h->L.soft[k].second)) {
        towr_data_t e = *m;
        e.index = (int32_t)k;
        cd.push_back(e);
      }
    if (int rs = towr_gpu_create_ex(&sd, (int32_t)cd.size(), cd.data(), device, &h->soft)) { delete h; return rs; }
    const Layout& C = h->soft->L;
    for (size_t k = 0; k < h->L.soft.size(); ++k) {   // b = (upper + lower) / 2 (soft_constraint.cc:40-45)
      const int rows = C.cons[k].rows;
      const towr_data_t* bd = find_data(n_data, data, TOWR_DATA_SOFT_BOUNDS, h->L.soft[k].first);
      if (!bd || (rows > 0 && !bd->data) || bd->count != 2 * (int64_t)rows) {
        const std::string msg = "SoftConstraint term " + std::to_string(h->L.soft[k].first) +
                                ": bounds (side data TOWR_DATA_SOFT_BOUNDS, lower then upper) missing or not 2 x the set's rows";
        towr_gpu_destroy(h);   // the message is built first: destroy frees h
        return fail(nullptr, TOWR_ERR_INVALID, msg);
      }
      for (int r = 0; r < rows; ++r) h->soft_b.push_back((bd->data[rows + r] + bd->data[r]) / 2.);
    }
  }
  if (device < 0) {   // layout-only handle: sizes / structure / x0, no evaluation (CPU-side tests)
    h->device = -1;
    *out = h;
    return TOWR_OK;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device >= ndev) {
    fail(nullptr, TOWR_ERR_NO_DEVICE, "no HIP device available for towr_gpu_create");
    delete h;
    return TOWR_ERR_NO_DEVICE;
  }
  h->device = device;
  auto bail = [&](int code) { std::string m = h->err; towr_gpu_destroy(h); fail(nullptr, code, m); return code; };
  if (hipSetDevice(device) != hipSuccess) { h->err = "hipSetDevice failed"; return bail(TOWR_ERR_HIP); }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    h->err = std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only";
    return bail(TOWR_ERR_NO_DEVICE);
  }
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) { h->err = "hipStreamCreate failed"; return bail(TOWR_ERR_HIP); }
  const Layout& L = h->L;
  std::vector<towr_terrain_t> ter(1, L.terrain);
  std::vector<int32_t> nodecol16(L.nodecol);   // constant node values -> x[n] = 0; whole 16-B units
  for (int32_t& c : nodecol16) if (c < 0) c = L.n;
  nodecol16.resize((nodecol16.size() + 3) / 4 * 4, L.n);
  std::vector<MiscWave> mwave;   // the small-kind groups' waves, one descriptor and 64 items each (layout.h MiscWave)
  std::vector<ItemDesc> mitems;
  for (size_t q = 0; q < L.misc_tiles.size(); ++q) {
    const int32_t ti = L.misc_tiles[q];
    MiscWave w{};
    w.ti = ti;
    w.wl_off = L.misc_lds[2 * q];
    w.rows_off = L.misc_lds[2 * q + 1];
    ItemDesc none{};
    none.type = IT_NONE;
    if (ti >= 0) {
      const TileDesc& T = L.tiles[ti];
      w.r0 = T.r0; w.r1 = T.r1; w.v0 = T.v0; w.v1 = T.v1;
      for (int l = 0; l < 64; ++l) mitems.push_back(T.i0 + l < T.i1 ? L.items[T.i0 + l] : none);
    } else {
      for (int l = 0; l < 64; ++l) mitems.push_back(none);
    }
    mwave.push_back(w);
  }
  int r;
  if ((r = upload(h, &h->d_items, L.items)) || (r = upload(h, &h->d_misc_wave, mwave)) || (r = upload(h, &h->d_misc_items, mitems)) || (r = upload(h, &h->d_slots, L.slot_groups)) ||
      (r = upload(h, &h->d_tiles, L.tiles)) || (r = upload(h, &h->d_nodecol, nodecol16)) ||
      (r = upload(h, &h->d_spl, L.spl)) || (r = upload(h, &h->d_dur, L.dur)) || (r = upload(h, &h->d_terrain, ter)) ||
      (r = upload(h, &h->d_pinfo, L.pinfo)) || (r = upload(h, &h->d_pcols, L.pcols)) || (r = upload(h, &h->d_pact, L.pact)) || (r = upload(h, &h->d_sched, L.sched)) ||
      (r = upload(h, &h->d_misc, L.misc_tiles)) || (r = upload(h, &h->d_misc_lds, L.misc_lds)) || (r = upload(h, &h->d_xspan, L.misc_xspan)) || (r = upload(h, &h->d_eelin, L.eelin)) ||
      (r = upload(h, &h->d_lin, L.lin)) ||
      (r = upload(h, &h->d_citems, L.cost_items)) || (r = upload(h, &h->d_cq, L.cost_q)) ||
      (r = upload(h, &h->d_c_cptr, padded(L.cost_cptr, 8))) || (r = upload(h, &h->d_c_cslot, cost_slot_table(L))) || (r = upload(h, &h->d_gtab, gait_blob(L))) ||
      (r = upload(h, &h->d_idir, L.idirect)) || (r = upload(h, &h->d_fsb, L.fs_blocks)) || (r = upload(h, &h->d_fs_t, L.fs_t)) ||
      (r = upload(h, &h->d_fs_tmpl, L.fs_tmpl)) || (r = upload(h, &h->d_fs_ws, L.fs_ws)) ||
      (r = upload(h, &h->d_fs_iee, L.fs_iee)) || (r = upload(h, &h->d_fs_irow, L.fs_irow)) || (r = upload(h, &h->d_fs_iblk, L.fs_iblk)) ||
      (r = upload(h, &h->d_gs_geo, L.gs_geo)) || (r = upload(h, &h->d_gs_tmpl, L.gs_tmpl)) || (r = upload(h, &h->d_gs_pcode, L.gs_pcode)) ||
      (r = upload(h, &h->d_gs_blk[GS_ROM], L.gs_blocks[GS_ROM])) || (r = upload(h, &h->d_gs_blk[GS_DYN], L.gs_blocks[GS_DYN])) ||
      (r = upload(h, &h->d_gs_blk[GS_TQ], L.gs_blocks[GS_TQ])) || (r = upload(h, &h->d_gs_inst[GS_TQ], L.gs_inst[GS_TQ])) ||
      (r = upload(h, &h->d_gs_inst[GS_ROM], L.gs_inst[GS_ROM])) || (r = upload(h, &h->d_gs_inst[GS_DYN], L.gs_inst[GS_DYN])) ||
      (r = upload(h, &h->d_rvi, L.rv_inst)) || (r = upload(h, &h->d_gs_segs, L.gs_segs)) || (r = upload(h, &h->d_gs_tseg, L.gs_tseg)) || (r = upload(h, &h->d_gs_vmap, L.gs_vmap)) ||
      (r = upload(h, &h->d_gs_ws, L.gs_ws)) || (r = upload(h, &h->d_gs_blob, L.gs_blob)))
    return bail(r);
  if (hipEventCreateWithFlags(&h->scr_ev, hipEventDisableTiming) != hipSuccess) { h->err = "hipEventCreate failed"; return bail(TOWR_ERR_HIP); }
  {   // trajectory export: phase durations of the description (fixed gait), counts, contact at start
    const towr_problem_desc_t& d = L.desc;
    std::vector<double> pd((size_t)TOWR_MAX_EE * TOWR_MAX_PHASES, 0.0);
    std::vector<int32_t> pn(TOWR_MAX_EE, 0), pc(TOWR_MAX_EE, 0);
    for (int ee = 0; ee < d.robot.n_ee; ++ee) {
      pn[ee] = d.n_phases[ee]; pc[ee] = d.contact_at_start[ee] != 0;
      for (int q = 0; q < d.n_phases[ee]; ++q) pd[(size_t)ee * TOWR_MAX_PHASES + q] = d.phase_durations[ee][q];
    }
    if ((r = upload(h, &h->d_traj_pd, pd)) || (r = upload(h, &h->d_traj_n, pn)) || (r = upload(h, &h->d_traj_c0, pc))) return bail(r);
  }
  if (h->soft) {   // the soft child's pattern by column, rows ascending (int32: its nnz is small), and b
    const Layout& C = h->soft->L;
    std::vector<int32_t> cptr(L.n + 1, 0);
    for (int32_t c : C.col) ++cptr[c + 1];
    for (int j = 0; j < L.n; ++j) cptr[j + 1] += cptr[j];
    std::vector<int2> cent(C.col.size());
    std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
    for (int row = 0; row < C.m; ++row)
      for (int64_t k = C.row_ptr[row]; k < C.row_ptr[row + 1]; ++k) cent[fill[C.col[k]]++] = make_int2((int)k, row);
    if ((r = upload(h, &h->d_soft_cptr, cptr)) || (r = upload(h, &h->d_soft_cent, cent)) || (r = upload(h, &h->d_soft_b, h->soft_b))) return bail(r);
  }
  {   // segment table in 32-row blocks (see SegSoA)
    const int nspl = (int)L.spl.size();
    const int nr = L.segs.empty() ? 0 : (int)(L.segs.size() / nspl);
    const int ng = std::max(1, (nr + kSegGroup - 1) / kSegGroup);
    std::vector<double> dv((size_t)nspl * ng * kSegDoubles * kSegGroup, 0.0);
    std::vector<int32_t> iv((size_t)nspl * ng * kSegInts * kSegGroup, L.n);
    for (int sp = 0; sp < nspl; ++sp)
      for (int k = 0; k < ng * kSegGroup; ++k) {
        const size_t blk = (size_t)sp * ng + k / kSegGroup;
        double* D = dv.data() + blk * kSegDoubles * kSegGroup + k % kSegGroup;
        int32_t* I = iv.data() + blk * kSegInts * kSegGroup + k % kSegGroup;
        if (k >= nr) { D[kSegGroup] = 1.0; I[0] = 0; continue; }   // padding rows: a harmless polynomial
        const SegRec& rr = L.segs[(size_t)k * nspl + sp];
        D[0] = rr.tl; D[kSegGroup] = rr.T; I[0] = rr.poly;
        for (int f = 0; f < 12; ++f) {
          D[(2 + f) * kSegGroup] = rr.H[f / 4][f % 4];
          I[(1 + f) * kSegGroup] = rr.col[f / 3][f % 3];
        }
      }
    const size_t db = sizeof(double) * dv.size(), ib = sizeof(int32_t) * iv.size();
    if (hipMalloc(&h->d_segs, db + ib) != hipSuccess || hipMemcpy(h->d_segs, dv.data(), db, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(static_cast<char*>(h->d_segs) + db, iv.data(), ib, hipMemcpyHostToDevice) != hipSuccess) {
      h->err = "segment table upload failed"; return bail(TOWR_ERR_HIP);
    }
    h->sg.d = static_cast<const double*>(h->d_segs);
    h->sg.i = reinterpret_cast<const int32_t*>(static_cast<const char*>(h->d_segs) + db);
    h->sg.ng = ng;
  }
  {
    const char* ns = std::getenv("TOWR_GPU_STREAMS");
    // Fixed phase durations with a fusion group: one side stream, on which the other classes (Dynamic, then the
    // small kinds) run beside the fused launch (launch_classes; ANYmal, B = 4096, one box: 0.2450 vs 0.2514 ms
    // per step serial; Dynamic and the small kinds on two side streams 0.2547, the small kinds after the fused
    // launch 0.2500). Without a fusion group (RotVec): serial launches (1, 2, 4 streams in round 1: 0.524, 0.521,
    // 0.550 ms; RotVec with the classes beside each other: no change). Under phase-duration optimisation (the
    // streaming path) one or two side streams: the write-bound compose launches run beside the latency-bound
    // record work (launch_stream_path).
    const bool streamed = h->L.gait && (h->L.fstream || h->L.gstream[GS_TQ]);
    h->rv_overlap = h->L.rotvec;
    const int want = ns ? std::atoi(ns) - 1 : streamed ? (h->L.gstream[GS_TQ] ? 2 : 1) : (h->n_fuse > 0 || h->rv_overlap) ? 1 : 0;
    h->n_side = std::max(0, std::min(towr_gpu_handle_s::kMaxSide, want));
    if (h->n_side > 0 && hipEventCreateWithFlags(&h->fork, hipEventDisableTiming) != hipSuccess) {
      h->err = "hipEventCreate failed"; return bail(TOWR_ERR_HIP);
    }
    // side streams at the device's greatest priority: the streaming path runs its critical chains there (the
    // FDISC / TQDISC records, whose blocks must not wait behind the other chain's, see launch_stream_path;
    // ANYmal gait + Torque, B = 1024: the TQDISC records on a low-priority stream took 730 us instead of ~50)
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = least = 0;
    // (round 5, ANYmal gait, B = 1024, one box: side streams at the default priority 0.6225-0.6335 vs 0.6263-0.6371 ms
    // per step, + Torque 1.216-1.219 vs 1.209-1.211: noise without Torque, the greatest priority kept)
    for (int i = 0; i < h->n_side; ++i)
      if (hipStreamCreateWithPriority(&h->side[i], hipStreamNonBlocking, greatest) != hipSuccess ||
          hipEventCreateWithFlags(&h->join[i], hipEventDisableTiming) != hipSuccess) {
        h->err = "side stream creation failed"; return bail(TOWR_ERR_HIP);
      }
  }
  for (int g = 0; g < h->n_fuse; ++g) {   // fusion groups (set up with the layout): unit tables
    towr_gpu_handle_s::FuseGroup& fg = h->fuse[g];
    const std::vector<UnitDesc> units = fused_units(L, fg.mask);
    if ((r = upload(h, &fg.d_units, units))) return bail(r);
    if (fg.lds > 64 * 1024 && hipFuncSetAttribute(step_kernel_for(L.gait, L.rotvec, fg.kblock), hipFuncAttributeMaxDynamicSharedMemorySize, (int)fg.lds) != hipSuccess) {
      h->err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; return bail(TOWR_ERR_HIP);
    }
  }
  if (h->single.n_units > 0) {
    towr_gpu_handle_s::FuseGroup& sg = h->single;
    if ((r = upload(h, &sg.d_units, fused_units(L, sg.mask)))) return bail(r);
    if (sg.lds > 64 * 1024 && hipFuncSetAttribute(step_kernel_for(L.gait, L.rotvec, sg.kblock), hipFuncAttributeMaxDynamicSharedMemorySize, (int)sg.lds) != hipSuccess) {
      h->err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; return bail(TOWR_ERR_HIP);
    }
  }
  if (hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking) != hipSuccess) { h->err = "hipStreamCreate failed"; return bail(TOWR_ERR_HIP); }
  for (int lc = 0; lc < LC_COUNT; ++lc) {
    if (class_units(L, lc) == 0) continue;
    const size_t lds = lds_bytes(L, lc);
    if (lds > 160 * 1024) { h->err = "tile too large for LDS"; return bail(TOWR_ERR_UNSUPPORTED); }
    if (lds > 64 * 1024 && (hipFuncSetAttribute(kernel_for_class(lc, L.gait, L.rotvec, streamed_class(L, lc)), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess ||
                            (streamed_class(L, lc) && !compose_lds_attr(lds)))) {
      h->err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; return bail(TOWR_ERR_HIP);
    }
  }
  if (L.fstream || L.gstream[GS_ROM] || L.gstream[GS_DYN] || L.gstream[GS_TQ]) {   // the record kernels share fs_inst_lds_bytes' layout
    // (fixed-gait RotVec also uses scratch, for its coefficient pre-pass, but launches no record kernel)
    const size_t lds = fs_inst_lds_bytes(L);
    if (lds > kLdsMax) { h->err = "problem too large for the streaming instant kernel's LDS"; return bail(TOWR_ERR_UNSUPPORTED); }
    // every record launch's LDS (rec_launch_lds): a Dynamic part, or the FDISC part with its staged tables
    const size_t need = std::max(rec_launch_lds(L, true, false, nullptr), rec_launch_lds(L, false, true, nullptr));
    if (need > kLdsMax) { h->err = "problem too large for the record kernel's LDS"; return bail(TOWR_ERR_UNSUPPORTED); }
    bool ok = true;
    for (int roles = 1; roles < 8 && need > 64 * 1024; ++roles)
      ok = ok && hipFuncSetAttribute(gait_rec_kernel(L.rotvec, roles), hipFuncAttributeMaxDynamicSharedMemorySize, (int)need) == hipSuccess;
    if (!ok) {
      h->err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; return bail(TOWR_ERR_HIP);
    }
  }
  {
    // the cost kernel's persistent grid: as many blocks as the device holds at once (cost_traj.hip)
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess || cus <= 0) cus = 256;
    for (int g = 0; g < 2; ++g) {
      const int acc = cost_acc(L, g != 0);
      const size_t lds = cost_lds_bytes(L, acc);
      const void* fn = cost_kernel_for(L.gait, acc, L.rotvec);
      if (lds > 160 * 1024) { h->err = "problem too large for the cost kernel's LDS gradient"; return bail(TOWR_ERR_UNSUPPORTED); }
      if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) {
        h->err = "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed"; return bail(TOWR_ERR_HIP);
      }
      // blocks per CU: 160 kB of LDS, and the waves per SIMD the registers allow (512 VGPRs per lane and SIMD,
      // granules of 8; a block of kCostBlock threads puts kCostBlock / 256 waves on each SIMD)
      hipFuncAttributes fa{};
      int per_cu = 1;
      if (hipFuncGetAttributes(&fa, fn) == hipSuccess && fa.numRegs > 0) {
        const int by_regs = 512 / ((fa.numRegs + 7) / 8 * 8) / std::max(1, kCostBlock / 256);
        const int by_lds = (int)(160 * 1024 / std::max<size_t>(lds, 1));
        per_cu = std::max(1, std::min({by_regs, by_lds, 8}));
      }
      h->cost_grid[acc] = per_cu * cus;
      if (launch_log_on()) std::fprintf(stderr, "towr-cost acc %d regs %d lds %zu blocks/CU %d\n", acc, fa.numRegs, lds, per_cu);
    }
  }
  *out = h;
  return TOWR_OK;
}

int towr_gpu_destroy(towr_gpu_handle h) {
  if (!h) return TOWR_OK;
  void* dev[] = {h->d_items, h->d_slots, h->d_tiles, h->d_nodecol, h->d_spl, h->d_dur, h->d_segs, h->d_terrain,
                 h->d_pinfo, h->d_pcols, h->d_pact, h->d_sched, h->d_misc, h->d_misc_lds, h->d_misc_wave, h->d_misc_items, h->d_xspan, h->d_eelin, h->d_gtab, h->d_idir, h->d_citems, h->d_cq, h->fuse[0].d_units, h->fuse[1].d_units,
                 h->d_bterrain, h->d_x, h->d_g, h->d_v, h->d_f, h->d_grad,
                 h->d_traj_pd, h->d_traj_n, h->d_traj_c0, h->d_traj_t, h->d_fsb, h->d_fs_t, h->d_fs_tmpl, h->d_fs_ws, 
                 h->d_fs_iee, h->d_fs_irow, h->d_fs_iblk, h->d_fsrec, h->d_lin, h->d_soft_b, h->d_soft_cptr, h->d_soft_cent, h->d_c_cptr, h->d_c_cslot, h->d_sg, h->d_sv,
                 h->single.d_units, h->d_gs_geo, h->d_gs_tmpl, h->d_gs_pcode, h->d_gs_blk[0], h->d_gs_blk[1], h->d_gs_blk[2],
                 h->d_gs_inst[0], h->d_gs_inst[1], h->d_gs_inst[2], h->d_gsrec, h->d_rvc, h->d_rvi, h->d_gs_segs, h->d_gs_tseg, h->d_gs_vmap, h->d_gs_ws, h->d_gs_blob};
  if (h->device >= 0) for (void* p : dev) if (p) (void)hipFree(p);
  void* host[] = {h->h_x, h->h_g, h->h_v};
  for (void* p : host) if (p) (void)hipHostFree(p);
  for (const auto& r : h->pinned) (void)hipHostUnregister(const_cast<char*>(r.p));
  for (hipEvent_t e : h->ev_c) (void)hipEventDestroy(e);
  for (hipEvent_t e : h->ev_d) (void)hipEventDestroy(e);
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  for (int i = 0; i < towr_gpu_handle_s::kMaxSide; ++i) {
    if (h->side[i]) (void)hipStreamDestroy(h->side[i]);
    if (h->join[i]) (void)hipEventDestroy(h->join[i]);
  }
  if (h->fork) (void)hipEventDestroy(h->fork);
  if (h->scr_ev) (void)hipEventDestroy(h->scr_ev);
  if (h->soft) towr_gpu_destroy(h->soft);
  delete h;
  return TOWR_OK;
}

int towr_gpu_sizes(towr_gpu_handle h, int32_t* n, int32_t* m, int64_t* nnz) {
  if (!h) return fail(nullptr, TOWR_ERR_INVALID, "null handle");
  if (n) *n = h->L.n;
  if (m) *m = h->L.m;
  if (nnz) *nnz = h->L.nnz;
  return TOWR_OK;
}

int towr_gpu_jac_structure(towr_gpu_handle h, int32_t* iRow, int32_t* jCol) {
  if (!h || !iRow || !jCol) return fail(h, TOWR_ERR_INVALID, "null argument");
  const Layout& L = h->L;
  for (int r = 0; r < L.m; ++r)
    for (int64_t k = L.row_ptr[r]; k < L.row_ptr[r + 1]; ++k) { iRow[k] = r; jCol[k] = L.col[k]; }
  return TOWR_OK;
}

int towr_gpu_jac_csr(towr_gpu_handle h, int64_t* row_ptr, int32_t* col) {
  if (!h || !row_ptr || !col) return fail(h, TOWR_ERR_INVALID, "null argument");
  std::memcpy(row_ptr, h->L.row_ptr.data(), sizeof(int64_t) * h->L.row_ptr.size());
  if (h->L.nnz) std::memcpy(col, h->L.col.data(), sizeof(int32_t) * h->L.col.size());
  return TOWR_OK;
}

int towr_gpu_initial_x(towr_gpu_handle h, double* x0) {
  if (!h || !x0) return fail(h, TOWR_ERR_INVALID, "null argument");
  std::memcpy(x0, h->L.x0.data(), sizeof(double) * h->L.x0.size());
  return TOWR_OK;
}

int towr_gpu_initial_x_for(towr_gpu_handle h, const towr_init_t* init, const towr_terrain_t* terrain, double* x0) {
  if (!h || !init || !terrain || !x0) return fail(h, TOWR_ERR_INVALID, "null argument");
  std::vector<double> v;
  std::string err;
  if (int rc = initial_x_for(h->L.desc, *init, *terrain, v, err)) return fail(h, rc, err);
  std::memcpy(x0, v.data(), sizeof(double) * v.size());
  return TOWR_OK;
}

int towr_gpu_varset_info(towr_gpu_handle h, int32_t i, int32_t* kind, int32_t* ee, int32_t* col0, int32_t* n) {
  if (!h || i < 0 || i >= (int32_t)h->L.varsets.size()) return fail(h, TOWR_ERR_INVALID, "bad variable set index");
  const VarSetInfo& v = h->L.varsets[i];
  if (kind) *kind = v.kind;
  if (ee) *ee = v.ee;
  if (col0) *col0 = v.col0;
  if (n) *n = v.n;
  return TOWR_OK;
}

int towr_gpu_eval_g(towr_gpu_handle h, const double* x, double* g) {
  if (!h || !x || !g) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return host_eval(h, 1, x, g, nullptr, true);
}

int towr_gpu_eval_jac_values(towr_gpu_handle h, const double* x, double* values) {
  if (!h || !x || !values) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return host_eval(h, 1, x, nullptr, values, true);
}

int towr_gpu_eval_g_jac(towr_gpu_handle h, const double* x, double* g, double* values) {
  if (!h || !x || !g || !values) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return host_eval(h, 1, x, g, values, true);
}

// IPOPT's callback pair at one x (eval_g, then eval_jac_g): towr_gpu_eval_g_keep_jac evaluates g AND the Jacobian
// into the device staging (HBM, no PCIe traffic for the values: the composers / the single launch write at device
// speed), returns g, and keeps the values with a copy of x; towr_gpu_eval_jac_values_kept then DMAs them into the
// caller's array (in place when it is registered) if x is bit-identical, else it evaluates afresh. IPOPT's values
// array is written only inside eval_jac_g, for the x it asked for. (Round 5's pair: g alone, then the Jacobian
// zero-copy over PCIe into IPOPT's registered array: 111.5 us for ANYmal gait, B = 1; this pair 91.1 us. Returning g
// before the compose launch ends, with the small kinds in a launch of their own and g copied on the copy stream after an
// event between the record and compose launches: 105.6 us, a cross-stream event costs more than the overlap gains.)
int eval_single_kept(towr_gpu_handle h, const double* x, double* g) {
  h->kept = false;
  const towr_terrain_t* ter;
  int per;
  if (int rc = batch_terrain(h, 1, true, &ter, &per)) return rc;
  if (int rc = ensure_stage(h, 1)) return rc;
  const Layout& L = h->L;
  const size_t xb = sizeof(double) * (size_t)L.n, gp = sizeof(double) * (size_t)L.m;
  const double* xd = device_view(h, x, xb);
  if (!xd) { std::memcpy(h->h_x, x, xb); xd = h->hd_x; }
  h->sync_call = true;   // (the scratch event: this call ends with a synchronisation below)
  const bool scr = uses_scratch(L);
  if (scr && h->single.n_units > 0)
    if (int rc = scratch_acquire(h, h->stream)) { h->sync_call = false; return rc; }
  int rc = h->single.n_units > 0
               ? launch_fused(h, h->single, 1, xd, L.n, h->d_g, L.m, h->d_v, L.nnz, 1, 1, h->stream, ter, per)
               : launch(h, 1, xd, L.n, h->d_g, L.m, h->d_v, L.nnz, 1, 1, h->stream, ter, per, -1);
  if (scr && h->single.n_units > 0) (void)scratch_release(h, h->stream);
  h->sync_call = false;
  double* gdst = is_registered(h, g, gp) ? g : h->h_g;
  if (rc == TOWR_OK && hipMemcpyAsync(gdst, h->d_g, gp, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
    rc = fail(h, TOWR_ERR_HIP, "hipMemcpyAsync (g) failed");
  if (hipStreamSynchronize(h->stream) != hipSuccess && rc == TOWR_OK) rc = fail(h, TOWR_ERR_HIP, "hipStreamSynchronize failed");
  if (rc) return rc;
  if (gdst != g) std::memcpy(g, h->h_g, gp);
  h->kept_x.assign(x, x + L.n);
  h->kept = true;
  return TOWR_OK;
}

int towr_gpu_eval_g_keep_jac(towr_gpu_handle h, const double* x, double* g) {
  if (!h || !x || !g) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return eval_single_kept(h, x, g);
}

int towr_gpu_eval_jac_values_kept(towr_gpu_handle h, const double* x, double* values) {
  if (!h || !x || !values) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  const Layout& L = h->L;
  if (!h->kept || h->kept_x.size() != (size_t)L.n || std::memcmp(h->kept_x.data(), x, sizeof(double) * (size_t)L.n) != 0)
    return host_eval(h, 1, x, nullptr, values, true);
  const size_t vp = sizeof(double) * (size_t)L.nnz;
  const bool vr = is_registered(h, values, vp);
  HIPCHK(h, hipMemcpyAsync(vr ? values : h->h_v, h->d_v, vp, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (!vr) par_copy(values, h->h_v, vp);
  return TOWR_OK;
}

// one problem through the staging buffers: x -> HBM, cost launch, f (and gradient) -> host
static int host_cost(towr_gpu_handle h, const double* x, double* f, double* grad) {
  if (int rc = ensure_stage(h, 1)) return rc;
  const Layout& L = h->L;
  const size_t xb = sizeof(double) * (size_t)L.n;
  std::memcpy(h->h_x, x, xb);
  HIPCHK(h, hipMemcpyAsync(h->d_x, h->h_x, xb, hipMemcpyHostToDevice, h->stream));
  if (int rc = launch_cost(h, 1, h->d_x, L.n, h->d_f, grad ? h->d_grad : nullptr, L.n, h->stream, h->d_terrain, 0)) return rc;
  double fv = 0.0;
  HIPCHK(h, hipMemcpyAsync(h->h_g, h->d_f, sizeof(double), hipMemcpyDeviceToHost, h->stream));
  if (grad) HIPCHK(h, hipMemcpyAsync(h->h_x, h->d_grad, xb, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  std::memcpy(&fv, h->h_g, sizeof(double));
  if (f) *f = fv;
  if (grad) std::memcpy(grad, h->h_x, xb);
  return TOWR_OK;
}

int towr_gpu_eval_f(towr_gpu_handle h, const double* x, double* f) {
  if (!h || !x || !f) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return host_cost(h, x, f, nullptr);
}

int towr_gpu_eval_grad_f(towr_gpu_handle h, const double* x, double* grad) {
  if (!h || !x || !grad) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  return host_cost(h, x, nullptr, grad);
}

int towr_gpu_eval_cost_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx, double* F,
                                    double* GRAD, int64_t ldgrad, void* stream) {
  if (!h || B < 0 || !X || !F) return fail(h, TOWR_ERR_INVALID, "bad argument");
  const Layout& L = h->L;
  if (ldx < L.n || (GRAD && ldgrad < L.n)) return fail(h, TOWR_ERR_INVALID, "leading dimension smaller than n");
  if (int rc = bind(h)) return rc;
  const towr_terrain_t* ter;
  int per;
  if (int rc = batch_terrain(h, B, false, &ter, &per)) return rc;
  return launch_cost(h, B, X, ldx, F, GRAD, ldgrad, reinterpret_cast<hipStream_t>(stream), ter, per);
}

int towr_gpu_trajectory_size(towr_gpu_handle h, double dt, int32_t* n_samples, int32_t* n_cols) {
  if (!h || !(dt > 0.0)) return fail(h, TOWR_ERR_INVALID, "bad argument");
  const std::vector<double> ts = traj_times(h->L, dt);
  if ((int64_t)ts.size() > kTrajMaxSamples) return fail(h, TOWR_ERR_INVALID, "too many trajectory samples");
  if (n_samples) *n_samples = (int32_t)ts.size();
  if (n_cols) *n_cols = traj_cols(h->L.rb.n_ee);
  return TOWR_OK;
}

int towr_gpu_sample_trajectory(towr_gpu_handle h, const double* x, double dt, double* out) {
  if (!h || !x || !out) return fail(h, TOWR_ERR_INVALID, "null argument");
  if (int rc = bind(h)) return rc;
  if (int rc = ensure_stage(h, 1)) return rc;
  int32_t ns = 0, cols = 0;
  if (int rc = towr_gpu_trajectory_size(h, dt, &ns, &cols)) return rc;
  const Layout& L = h->L;
  HIPCHK(h, hipMemcpyAsync(h->d_x, x, sizeof(double) * L.n, hipMemcpyHostToDevice, h->stream));
  double* d_out = nullptr;
  const size_t bytes = sizeof(double) * (size_t)ns * cols;
  HIPCHK(h, hipMalloc(&d_out, bytes));
  int rc = launch_traj(h, 1, h->d_x, L.n, dt, d_out, (int64_t)ns * cols, h->stream);
  if (rc == TOWR_OK && (hipMemcpyAsync(out, d_out, bytes, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
                        hipStreamSynchronize(h->stream) != hipSuccess))
    rc = fail(h, TOWR_ERR_HIP, "trajectory copy failed");
  (void)hipFree(d_out);
  return rc;
}

int towr_gpu_sample_trajectory_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx, double dt,
                                            double* OUT, int64_t ldo, void* stream) {
  if (!h || B < 0 || !X || !OUT) return fail(h, TOWR_ERR_INVALID, "bad argument");
  if (ldx < h->L.n) return fail(h, TOWR_ERR_INVALID, "leading dimension smaller than n");
  if (int rc = bind(h)) return rc;
  return launch_traj(h, B, X, ldx, dt, OUT, ldo, reinterpret_cast<hipStream_t>(stream));
}

int towr_gpu_set_batch_terrain(towr_gpu_handle h, int32_t B, const towr_terrain_t* terrains) {
  if (!h || B < 0 || (B > 0 && !terrains)) return fail(h, TOWR_ERR_INVALID, "bad argument");
  // The shared pattern holds only while every terrain keeps the base terrain's curvature class:
  // ForceConstraintDiscretized inserts motion entries only where f . d(basis) != 0 (quirk A22 iv).
  // The shared pattern is the description's at x0. On a terrain without curvature it never moves; on curved
  // (Gap) terrain the reference's moves with x and terrain: every problem is evaluated on the frozen pattern,
  // and towr_gpu_pattern_outside_batch_device reports what the reference would add outside it. A batch
  // terrain of another curvature class than the description's would change which blocks exist at all.
  for (int i = 0; i < B; ++i)
    if (ter_has_curvature(terrains[i].id) != ter_has_curvature(h->L.terrain.id))
      return fail(h, TOWR_ERR_UNSUPPORTED, "batch terrain changes the Jacobian pattern (curvature class differs from the base terrain)");
  if (int rc = bind(h)) return rc;
  if (h->d_bterrain) { (void)hipFree(h->d_bterrain); h->d_bterrain = nullptr; h->bterrain_n = 0; h->bterrain_h.clear(); }
  if (B == 0) return TOWR_OK;
  std::vector<towr_terrain_t> v(terrains, terrains + B);
  if (int rc = upload(h, &h->d_bterrain, v)) return rc;
  h->bterrain_h = v;
  h->bterrain_n = B;
  return TOWR_OK;
}

int towr_gpu_eval_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx, double* G, int64_t ldg,
                               double* V, int64_t ldv, int32_t want_g, int32_t want_jac, void* stream) {
  if (!h || B < 0 || !X) return fail(h, TOWR_ERR_INVALID, "bad argument");
  const Layout& L = h->L;
  if (ldx < L.n || (want_g && (!G || ldg < L.m)) || (want_jac && (!V || ldv < L.nnz)))
    return fail(h, TOWR_ERR_INVALID, "leading dimension smaller than n / m / nnz, or missing output");
  if (int rc = bind(h)) return rc;
  const towr_terrain_t* ter;
  int per;
  if (int rc = batch_terrain(h, B, false, &ter, &per)) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);   // NULL = HIP's default stream
  return launch(h, B, X, ldx, G, ldg, V, ldv, want_g, want_jac, s, ter, per, -1);
}

int towr_gpu_kernel_info(towr_gpu_handle h, int32_t kernel, const char** name, int32_t* n_tiles, int64_t* bytes_per_problem) {
  static const char* names[LC_COUNT] = {"dynamic", "range_of_motion", "force_discretized", "torque_discretized", "small_kinds"};
  if (!h || kernel < 0 || kernel >= towr_gpu_num_kernels()) return fail(h, TOWR_ERR_INVALID, "bad kernel index");
  if (kernel >= LC_COUNT) {   // fusion group slot
    const int g = kernel - LC_COUNT;
    const bool on = g < h->n_fuse;
    if (name) {
      h->fuse_name[g].clear();
      for (int lc = 0; on && lc < LC_COUNT; ++lc)
        if ((h->fuse[g].mask >> lc) & 1) h->fuse_name[g] += (h->fuse_name[g].empty() ? "" : "+") + std::string(names[lc]);
      *name = h->fuse_name[g].c_str();
    }
    if (n_tiles) *n_tiles = on ? h->fuse[g].n_units : 0;
    if (bytes_per_problem) *bytes_per_problem = on ? mask_bytes(h->L, h->fuse[g].mask) : 0;
    return TOWR_OK;
  }
  if (name) *name = names[kernel];
  if (n_tiles) *n_tiles = class_units(h->L, kernel);
  if (bytes_per_problem) *bytes_per_problem = class_bytes(h->L, kernel);
  return TOWR_OK;
}
int towr_gpu_step_launches(towr_gpu_handle h, int32_t* kernels, int32_t cap) {
  if (!h || (cap > 0 && !kernels)) return fail(h, TOWR_ERR_INVALID, "bad argument");
  int cnt = 0;
  uint32_t fused = 0;
  for (int g = 0; g < h->n_fuse; ++g) {
    if (cnt < cap) kernels[cnt] = LC_COUNT + g;
    ++cnt;
    fused |= h->fuse[g].mask;
  }
  for (int lc = 0; lc < LC_COUNT; ++lc)
    if (class_units(h->L, lc) > 0 && !((fused >> lc) & 1)) {
      if (cnt < cap) kernels[cnt] = lc;
      ++cnt;
    }
  return cnt;
}
int towr_gpu_kernel_path(towr_gpu_handle h, int32_t kernel) {
  if (!h || kernel < 0 || kernel >= LC_COUNT) return fail(h, TOWR_ERR_INVALID, "bad kernel index");
  if (class_units(h->L, kernel) == 0) return -1;
  return fstream_class(h->L, kernel) || gstream_cls(h->L, kernel) >= 0 ? 1 : 0;
}
int towr_gpu_eval_batch_device_kernel(towr_gpu_handle h, int32_t kernel, int32_t B, const double* X, int64_t ldx,
                                      double* G, int64_t ldg, double* V, int64_t ldv, void* stream) {
  if (!h || B < 0 || !X || !G || !V || kernel < 0 || kernel >= towr_gpu_num_kernels()) return fail(h, TOWR_ERR_INVALID, "bad argument");
  const Layout& L = h->L;
  if (ldx < L.n || ldg < L.m || ldv < L.nnz) return fail(h, TOWR_ERR_INVALID, "leading dimension too small");
  if (int rc = bind(h)) return rc;
  const towr_terrain_t* ter;
  int per;
  if (int rc = batch_terrain(h, B, false, &ter, &per)) return rc;
  if (kernel >= LC_COUNT) {
    const int g = kernel - LC_COUNT;
    if (g >= h->n_fuse) return fail(h, TOWR_ERR_INVALID, "no fusion group at this kernel index");
    return launch_fused(h, h->fuse[g], B, X, ldx, G, ldg, V, ldv, 1, 1, reinterpret_cast<hipStream_t>(stream), ter, per);
  }
  return launch(h, B, X, ldx, G, ldg, V, ldv, 1, 1, reinterpret_cast<hipStream_t>(stream), ter, per, kernel);
}

// The frozen-pattern check runs on the host, with the structure pass's own arithmetic (engine_math.h at the
// reference's operation order and std::pow): whether a motion block's scale is exactly 0.0 is a
// floating-point tie that the device's correctly rounded powers can resolve differently from the
// reference's libm (measured: a force residue of 2^-44 N at a phase junction on HyQ Gap).
int towr_gpu_pattern_outside_batch_device(towr_gpu_handle h, int32_t B, const double* X, int64_t ldx, int32_t* counts, void* stream) {
  if (!h || B < 0 || !X || !counts) return fail(h, TOWR_ERR_INVALID, "bad argument");
  const Layout& L = h->L;
  if (ldx < L.n) return fail(h, TOWR_ERR_INVALID, "leading dimension smaller than n");
  if (B == 0) return TOWR_OK;
  if (h->bterrain_n && h->bterrain_n != B)
    return fail(h, TOWR_ERR_INVALID, "batch terrains are set for " + std::to_string(h->bterrain_n) + " problems, the call has " + std::to_string(B));
  if (L.watch.empty()) { std::memset(counts, 0, sizeof(int32_t) * (size_t)B); return TOWR_OK; }
  if (int rc = bind(h)) return rc;
  std::vector<double> xh((size_t)B * L.n);
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  HIPCHK(h, hipMemcpy2DAsync(xh.data(), sizeof(double) * L.n, X, sizeof(double) * ldx, sizeof(double) * L.n, B, hipMemcpyDeviceToHost, s));
  HIPCHK(h, hipStreamSynchronize(s));
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const int nt = (int)std::min<int64_t>(hw, B);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      for (int b = t; b < B; b += nt)
        counts[b] = (int32_t)pattern_outside_host(L, xh.data() + (size_t)b * L.n, h->bterrain_n ? h->bterrain_h[b] : L.terrain);
    });
  for (auto& q : th) q.join();
  return TOWR_OK;
}

int towr_gpu_pattern_outside(towr_gpu_handle h, const double* x, int64_t* count) {
  if (!h || !x || !count) return fail(h, TOWR_ERR_INVALID, "null argument");
  *count = pattern_outside_host(h->L, x, h->L.terrain);   // host only: layout-only handles answer too
  return TOWR_OK;
}

int towr_gpu_eval_batch(towr_gpu_handle h, int32_t B, const double* X, double* G, double* V) {
  if (!h || B < 0 || !X) return fail(h, TOWR_ERR_INVALID, "bad argument");
  if (int rc = bind(h)) return rc;
  return host_eval(h, B, X, G, V, false);
}

int towr_gpu_register_host(towr_gpu_handle h, void* ptr, int64_t bytes) {
  if (!h || !ptr || bytes <= 0) return fail(h, TOWR_ERR_INVALID, "bad argument");
  if (int rc = bind(h)) return rc;
  const char* c = static_cast<const char*>(ptr);
  for (const auto& r : h->pinned)
    if (c < r.p + r.n && r.p < c + bytes) return fail(h, TOWR_ERR_INVALID, "range overlaps a registered range");
  HIPCHK(h, hipHostRegister(ptr, (size_t)bytes, hipHostRegisterMapped));
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess || !dev) {
    (void)hipHostUnregister(ptr);
    return fail(h, TOWR_ERR_HIP, "hipHostGetDevicePointer failed for the registered range");
  }
  h->pinned.push_back({c, (size_t)bytes, static_cast<char*>(dev)});
  return TOWR_OK;
}

int towr_gpu_unregister_host(towr_gpu_handle h, void* ptr) {
  if (!h || !ptr) return fail(h, TOWR_ERR_INVALID, "bad argument");
  for (size_t i = 0; i < h->pinned.size(); ++i)
    if (h->pinned[i].p == static_cast<const char*>(ptr)) {
      if (h->device >= 0) {
        if (int rc = bind(h)) return rc;
        HIPCHK(h, hipStreamSynchronize(h->stream));
        HIPCHK(h, hipStreamSynchronize(h->copy_stream));
        HIPCHK(h, hipHostUnregister(ptr));
      }
      h->pinned.erase(h->pinned.begin() + (std::ptrdiff_t)i);
      return TOWR_OK;
    }
  return fail(h, TOWR_ERR_INVALID, "pointer was not registered with this handle");
}

int towr_gpu_set_tiles_per_block(towr_gpu_handle h, int32_t tiles_per_block) {
  if (!h || tiles_per_block < 0) return fail(h, TOWR_ERR_INVALID, "bad argument");
  (void)tiles_per_block;   // one block per (problem, tile) since the per-type kernels; kept for ABI stability
  return TOWR_OK;
}

int64_t towr_gpu_algorithmic_bytes_per_call(towr_gpu_handle h) {
  if (!h) return 0;
  return 8 * ((int64_t)h->L.n + h->L.m + h->L.nnz) + (int64_t)sizeof(towr_terrain_t);
}

}  // extern "C"
