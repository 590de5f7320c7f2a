// TEST INFRASTRUCTURE ONLY — host emulation of towr_eval_kernel's per-item loop, used by the
// CPU test suite to check engine_math.h values against the oracle before GPU runs. It is built
// into tests/host_emu/build/libemu.so and is never linked into or loaded by the product.
#include "../../towr2025_amd/csrc/gs_cls.h"
#include "../../towr2025_amd/csrc/layout.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

using namespace tg;

namespace {
// same semantics as the kernel's TileEmit: 8 tile-relative positions per SlotGroup, one plain store
// per present candidate (a position written twice would be a layout bug: the check leaves NaN)
struct AccEmit {
  const SlotGroup* slot; int stride; double* v; double* gout; int nvals; int flo = 0, fcnt = 0; ItemDirect dd{}; int j = 0;
  static constexpr bool kFilter = true;   // row-split items (ItemDesc::rsel), as the kernel's TileEmit
  bool want(int row) const { return fcnt == 0 || (unsigned)(row - flo) < (unsigned)fcnt; }
  void g(int row, double val) { gout[row] = val; }
  void operator()(int row, int col, double val, bool) {
    if (!want(row)) return;
    int s = slot_pick(slot[(j / 8) * stride], j % 8);
    // the kernel's direct ranges (TileEmit DIRECT): must give the slot table's position
    if (col >= dd.c0[0] && col < dd.c1[0]) s = dd.off[0] + col;
    else if (col >= dd.c0[1] && col < dd.c1[1]) s = dd.off[1] + col;
    ++j;
    if (s >= nvals) return;   // the lane's dummy slot (absent candidate)
    v[s] = std::isnan(v[s]) ? val : std::nan("");
  }
  void flush() {}
};
}

extern "C" int emu_eval_ex(const towr_problem_desc_t* d, int n_data, const towr_data_t* data, const double* x, double* g,
                           double* v, char* err, int errlen) {
  Layout L; std::string e;
  int rc = build_layout_ex(*d, n_data, data, L, e);
  if (rc) { if (err) std::snprintf(err, errlen, "%s", e.c_str()); return rc; }
  std::memset(g, 0, sizeof(double) * L.m);
  for (int64_t k = 0; k < L.nnz; ++k) v[k] = std::nan("");   // every slot must be stored
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  c.gait = L.gait; c.pinfo = L.pinfo.data(); c.pcols = L.pcols.data(); c.sched = L.sched.data();
  c.eelin = L.eelin.data(); c.lin = L.lin.data(); c.rotvec = L.rotvec;
  // the small kinds see x as the kernel stages it (Layout::misc_xspan): every column outside the spans is NaN,
  // so an item reading an unstaged column fails the comparison with the oracle
  std::vector<double> xm;
  if (!L.misc_xspan.empty()) {
    xm.assign((size_t)L.n, std::nan(""));
    for (size_t k = 0; k + 1 < L.misc_xspan.size(); k += 2)
      for (int32_t u = L.misc_xspan[k]; u < L.misc_xspan[k] + L.misc_xspan[k + 1]; ++u)
        for (int j = 2 * u; j < 2 * u + 2 && j < L.n; ++j) xm[(size_t)j] = x[j];
  }
  for (const TileDesc& td : L.tiles)
    for (int l = td.i0; l < td.i1; ++l) {
      const ItemDesc& it = L.items[l];
      if (it.type == IT_NONE) continue;
      c.x = is_misc_kind(it.type) && !xm.empty() ? xm.data() : x;
      AccEmit em{L.slot_groups.data() + it.slot, td.i1 - td.i0, v + td.v0, g, td.v1 - td.v0,
                 it.rsel > 0 ? it.row0 + rsel_first(it.rsel) : 0, it.rsel > 0 ? rsel_count(it.rsel) : 0,
                 L.idirect.empty() ? ItemDirect{} : L.idirect[l]};
      c.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
      eval_item(c, it, em);
      em.flush();
    }
  c.x = x;
  if (L.fstream) {   // the kernel's streaming ForceConstraintDiscretized composition (fdisc_stream_body)
    c.pact = L.pact.data();
    for (const FsBlock& fb : L.fs_blocks) {
      std::vector<FdiscInstant> in(fb.n_inst);
      std::vector<int> ws(fb.n_inst);
      for (int k = 0; k < fb.n_inst; ++k) {
        c.seg = nullptr;
        fdisc_instant(c, fb.ee, L.fs_t[fb.t0 + k], in[k]);
        ws[k] = L.fs_ws[3 * (fb.wsoff + in[k].poly)];   // (window start, dimension codes, slot codes) triples
        for (int i = 0; i < 5; ++i) g[fb.r0 + 5 * k + i] = in[k].g[i];
      }
      for (int e = 0; e < fb.nv; ++e) {
        const int r = (int)((e + 0.5) * (1.0 / fb.L)), j = e - r * fb.L, k = r / 5, i = r - 5 * k;
        const FdiscInstant& o = in[k];
        double val = 0.0;
        if ((unsigned)(j - fb.js0) < (unsigned)fb.ns1) {
          val = fdisc_sched_value(o.b[i], o.Jf, j - fb.js0);
        } else if ((unsigned)(j - ws[k]) < (unsigned)kFsWin) {
          const int32_t te = L.fs_tmpl[fb.tmpl + j];
          if (te >= 0) {
            const double s = phase_basis_sum(L.pcols[te & 0xFFFFFF], o.poly, o.H[0], o.H[1], o.H[2], o.H[3]);
            val = s == 0.0 ? 0.0 : o.b[i][(te >> 24) & 3] * s;
          }
        }
        v[fb.v0 + e] = val;
      }
    }
  }
  if (L.gstream[GS_TQ]) {   // the streaming TorqueConstraintDiscretized composition (gstream.hip tq_records + gs_compose)
    c.pact = L.pact.data();
    constexpr int RS = kTqND + kTqNI;
    for (const GsBlock& bl : L.gs_blocks[GS_TQ]) {
      const GsGeo& gg = L.gs_geo[bl.geo];
      std::vector<double> rec((size_t)bl.n_inst * RS);
      for (int kk = 0; kk < bl.n_inst; ++kk) {   // the record lanes
        const GsInst& gi = L.gs_inst[GS_TQ][gg.rec0 + bl.k0 + kk];
        c.seg = L.segs.data() + (size_t)gi.seg * L.spl.size();
        double gq[4];
        tq_record(c, gi, [&](int f, double val) { rec[(size_t)kk * RS + f] = val; }, gq);
        for (int i = 0; i < 4; ++i) g[gi.row0 + i] = gq[i];
      }
      for (int e = 0; e < bl.nv; ++e) {   // every entry of the block's range: segment, window, value or 0
        const int kk = e / gg.Li, rr = e - kk * gg.Li;
        const GsSeg& sg = L.gs_segs[gg.seg0 + L.gs_tseg[gg.ts0 + rr]];
        const double* d = rec.data() + (size_t)kk * RS;
        const int32_t* ci = reinterpret_cast<const int32_t*>(d + kTqND);
        const int ws = sg.type == 1 ? L.gs_ws[sg.wsoff + TqCls::poly(ci, sg.kind, sg.ee)] : 0;
        const int q = rr - (sg.p0 + ws);
        v[bl.v0 + e] = q >= 0 && q < sg.W && rr < sg.p0 + sg.len
                           ? TqCls::value(L.rb, L.gs_tmpl.data(), sg, rr, d, ci, nullptr, L.sched[gg.ee].n_phases) : 0.0;
      }
    }
  }
  return 0;
}
extern "C" int emu_eval(const towr_problem_desc_t* d, const double* x, double* g, double* v, char* err, int errlen) {
  return emu_eval_ex(d, 0, nullptr, x, g, v, err, errlen);
}

// objective and dense gradient through engine_math.h's cost items (host instantiation)
namespace {
struct GradEmit {
  double* grad; double f = 0.0;
  void operator()(int, int col, double v, bool pres) { if (pres && col >= 0) grad[col] += v; }
};
}
extern "C" int emu_cost(const towr_problem_desc_t* d, const double* x, double* f, double* grad, char* err, int errlen) {
  Layout L; std::string e;
  int rc = build_layout(*d, L, e);
  if (rc) { if (err) std::snprintf(err, errlen, "%s", e.c_str()); return rc; }
  std::memset(grad, 0, sizeof(double) * L.n);
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  c.gait = L.gait; c.pinfo = L.pinfo.data(); c.pcols = L.pcols.data(); c.sched = L.sched.data();
  c.eelin = L.eelin.data(); c.rotvec = L.rotvec; c.cq = L.cost_q.data();
  GradEmit em{grad};
  for (const CostItem& it : L.cost_items) {
    c.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
    eval_cost_item(c, it, em);
  }
  *f = em.f;
  return 0;
}

// The objective kernel's deterministic gradient (cost_traj.hip) on the host, with its own emitters:
// acc 1 = the slot path (returns 1 when the layout has no slots), 2 = the fixed-point limb path.
extern "C" int emu_cost_acc(const towr_problem_desc_t* d, const double* x, int acc, double* f, double* grad) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  if (acc == 1 && L.cost_nslot == 0) return 1;
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  c.gait = L.gait; c.pinfo = L.pinfo.data(); c.pcols = L.pcols.data(); c.pact = L.pact.data(); c.sched = L.sched.data();
  c.eelin = L.eelin.data(); c.rotvec = L.rotvec; c.cq = L.cost_q.data();
  const int n_pad = (L.n + 2) & ~1;
  std::vector<double> cs((size_t)std::max(1, L.cost_nslot), std::nan(""));
  std::vector<unsigned long long> lacc(3 * (size_t)n_pad, 0);
  int bad = 0;
  double fs = 0.0;
  for (const CostItem& it : L.cost_items) {
    c.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
    if (acc == 1) {
      CostSlotEmit em{cs.data(), L.cost_cslot.data() + it.cslot, L.n};
      eval_cost_item(c, it, em);
      if (em.slot != L.cost_cslot.data() + it.cslot + it.cn) return 2;   // the host pass's slot count disagrees
      fs += em.f;
    } else {
      CostLimbEmit em{lacc.data(), n_pad, &bad};
      eval_cost_item(c, it, em);
      fs += em.f;
    }
  }
  for (int j = 0; j < L.n; ++j) {
    if (acc == 1) {
      double s = 0.0;
      for (int k = L.cost_cptr[j]; k < L.cost_cptr[j + 1]; ++k) s += cs[k];
      grad[j] = s;
    } else {
      grad[j] = bad ? std::nan("") : limb_value((long long)lacc[j], (long long)lacc[n_pad + j], (long long)lacc[2 * n_pad + j]);
    }
  }
  *f = fs;
  return 0;
}

namespace {
struct CountEmit {
  static constexpr bool kSparse = true;
  double f = 0.0; long emits = 0, pres = 0; std::vector<int>* colcnt;
  void skip(int) {}
  void operator()(int, int col, double, bool p) { ++emits; if (p && col >= 0) { ++pres; ++(*colcnt)[col]; } }
};
}
// cost work statistics at x (experiment aid): items per type, emissions, contributions per column
extern "C" int emu_cost_stats(const towr_problem_desc_t* d, const double* x) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  std::vector<int> colcnt(L.n + 1, 0);
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  c.gait = L.gait; c.pinfo = L.pinfo.data(); c.pcols = L.pcols.data(); c.pact = L.pact.data(); c.sched = L.sched.data();
  c.eelin = L.eelin.data(); c.rotvec = L.rotvec; c.cq = L.cost_q.data();
  long n_t[CT_COUNT] = {}, em_t[CT_COUNT] = {}, pr_t[CT_COUNT] = {}, mx_t[CT_COUNT] = {};
  for (const CostItem& it : L.cost_items) {
    if (it.type >= CT_COUNT) continue;   // a no-op lane of the wave schedule
    c.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
    CountEmit em{}; em.colcnt = &colcnt;
    eval_cost_item(c, it, em);
    n_t[it.type]++; em_t[it.type] += em.emits; pr_t[it.type] += em.pres; mx_t[it.type] = std::max(mx_t[it.type], em.emits);
  }
  for (int t = 0; t < CT_COUNT; ++t)
    if (n_t[t]) std::printf("cost type %d: items %ld emits %ld present %ld max/item %ld\n", t, n_t[t], em_t[t], pr_t[t], mx_t[t]);
  int touched = 0, mx = 0; long tot = 0;
  for (int j = 0; j < L.n; ++j) if (colcnt[j]) { ++touched; mx = std::max(mx, colcnt[j]); tot += colcnt[j]; }
  std::printf("n %d touched %d contributions %ld max/col %d\n", L.n, touched, tot, mx);
  return 0;
}

// The composers' encoding bounds over every streamed block (layout.h kFloatDivMax, GsSeg int16 positions):
// out[0..2] per GsClass: streamed (0/1); out[3..5]: its largest positions per instant (Lsum, GsGeo::Li);
// out[6]: the largest CSR range of any FsBlock or GsBlock; out[7]: FDISC streamed
extern "C" int emu_stream_limits(const towr_problem_desc_t* d, int64_t* out) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  int64_t nv = 0;
  for (int c = 0; c < GS_COUNT; ++c) {
    out[c] = L.gstream[c];
    int64_t li = 0;
    for (const GsGeo& g : L.gs_geo) if (g.cls == c) li = std::max<int64_t>(li, g.Li);
    out[3 + c] = li;
    for (const GsBlock& bl : L.gs_blocks[c]) nv = std::max<int64_t>(nv, bl.nv);
  }
  for (const FsBlock& fb : L.fs_blocks) nv = std::max<int64_t>(nv, fb.nv);
  out[6] = nv;
  out[7] = L.fstream;
  return 0;
}

// the small kinds' staged x (Layout::misc_xspan): out = {spans, 16-byte units staged, units of all of x}
extern "C" int emu_misc_xspan(const towr_problem_desc_t* d, int64_t* out) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  int64_t units = 0;
  for (size_t k = 1; k < L.misc_xspan.size(); k += 2) units += L.misc_xspan[k];
  out[0] = (int64_t)L.misc_xspan.size() / 2;
  out[1] = units;
  out[2] = (L.n + 1) / 2;
  return 0;
}

// layout statistics per item type (tiles, lanes used, candidates per wave, values per tile)
extern "C" int emu_stats(const towr_problem_desc_t* d) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  std::printf("fs tables: fs_t %zu fs_tmpl %zu fs_ws %zu fs_blocks %zu (bytes %zu)\n", L.fs_t.size(), L.fs_tmpl.size(), L.fs_ws.size(),
              L.fs_blocks.size(), 8 * L.fs_t.size() + 4 * L.fs_tmpl.size() + 4 * L.fs_ws.size() + sizeof(FsBlock) * L.fs_blocks.size() + 12 * L.fs_t.size());
  std::printf("fstream %d blocks %zu tmpl_max %d | gstream rom %d (%zu blocks) dyn %d (%zu blocks) tq %d (%zu blocks)\n", (int)L.fstream,
              L.fs_blocks.size(), L.fs_tmpl_max, (int)L.gstream[GS_ROM], L.gs_blocks[GS_ROM].size(), (int)L.gstream[GS_DYN],
              L.gs_blocks[GS_DYN].size(), (int)L.gstream[GS_TQ], L.gs_blocks[GS_TQ].size());
  std::printf("n %d m %d nnz %lld nodecol %zu | gait tables: spl %zu pinfo %zu pcols %zu pact %zu sched %zu\n", L.n, L.m,
              (long long)L.nnz, L.nodecol.size(), L.spl.size(), L.pinfo.size(), L.pcols.size(), L.pact.size(), L.sched.size());
  {
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    int phs = 0;
    for (const SchedInfo& si : L.sched) phs = std::max(phs, (int)si.n_phases);
    const size_t tabs = a16(sizeof(SplineMeta) * L.spl.size()) + a16(sizeof(SchedInfo) * L.sched.size()) + a16(sizeof(PolyPhase) * L.pinfo.size()) +
                        a16(sizeof(int32_t) * L.pact.size()) + a16(sizeof(PhaseCol) * L.pcols.size());
    std::printf("record staging bytes: x %zu nodecol %zu tables %zu (spl %zu pinfo %zu pact %zu pcols %zu) timings %zu | state euler %zu rv %zu\n",
                8 * (size_t)((L.n + 2) & ~1), 16 * ((L.nodecol.size() + 3) / 4), tabs, sizeof(SplineMeta) * L.spl.size(),
                sizeof(PolyPhase) * L.pinfo.size(), sizeof(int32_t) * L.pact.size(), sizeof(PhaseCol) * L.pcols.size(),
                8 * (2 * L.pinfo.size() + L.sched.size() * phs), sizeof(DynEulerState), sizeof(DynRvState));
  }
  for (int cls = 0; cls < GS_COUNT; ++cls) {
    if (!L.gstream[cls]) continue;
    long nv = 0; int maxnv = 0;
    for (const GsBlock& bl : L.gs_blocks[cls]) { nv += bl.nv; maxnv = std::max(maxnv, bl.nv); }
    std::printf("gstream %d: instants %zu blocks %zu nmax %d geo_max {%d %d %d %d} values %ld max/block %d\n", cls, L.gs_inst[cls].size(),
                L.gs_blocks[cls].size(), L.gs_nmax[cls], L.gs_geo_max[cls][0], L.gs_geo_max[cls][1], L.gs_geo_max[cls][2],
                L.gs_geo_max[cls][3], nv, maxnv);
  }
  for (int t = 0; t < IT_COUNT; ++t) {
    int nt = L.type_tile0[t + 1] - L.type_tile0[t];
    if (!nt) continue;
    long used = 0, lanes = 0, candw = 0, cand = 0; int maxv = 0;
    for (int ti = L.type_tile0[t]; ti < L.type_tile0[t + 1]; ++ti) {
      const TileDesc& td = L.tiles[ti];
      maxv = std::max(maxv, td.v1 - td.v0);
      for (int w = td.i0; w < td.i1; w += 64) {
        int mc = 0;
        for (int l = w; l < std::min(w + 64, td.i1); ++l) {
          ++lanes;
          if (L.items[l].type != IT_NONE) { ++used; mc = std::max(mc, L.items[l].ncand); cand += L.items[l].ncand; }
        }
        candw += mc;
      }
    }
    std::printf("type %d: tiles %d block %d lanes %ld used %ld maxvals %d cand %ld sum_wave_maxcand %ld lds %d\n", t, nt,
                L.type_block[t], lanes, used, maxv, cand, candw, L.type_lds[t]);
  }
  return 0;
}

// LDS bank-conflict degree of the tile emission (ds_write_b64: 4 groups of 16 lanes, bank pair =
// double position mod 16): per item type, LDS cycles spent / conflict-free cycles, with the
// position map `swz` applied (0 = identity, 1 = the kernel's XOR swizzle)
extern "C" int emu_conflicts(const towr_problem_desc_t* d, int swz) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  for (int t = 0; t < IT_COUNT; ++t) {
    long cyc = 0, ideal = 0, wc[4] = {0, 0, 0, 0}, wi[4] = {0, 0, 0, 0};
    for (int ti = L.type_tile0[t]; ti < L.type_tile0[t + 1]; ++ti) {
      const TileDesc& td = L.tiles[ti];
      const int block = td.i1 - td.i0;
      for (int w = 0; w < block; w += 64) {
        int maxc = 0;
        for (int l = w; l < w + 64 && l < block; ++l)
          if (L.items[td.i0 + l].type != IT_NONE) maxc = std::max(maxc, L.items[td.i0 + l].ncand);
        for (int j = 0; j < maxc; ++j)
          for (int g = 0; g < 4; ++g) {
            int cnt[16] = {0}; bool any = false;
            for (int l = w + 16 * g; l < w + 16 * g + 16 && l < block; ++l) {
              const ItemDesc& it = L.items[td.i0 + l];
              if (it.type == IT_NONE || j >= it.ncand) continue;
              int pos = slot_pick(L.slot_groups[it.slot + (size_t)(j / 8) * block], j % 8);
              if (swz == 1 && pos < td.v1 - td.v0) { const int q = pos + (td.v0 & 1); pos = q ^ (((q >> 5) & 15) << 1); }
              if (swz == 2 && pos < td.v1 - td.v0) { const int q = pos + (td.v0 & 1); pos = q ^ (((q >> 4) & 7) << 1); }
              if (swz == 3 && pos < td.v1 - td.v0) { const int q = pos + (td.v0 & 1); pos = q ^ ((((q >> 4) ^ (q >> 7)) & 7) << 1); }
              cnt[pos & 15]++; any = true;
            }
            if (!any) continue;
            int m = 0; for (int q = 0; q < 16; ++q) m = std::max(m, cnt[q]);
            cyc += m; ideal += 1;
            if (w / 64 < 4) { wc[w / 64] += m; wi[w / 64] += 1; }
          }
      }
    }
    if (ideal) std::printf("type %d: lds write cycles %ld conflict-free %ld (x%.2f)  per wave %ld/%ld %ld/%ld %ld/%ld %ld/%ld\n", t, cyc, ideal,
                           (double)cyc / ideal, wc[0], wi[0], wc[1], wi[1], wc[2], wi[2], wc[3], wi[3]);
  }
  return 0;
}

// trajectory rows through engine_math.h's traj_row (host instantiation)
extern "C" int emu_traj(const towr_problem_desc_t* d, const double* x, double dt, double* out, int max_rows) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  std::vector<double> pd((size_t)TOWR_MAX_EE * TOWR_MAX_PHASES, 0.0);
  std::vector<int32_t> pn(TOWR_MAX_EE, 0), pc(TOWR_MAX_EE, 0);
  for (int ee = 0; ee < d->robot.n_ee; ++ee) {
    pn[ee] = d->n_phases[ee]; pc[ee] = d->contact_at_start[ee] != 0;
    for (int q = 0; q < d->n_phases[ee]; ++q) pd[(size_t)ee * TOWR_MAX_PHASES + q] = d->phase_durations[ee][q];
  }
  TrajPhases ph{pd.data(), pn.data(), pc.data()};
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  c.gait = L.gait; c.pinfo = L.pinfo.data(); c.pcols = L.pcols.data(); c.sched = L.sched.data();
  c.eelin = L.eelin.data(); c.rotvec = L.rotvec;
  double T = 0.0;
  for (int i = 0; i < L.spl[0].n_polys; ++i) T += L.dur[L.spl[0].dur_off + i];
  const int cols = traj_cols(L.rb.n_ee);
  int k = 0;
  for (double t = 0.0; t <= T + 1e-9; t += dt, ++k)
    if (k < max_rows) traj_row(c, ph, t, out + (size_t)k * cols, 1);
  return k;
}

// whether every polynomial's active-window PhaseCols (pact window, then up to kGsAct entries: n, ids, derivs) coincide
// over the three dimensions, per spline (experiment aid: the record composers' window sums per dimension)
extern "C" int emu_window_dims(const towr_problem_desc_t* d) {
  Layout L; std::string e;
  if (build_layout(*d, L, e)) return -1;
  for (size_t s = 0; s < L.spl.size(); ++s) {
    const SplineMeta& m = L.spl[s];
    if (m.ee < 0) continue;
    int same = 1;
    for (int p = 0; p < m.n_polys && same; ++p) {
      int a[3], z[3];
      for (int k = 0; k < 3; ++k) { a[k] = L.pact[m.pact_off + 2 * (k * m.n_polys + p)]; z[k] = L.pact[m.pact_off + 2 * (k * m.n_polys + p) + 1]; }
      for (int k = 1; k < 3 && same; ++k) {
        if (z[k] - a[k] != z[0] - a[0]) { same = 0; break; }
        for (int q = 0; q < kGsAct && a[0] + q <= z[0]; ++q) {
          const PhaseCol& c0 = L.pcols[m.pcol_off[0] + a[0] + q];
          const PhaseCol& ck = L.pcols[m.pcol_off[k] + a[k] + q];
          if (c0.n != ck.n) { same = 0; break; }
          for (int j = 0; j < c0.n; ++j) if (c0.id[j] != ck.id[j] || c0.deriv[j] != ck.deriv[j]) same = 0;
        }
      }
    }
    std::printf("spline %zu ee %d: dims coincide %d\n", s, m.ee, same);
  }
  return 0;
}
