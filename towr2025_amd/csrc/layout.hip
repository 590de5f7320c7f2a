// layout.hip — host-side problem builder (see layout.h). Compiled by hipcc as host code; it
// instantiates engine_math.h's item evaluators with a recording emitter to obtain the exact
// candidate (row, col) list of every work item (the structure pass) — no g/J values leave here.
#include "layout.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <unordered_map>

namespace tg {
namespace {

struct Nvi { int id, deriv, dim; };
struct PolyInfo { int phase, poly_in_phase, n_polys_in_phase, is_constant; };

// NodesVariables state needed at setup: index maps and (initial) node values.
struct NodeSet {
  int kind = 0, ee = 0, n_nodes = 0, n_rows = 0, col0 = -1;
  bool all = false;
  std::vector<PolyInfo> pinfo;
  std::vector<std::vector<Nvi>> map;   // opt index -> node values
  std::vector<double> val;             // [node][deriv][dim]

  std::vector<Nvi> info(int idx) const {   // GetNodeValuesInfo
    if (all) { int in = idx % 6; return {Nvi{idx / 6, in < 3 ? kPos : kVel, in % 3}}; }
    return map[idx];
  }
  double& v(int node, int deriv, int dim) { return val[(node * 2 + deriv) * 3 + dim]; }
  bool is_constant_node(int node) const {   // nodes_variables_phase_based.cc:101-113
    int last = n_nodes - 1;
    if (node == 0) return pinfo[0].is_constant;
    if (node == last) return pinfo[last - 1].is_constant;
    return pinfo[node - 1].is_constant || pinfo[node].is_constant;
  }
  int phase_of(int node) const {            // GetPhase :133-140
    int poly = node == 0 ? 0 : (node == n_nodes - 1 ? n_nodes - 2 : node - 1);
    return pinfo[poly].phase;
  }
  int node_at_start_of_phase(int phase) const {   // :142-165
    for (int i = 0; i < (int)pinfo.size(); ++i) if (pinfo[i].phase == phase) return i;
    return -1;
  }
};

NodeSet make_all(int kind, int n_nodes) {           // nodes_variables_all.cc:34-43
  NodeSet s; s.kind = kind; s.all = true; s.n_nodes = n_nodes; s.n_rows = n_nodes * 6;
  s.val.assign((size_t)n_nodes * 6, 0.0);
  return s;
}

// nodes_variables_phase_based.cc:39-73 + GetPhaseBasedEEParameterization (:201-396)
NodeSet make_phase_based(int kind, int ee, int phase_count, bool contact_at_start, int n_changing) {
  NodeSet s; s.kind = kind; s.ee = ee;
  bool first_constant = (kind == TOWR_VAR_EE_MOTION || kind == TOWR_VAR_EE_ANG) ? contact_at_start : !contact_at_start;
  bool c = first_constant;
  for (int i = 0; i < phase_count; ++i) {
    if (c) s.pinfo.push_back({i, 0, 1, 1});
    else for (int j = 0; j < n_changing; ++j) s.pinfo.push_back({i, j, n_changing, 0});
    c = !c;
  }
  s.n_nodes = (int)s.pinfo.size() + 1;
  s.val.assign((size_t)s.n_nodes * 6, 0.0);
  int idx = 0;
  auto push = [&](int i, int id, int deriv, int dim) {
    if ((int)s.map.size() <= i) s.map.resize(i + 1);
    s.map[i].push_back(Nvi{id, deriv, dim});
  };
  for (int id = 0; id < s.n_nodes; ++id) {
    if (!s.is_constant_node(id)) {
      for (int dim = 0; dim < 3; ++dim) {
        push(idx++, id, kPos, dim);
        if (kind == TOWR_VAR_EE_MOTION && dim == Z) continue;   // swing z-velocity fixed to 0
        push(idx++, id, kVel, dim);
      }
    } else {
      if (kind == TOWR_VAR_EE_MOTION || kind == TOWR_VAR_EE_ANG) {
        for (int dim = 0; dim < 3; ++dim) { push(idx, id, kPos, dim); push(idx, id + 1, kPos, dim); ++idx; }
      }
      id += 1;   // the next (constant) node is handled with this one
    }
  }
  s.n_rows = idx;
  return s;
}

void set_linear(NodeSet& s, const double ini[3], const double fin[3], double T) {   // nodes_variables.cc:131-154
  double dp[3], avg[3];
  for (int k = 0; k < 3; ++k) { dp[k] = fin[k] - ini[k]; avg[k] = dp[k] / T; }
  for (int idx = 0; idx < s.n_rows; ++idx)
    for (const Nvi& q : s.info(idx)) {
      if (q.deriv == kPos) s.v(q.id, kPos, q.dim) = ini[q.dim] + q.id / (double)(s.n_nodes - 1) * dp[q.dim];
      if (q.deriv == kVel) s.v(q.id, kVel, q.dim) = avg[q.dim];
    }
}

void rot(const double rpy[3], double R[3][3]) { euler_R(trig(rpy), R); }

std::vector<double> get_values(const NodeSet& s) {   // nodes_variables.cc:56-66
  std::vector<double> x((size_t)s.n_rows);
  NodeSet& m = const_cast<NodeSet&>(s);
  for (int idx = 0; idx < s.n_rows; ++idx)
    for (const Nvi& q : s.info(idx)) x[idx] = m.v(q.id, q.deriv, q.dim);
  return x;
}
void set_values(NodeSet& s, const std::vector<double>& x) {
  for (int idx = 0; idx < s.n_rows; ++idx)
    for (const Nvi& q : s.info(idx)) s.v(q.id, q.deriv, q.dim) = x[idx];
}

// nodes_variables.cc:157-217
void set_linear_rel_base(NodeSet& s, const double ee0[3], const double ee1[3], const double b0[3], const double b1[3],
                         const double rpy0[3], const double rpy1[3], double T) {
  const int N = s.n_nodes;
  if (N < 2) return;
  double R0[3][3], RT[3][3], r0B[3], rTB[3], dpB[3], avgB[3], bavg[3], d0[3], dT[3];
  rot(rpy0, R0); rot(rpy1, RT);
  for (int k = 0; k < 3; ++k) { d0[k] = ee0[k] - b0[k]; dT[k] = ee1[k] - b1[k]; }
  for (int i = 0; i < 3; ++i) {
    r0B[i] = R0[0][i] * d0[0] + R0[1][i] * d0[1] + R0[2][i] * d0[2];
    rTB[i] = RT[0][i] * dT[0] + RT[1][i] * dT[1] + RT[2][i] * dT[2];
  }
  for (int k = 0; k < 3; ++k) { dpB[k] = rTB[k] - r0B[k]; avgB[k] = dpB[k] / T; bavg[k] = (b1[k] - b0[k]) / T; }
  for (int idx = 0; idx < s.n_rows; ++idx)
    for (const Nvi& q : s.info(idx)) {
      double a = q.id / (double)(N - 1), bp[3], rpy[3], R[3][3], rB[3];
      for (int k = 0; k < 3; ++k) {
        bp[k] = (1.0 - a) * b0[k] + a * b1[k];
        rpy[k] = (1.0 - a) * rpy0[k] + a * rpy1[k];
        rB[k] = r0B[k] + a * dpB[k];
      }
      rot(rpy, R);
      const int d = q.dim;
      if (q.deriv == kPos) s.v(q.id, kPos, d) = bp[d] + (R[d][0] * rB[0] + R[d][1] * rB[1] + R[d][2] * rB[2]);
      if (q.deriv == kVel) s.v(q.id, kVel, d) = bavg[d] + (R[d][0] * avgB[0] + R[d][1] * avgB[1] + R[d][2] * avgB[2]);
    }
  set_values(s, get_values(s));   // SetVariables(GetValues())
}

// recording emitter of the structure pass
struct RecordEmit {
  std::vector<int32_t>* rows;
  std::vector<int32_t>* cols;
  std::vector<uint8_t>* present;
  int g_rows_lo = 0, g_rows_hi = 0;
  bool bad_g = false;
  void g(int row, double) { if (row < g_rows_lo || row >= g_rows_hi) bad_g = true; }
  // row-split items (ItemDesc::rsel): only the selected rows' candidates, as the kernel's TileEmit
  int flo = 0, fcnt = 0;   // rows flo .. flo + fcnt - 1, fcnt 0 = all
  static constexpr bool kFilter = true;
  bool want(int row) const { return fcnt == 0 || (unsigned)(row - flo) < (unsigned)fcnt; }
  void operator()(int row, int col, double, bool pres) {
    if (!want(row)) return;
    rows->push_back(row); cols->push_back(col); present->push_back(pres && col >= 0 ? 1 : 0);
  }
};


// NodesVariables of every spline, in spline order: base-lin, base-ang, per ee {motion, ang, force, torque}
int make_sets(const towr_problem_desc_t& d, std::vector<double>& base_d, std::vector<NodeSet>& sets, std::string& err) {
  const int E = d.robot.n_ee;
  const double T = d.total_time;
  // ---- base polynomial durations (parameters.cc:114-130)
  { double dt = d.duration_base_polynomial, tl = T;
    while (tl > 1e-10) { base_d.push_back(tl > dt ? dt : tl); tl -= dt; } }

  // ---- node sets
  sets.push_back(make_all(TOWR_VAR_BASE_LIN, (int)base_d.size() + 1));
  sets.push_back(make_all(TOWR_VAR_BASE_ANG, (int)base_d.size() + 1));
  for (int ee = 0; ee < E; ++ee) {
    const int np = d.n_phases[ee];
    if (np < 1 || np > TOWR_MAX_PHASES) { err = "n_phases out of range"; return TOWR_ERR_INVALID; }
    const bool cs = d.contact_at_start[ee] != 0;
    sets.push_back(make_phase_based(TOWR_VAR_EE_MOTION, ee, np, cs, d.ee_polynomials_per_swing_phase));
    sets.push_back(make_phase_based(TOWR_VAR_EE_ANG, ee, np, cs, d.ee_polynomials_per_swing_phase));
    sets.push_back(make_phase_based(TOWR_VAR_EE_FORCE, ee, np, cs, d.force_polynomials_per_stance_phase));
    sets.push_back(make_phase_based(TOWR_VAR_EE_TORQUE, ee, np, cs, d.torque_polynomials_per_stance_phase));
  }
  return TOWR_OK;
}

// initial node values (nlp_formulation.cc:121-346, or procedural_example.cc:134-166)
int init_values(const towr_problem_desc_t& d, const towr_init_t& in, const towr_terrain_t& ter, std::vector<NodeSet>& sets, std::string& err) {
  const int E = d.robot.n_ee;
  const double T = d.total_time;
  const towr_robot_t& rb = d.robot;
  const double z3[3] = {0, 0, 0};
  if (in.mode == TOWR_INIT_FORMULATION) {
    double fp[3] = {in.base_lin_p1[0], in.base_lin_p1[1], 0.0};
    fp[2] = ter_h(ter, fp[0], fp[1]) - rb.nominal_stance[0][2];
    set_linear(sets[0], in.base_lin_p0, fp, T);
    set_linear(sets[1], in.base_ang_p0, in.base_ang_p1, T);
    for (int ee = 0; ee < E; ++ee) {
      double yaw[3] = {0.0, 0.0, in.base_ang_p1[2]}, R[3][3], fe[3];
      rot(yaw, R);
      for (int q = 0; q < 3; ++q)
        fe[q] = in.base_lin_p1[q] + (R[q][0] * rb.nominal_stance[ee][0] + R[q][1] * rb.nominal_stance[ee][1] + R[q][2] * rb.nominal_stance[ee][2]);
      double tgt[3] = {fe[0], fe[1], ter_h(ter, fe[0], fe[1])};
      set_linear_rel_base(sets[2 + 4 * ee], in.ee_p0[ee], tgt, in.base_lin_p0, in.base_lin_p1, in.base_ang_p0, in.base_ang_p1, T);
      set_linear(sets[3 + 4 * ee], in.base_ang_p0, in.base_ang_p1, T);
      double fs[3] = {0.0, 0.0, rb.mass * rb.gravity / E};
      set_linear(sets[4 + 4 * ee], fs, fs, T);
      set_linear(sets[5 + 4 * ee], z3, z3, T);
    }
  } else if (in.mode == TOWR_INIT_PROCEDURAL) {
    set_linear(sets[0], in.base_lin_p0, in.base_lin_p1, T);
    set_linear(sets[1], in.base_ang_p0, in.base_ang_p1, T);
    for (int ee = 0; ee < E; ++ee) {
      set_linear(sets[2 + 4 * ee], in.ee_p0[ee], in.ee_p1[ee], T);
      set_linear(sets[3 + 4 * ee], in.base_ang_p0, in.base_ang_p1, T);
      double fs[3] = {0.0, 0.0, rb.mass * rb.gravity / E};
      set_linear(sets[4 + 4 * ee], fs, fs, T);
      set_linear(sets[5 + 4 * ee], z3, z3, T);
    }
  } else { err = "unknown init mode"; return TOWR_ERR_INVALID; }
  return TOWR_OK;
}

// columns of every variable set in AddVariableSet order: node sets get NodeSet::col0, schedule
// sets (PhaseDurations, n_phases - 1 variables, phase_durations.cc:41-77) fill sched[ee]
int assign_columns(const towr_problem_desc_t& d, std::vector<NodeSet>& sets, std::vector<VarSetInfo>& vs,
                   std::vector<SchedInfo>& sched, std::string& err) {
  const int E = d.robot.n_ee;
  sched.assign((size_t)E, SchedInfo{-1, 0, 0.0});
  vs.clear();
  int col = 0;
  for (int i = 0; i < d.n_varsets; ++i) {
    const int kind = d.varsets[i].kind, ee = d.varsets[i].ee;
    if (kind != TOWR_VAR_BASE_LIN && kind != TOWR_VAR_BASE_ANG && (ee < 0 || ee >= E)) { err = "variable set endeffector out of range"; return TOWR_ERR_INVALID; }
    int n = 0;
    if (kind == TOWR_VAR_EE_SCHEDULE) {
      if (!d.optimize_timings) { err = "ee-schedule variables require optimize_timings"; return TOWR_ERR_INVALID; }
      if (sched[ee].col0 >= 0) { err = "variable set listed twice"; return TOWR_ERR_INVALID; }
      double tt = 0.0;
      for (int ph = 0; ph < d.n_phases[ee]; ++ph) tt += d.phase_durations[ee][ph];   // t_total_ (:47-50)
      sched[ee] = SchedInfo{col, d.n_phases[ee], tt};
      n = d.n_phases[ee] - 1;
    } else {
      int si = -1;
      switch (kind) {
        case TOWR_VAR_BASE_LIN: si = 0; break;
        case TOWR_VAR_BASE_ANG: si = 1; break;
        case TOWR_VAR_EE_MOTION: si = 2 + 4 * ee; break;
        case TOWR_VAR_EE_ANG: si = 3 + 4 * ee; break;
        case TOWR_VAR_EE_FORCE: si = 4 + 4 * ee; break;
        case TOWR_VAR_EE_TORQUE: si = 5 + 4 * ee; break;
        default: err = "unknown variable set kind " + std::to_string(kind); return TOWR_ERR_INVALID;
      }
      if (sets[si].col0 >= 0) { err = "variable set listed twice"; return TOWR_ERR_INVALID; }
      sets[si].col0 = col;
      n = sets[si].n_rows;
    }
    vs.push_back({kind, ee, col, n});
    col += n;
  }
  for (auto& st : sets)
    if (st.col0 < 0) { err = "every node variable set (base-lin, base-ang, ee motion/ang/force/torque) must be in the problem"; return TOWR_ERR_INVALID; }
  if (d.optimize_timings)
    for (int ee = 0; ee < E; ++ee)
      if (sched[ee].col0 < 0) { err = "optimize_timings needs the ee-schedule variable set of every endeffector"; return TOWR_ERR_INVALID; }
  return col;
}

// x0 of every set (node values; schedule = the first n_phases - 1 durations, phase_durations.cc:68-77)
void fill_x0(const towr_problem_desc_t& d, std::vector<NodeSet>& sets, const std::vector<SchedInfo>& sched, int n, std::vector<double>& x0) {
  x0.assign((size_t)n, 0.0);
  for (auto& st : sets) { auto v = get_values(st); std::copy(v.begin(), v.end(), x0.begin() + st.col0); }
  for (int ee = 0; ee < (int)sched.size(); ++ee)
    if (sched[ee].col0 >= 0)
      for (int ph = 0; ph < sched[ee].n_phases - 1; ++ph) x0[(size_t)sched[ee].col0 + ph] = d.phase_durations[ee][ph];
}

int item_rows(int type) {
  switch (type) {
    case IT_DYN: case IT_BMOT: return 6;
    case IT_ROM: case IT_SACC: return 3;
    case IT_FDISC: case IT_FNODE: return 5;
    case IT_TERR: case IT_BHGT: case IT_TDUR: case IT_THARD: case IT_EELIN: case IT_LINEQ: return 1;
    case IT_TQDISC: return 4;
    case IT_TQNODE: return 3;
    case IT_SWING: return 4;
  }
  return 0;
}

// one segment-table row: the reference's GetLocalTime scan of every spline at time t
int push_seg_row(Layout& L, double t) {
  const int nspl = (int)L.spl.size();
  const int row = (int)(L.segs.size() / nspl);
  for (int sp = 0; sp < nspl; ++sp) {
    SegRec r{};
    r.poly = seg_lookup(L.dur.data() + L.spl[sp].dur_off, L.spl[sp].n_polys, t, &r.tl);
    r.T = L.dur[L.spl[sp].dur_off + r.poly];
    hermite_dpos(r.T, r.tl, r.H[kPos]);   // polynomial.cc:135-234, batch-invariant
    hermite_dvel(r.T, r.tl, r.H[kVel]);
    hermite_dacc(r.T, r.tl, r.H[kAcc]);
    for (int bb = 0; bb < 4; ++bb)
      for (int e = 0; e < 3; ++e) {
        const int32_t col = L.nodecol[(size_t)(L.spl[sp].node_off + r.poly + (bb >> 1)) * 6 + (bb & 1) * 3 + e];
        r.col[bb][e] = col >= 0 ? col : L.n;
      }
    L.segs.push_back(r);
  }
  return row;
}

// cost work items (NlpFormulation::GetCosts, nlp_formulation.cc:604-680), grouped by type
constexpr int kNodeChunk = 4;   // NodeCost nodes per work item
// The cost kernel's wave schedule (cost_traj.hip: item i runs on lane i % kCostLanes in round i / kCostLanes, so in
// wave (i % kCostLanes) / 64). A wave's time is the sum over its rounds of its slowest item, and a wave whose lanes
// hold two kinds runs both paths. So each kind's items (sorted by kind) go in chunks of 64 lanes, one chunk per
// (round, wave), and the chunks are dealt to the waves heaviest first, each to the wave with the least work so far
// (longest processing time first): every wave runs one kind per round and the waves' loads are level. Lanes left
// over hold a no-op item (type CT_COUNT). The relative latencies per kind are from tools/cost_timing.py (MI355X,
// ANYmal, f + gradient of each kind alone).
std::vector<CostItem> cost_wave_schedule(const std::vector<CostItem>& items) {
#if defined(TOWR_COST_SCHED) && TOWR_COST_SCHED == 0   // (experiment builds: the items in kind order, round-robin)
  return items;
#endif
  constexpr int W = kCostLanes / 64;
  auto weight = [](int type) {
    switch (type) {
      case CT_EEBP: return 5.0;
      case CT_ANGMOM: return 3.0;
      case CT_ENERGY: return 3.0;
      case CT_BHC: return 2.0;
      case CT_ENERGYQ: return 1.5;
      default: return 1.0;
    }
  };
  struct Chunk { size_t i0, n; double w; };
  std::vector<Chunk> chunks;
  for (size_t i = 0; i < items.size();) {
    size_t j = i;
    while (j < items.size() && items[j].type == items[i].type && j - i < 64) ++j;
    chunks.push_back({i, j - i, weight(items[i].type)});
    i = j;
  }
  std::stable_sort(chunks.begin(), chunks.end(), [](const Chunk& a, const Chunk& b) { return a.w > b.w; });
  std::vector<std::vector<const Chunk*>> per(W);
  double load[W] = {};
  for (const Chunk& c : chunks) {
    const int w = (int)(std::min_element(load, load + W) - load);
    per[w].push_back(&c);
    load[w] += c.w;
  }
  size_t rounds = 0;
  for (const auto& v : per) rounds = std::max(rounds, v.size());
  CostItem none{};
  none.type = CT_COUNT; none.seg = -1;
  std::vector<CostItem> out(rounds * kCostLanes, none);
  for (int w = 0; w < W; ++w)
    for (size_t r = 0; r < per[w].size(); ++r)
      for (size_t l = 0; l < per[w][r]->n; ++l) out[r * kCostLanes + (size_t)w * 64 + l] = items[per[w][r]->i0 + l];
  while (!out.empty() && out.back().type == CT_COUNT) out.pop_back();
  return out;
}

int build_costs(const towr_problem_desc_t& d, const std::vector<double>& base_d, Layout& L, std::string& err) {
  const int E = d.robot.n_ee;
  if (d.n_costs < 0 || d.n_costs > TOWR_MAX_COSTS) { err = "n_costs out of range"; return TOWR_ERR_INVALID; }
  // GetSampleTimes (energy_cost.cc:41-55 and its copies): 0, dt, ... while t <= T + 1e-9, accumulated,
  // T = base_linear_->GetTotalTime() (the sum of the base polynomial durations)
  double Tb = 0.0;
  for (double v : base_d) Tb += v;
  auto sample_times = [&](double dt) {
    std::vector<double> ts;
    if (dt <= 0.0) { ts.push_back(0.0); ts.push_back(Tb); }
    else for (double t = 0.0; t <= Tb + 1e-9; t += dt) ts.push_back(t);
    return ts;
  };
  std::map<double, int> rows;   // one segment row per distinct sample time
  auto seg_of = [&](double t) {
    auto f = rows.find(t);
    if (f != rows.end()) return f->second;
    const int r = push_seg_row(L, t);
    rows[t] = r;
    return r;
  };
  std::vector<CostItem> items;
  for (int i = 0; i < d.n_costs; ++i) {
    const towr_cost_t& c = d.costs[i];
    CostItem it{};
    it.type = -1; it.seg = -1; it.w = c.weight;
    it.wdt = c.weight * (c.dt > 0.0 ? c.dt : 1.0);
    switch (c.kind) {
      case TOWR_COST_NODE: {   // node_cost.cc:36-79
        const int vk = c.ip[0];
        const bool base = vk == TOWR_VAR_BASE_LIN || vk == TOWR_VAR_BASE_ANG;
        if (vk < TOWR_VAR_BASE_LIN || vk > TOWR_VAR_EE_TORQUE || c.ip[1] < 0 || c.ip[1] > 1 || c.ip[2] < 0 || c.ip[2] > 2 ||
            (!base && (c.ee < 0 || c.ee >= E))) { err = "bad NodeCost term"; return TOWR_ERR_INVALID; }
        it.type = CT_NODE; it.ee = base ? 0 : c.ee;
        it.s = vk == TOWR_VAR_BASE_LIN ? 0 : vk == TOWR_VAR_BASE_ANG ? 1 : 2 + 4 * c.ee + (vk - TOWR_VAR_EE_MOTION);
        it.deriv = c.ip[1]; it.dim = c.ip[2];
        {   // the term's nodes in chunks of kNodeChunk: lanes share a long spline's node loop
          const int nn = L.spl[it.s].n_polys + 1;
          for (int a = 0; a < nn; a += kNodeChunk) { it.a0 = a; it.a1 = std::min(nn, a + kNodeChunk); items.push_back(it); }
        }
        break;
      }
      case TOWR_COST_ENERGY:   // energy_cost.cc:57-152
        if (c.weight <= 0.0) break;
        it.type = CT_ENERGY; it.tw = c.p[0];
        if (L.gait) {   // x-dependent polynomial durations: one item per (sample, ee)
          for (double t : sample_times(c.dt))
            for (int ee = 0; ee < E; ++ee) { it.t = t; it.seg = seg_of(t); it.ee = ee; items.push_back(it); }
        } else {        // fixed durations: one item per (spline, polynomial) with its Gram matrix
          // (cost_energy_q): Q(s, poly) = sum over the samples t on the polynomial of
          // w dt H(t) H(t)^T, times tw for the torque splines, in sample order
          const int nspl = (int)L.spl.size();
          std::map<std::pair<int, int>, std::array<double, 16>> gram;
          std::vector<std::pair<int, int>> order;
          for (double t : sample_times(c.dt)) {
            const int r = seg_of(t);
            for (int ee = 0; ee < E; ++ee)
              for (int k = 0; k < (it.tw != 0.0 ? 2 : 1); ++k) {
                const int sp = k == 0 ? sp_force(ee) : sp_torque(ee);
                const SegRec& sr = L.segs[(size_t)r * nspl + sp];
                const double wk = k == 0 ? it.wdt : it.wdt * it.tw;
                auto key = std::make_pair(sp, sr.poly);
                auto f = gram.find(key);
                if (f == gram.end()) { f = gram.emplace(key, std::array<double, 16>{}).first; order.push_back(key); }
                for (int a = 0; a < 4; ++a)
                  for (int b = 0; b < 4; ++b) f->second[4 * a + b] += wk * sr.H[kPos][a] * sr.H[kPos][b];
              }
          }
          for (const auto& key : order) {
            CostItem q = it;
            q.type = CT_ENERGYQ; q.seg = -1; q.s = key.first; q.deriv = key.second; q.ee = -1;
            q.a0 = (int32_t)(L.cost_q.size() / 16);
            const auto& Q = gram[key];
            L.cost_q.insert(L.cost_q.end(), Q.begin(), Q.end());
            items.push_back(q);
          }
        }
        break;
      case TOWR_COST_ANG_MOMENTUM:   // angular_momentum_cost.cc:67-208
        if (c.weight <= 0.0) break;
        it.type = CT_ANGMOM;
        for (double t : sample_times(c.dt)) { it.t = t; it.seg = seg_of(t); items.push_back(it); }
        break;
      case TOWR_COST_EE_BASE_POS: {   // ee_base_pos_cost.cc:57-162: swing samples only
        if (c.ee < 0 || c.ee >= E) { err = "bad EEBasePosCost endeffector"; return TOWR_ERR_INVALID; }
        if (c.weight <= 0.0) break;
        it.type = CT_EEBP; it.ee = c.ee; it.a0 = d.contact_at_start[c.ee] != 0;
        for (int k = 0; k < 3; ++k) it.p[k] = c.p[k];
        for (double t : sample_times(c.dt)) {
          if (!L.gait) {   // fixed phase durations: IsContactPhase once, here
            double tl;
            const int ph = seg_lookup(d.phase_durations[c.ee], d.n_phases[c.ee], t, &tl);
            if ((ph % 2 == 0) == (it.a0 != 0)) continue;
          }
          it.t = t; it.seg = seg_of(t); items.push_back(it);
        }
        break;
      }
      case TOWR_COST_BASE_HEIGHT: {   // base_height_cost.cc:55-142: one item per sample time
        if (!(c.dt > 0.0)) { err = "BaseHeightCost needs dt > 0"; return TOWR_ERR_INVALID; }
        it.type = CT_BHC; it.wdt = c.dt; it.p[0] = c.p[0]; it.a0 = 0;
        for (int ee = 0; ee < E; ++ee) if (d.contact_at_start[ee]) it.a0 |= 1 << ee;
        for (double t : sample_times(c.dt)) {
          it.a1 = -1;
          if (!L.gait) {   // fixed phase durations: PhaseDurations::IsContactPhase once, here
            it.a1 = 0;
            for (int ee = 0; ee < E; ++ee) {
              double tl;
              const int ph = seg_lookup(d.phase_durations[ee], d.n_phases[ee], t, &tl);
              if ((ph % 2 == 0) == (d.contact_at_start[ee] != 0)) it.a1 |= 1 << ee;
            }
          }
          it.t = t; it.seg = seg_of(t); items.push_back(it);
        }
        break;
      }
      case TOWR_COST_SOFT:   // soft_constraint.cc:34-69: evaluated by the handle's soft child
        if (c.ip[0] < 0 || c.ip[0] >= d.n_constraints) { err = "SoftConstraint: constraint index out of range"; return TOWR_ERR_INVALID; }
        // the child's description holds one constraint per term (soft_desc)
        if ((int)L.soft.size() >= TOWR_MAX_CONSTRAINTS) { err = "more SoftConstraint terms than TOWR_MAX_CONSTRAINTS"; return TOWR_ERR_INVALID; }
        L.soft.push_back({i, c.ip[0]});
        break;
      default: err = "unknown cost kind"; return TOWR_ERR_INVALID;
    }
  }
  std::stable_sort(items.begin(), items.end(), [](const CostItem& a, const CostItem& b) { return a.type < b.type; });
  L.cost_items = cost_wave_schedule(items);
  return TOWR_OK;
}

}  // namespace

// The host evaluation context of the structure pass (reference operation order, std::pow) at x
Ctx host_ctx(const Layout& L, const double* x, const towr_terrain_t& ter) {
  Ctx cx{};
  cx.x = x; cx.nodecol = L.nodecol.data(); cx.spl = L.spl.data(); cx.dur = L.dur.data();
  cx.ter = &ter; cx.rb = L.rb; cx.fdisc_motion = L.fdisc_motion;
  cx.gait = L.gait; cx.pinfo = L.pinfo.data(); cx.pcols = L.pcols.data(); cx.sched = L.sched.data(); cx.pact = L.pact.data();
  cx.eelin = L.eelin.data(); cx.lin = L.lin.data(); cx.rotvec = L.rotvec;
  return cx;
}
// Deterministic gradient slots (Layout::cost_nslot): with fixed phase durations every cost item's gradient
// entries go to columns that do not depend on x, so the host enumerates them once. An entry is present when
// its column is a variable (a constant node value has none). The slots are ordered by column, and within a
// column by item and emission order: entry k of item i (its k-th present entry) goes to slot
// cost_cslot[CostItem::cslot + k], column j owns slots [cost_cptr[j], cost_cptr[j + 1]), and one lane sums
// them in that order. No atomics: the same bits on every call.
namespace {
struct CostSlotPass {
  std::vector<int32_t>* cols;
  double f = 0.0;
  void operator()(int, int col, double, bool pres) { if (pres && col >= 0) cols->push_back(col); }
};
}
void build_cost_slots(Layout& L) {
  L.cost_nslot = 0; L.cost_cptr.clear(); L.cost_cslot.clear();
  if (L.gait || L.cost_items.empty()) return;   // PhaseSpline windows move with x: fixed-point limbs instead
  Ctx cx = host_ctx(L, L.x0.data(), L.terrain);
  cx.cq = L.cost_q.data();
  std::vector<int32_t> cols;
  for (CostItem& it : L.cost_items) {
    cx.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
    const size_t c0 = cols.size();
    CostSlotPass em{&cols};
    eval_cost_item(cx, it, em);
    it.cslot = (int32_t)c0; it.cn = (int32_t)(cols.size() - c0);
  }
  if (cols.empty() || cols.size() > (size_t)kCostSlotMax) {   // too many for the LDS budget: limbs
    for (CostItem& it : L.cost_items) it.cslot = it.cn = 0;
    return;
  }
  std::vector<int32_t> cptr(L.n + 1, 0);
  for (int32_t c : cols) ++cptr[c + 1];
  for (int j = 0; j < L.n; ++j) cptr[j + 1] += cptr[j];
  L.cost_cptr.assign(cptr.begin(), cptr.end());   // (below 2^16: kCostSlotMax)
  L.cost_cslot.resize(cols.size());
  std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
  for (size_t k = 0; k < cols.size(); ++k) L.cost_cslot[k] = (uint16_t)fill[cols[k]]++;   // ascending per column
  L.cost_nslot = (int32_t)cols.size();
}

// presence bits (dim * rows + row) of a watched instant's motion blocks at cx.x: the scales eval_fdisc /
// eval_tqdisc emit with, exactly as the structure pass evaluates them
int watch_presence(const Layout& L, Ctx& cx, const WatchItem& w) {
  cx.seg = L.segs.data() + (size_t)w.seg * L.spl.size();
  SplinePt P, F, Tq;
  spline_eval(cx, sp_motion(w.ee), w.t, P);
  spline_eval(cx, sp_force(w.ee), w.t, F);
  const double mu = cx.ter->friction_coeff;
  int mask = 0;
  if (w.type == IT_FDISC) {
    double sc[2][5];
    fdisc_motion_scales(*cx.ter, mu, P.p, F.p, sc);
    for (int dim = 0; dim < 2; ++dim) for (int i = 0; i < 5; ++i) if (sc[dim][i] != 0.0) mask |= 1 << (dim * 5 + i);
  } else {
    spline_eval(cx, sp_torque(w.ee), w.t, Tq);
    double sc[2][4];
    tqdisc_motion_scales(*cx.ter, mu, w.kf, P.p, F.p, Tq.p, sc);
    for (int dim = 0; dim < 2; ++dim) for (int i = 0; i < 4; ++i) if (sc[dim][i] != 0.0) mask |= 1 << (dim * 4 + i);
  }
  return mask;
}

int64_t pattern_outside_host(const Layout& L, const double* x, const towr_terrain_t& terrain) {
  if (L.watch.empty()) return 0;
  Ctx cx = host_ctx(L, x, terrain);
  int64_t n = 0;
  for (const WatchItem& w : L.watch) {
    const int rows = w.type == IT_FDISC ? 5 : 4, lo = (1 << rows) - 1;
    const int added = watch_presence(L, cx, w) & ~w.mask;   // present at x, outside the frozen pattern
    n += (int64_t)__builtin_popcount(added & lo) * w.cnt[0] + (int64_t)__builtin_popcount((added >> rows) & lo) * w.cnt[1];
  }
  return n;
}

// FsBlocks of the streaming ForceConstraintDiscretized path (layout.h): per constraint, its instants
// in chunks of <= kFsInst, provided every row of the constraint holds the same column list, each column
// is a force-set PhaseSpline column or a schedule column of the constraint's endeffector, and each force
// polynomial's columns fit a kFsWin window of the row. Otherwise the tile path stays.
// Whether every polynomial's active window (Layout::pact) of PhaseSpline s holds PhaseCols of one structure (count,
// node ids, derivatives) from one PhaseCol index in all three dimensions: then its kGsAct window basis sums and its first
// active PhaseCol are the same in every dimension (gs_window), and a record keeps one set (the TQDISC record, layout.h).
bool spline_dims_coincide(const Layout& L, int s) {
  const SplineMeta& m = L.spl[s];
  for (int p = 0; p < m.n_polys; ++p) {
    const int32_t* w0 = L.pact.data() + m.pact_off + 2 * p;
    for (int k = 1; k < 3; ++k) {
      const int32_t* wk = L.pact.data() + m.pact_off + 2 * (k * m.n_polys + p);
      if (wk[0] != w0[0] || wk[1] != w0[1]) return false;   // one first PhaseCol index: the records keep one qa
      for (int q = 0; q < kGsAct && w0[0] + q <= w0[1]; ++q) {
        const PhaseCol& a = L.pcols[(size_t)m.pcol_off[0] + w0[0] + q];
        const PhaseCol& b = L.pcols[(size_t)m.pcol_off[k] + wk[0] + q];
        if (a.n != b.n) return false;
        for (int j = 0; j < a.n; ++j)
          if (a.id[j] != b.id[j] || a.deriv[j] != b.deriv[j]) return false;
      }
    }
  }
  return true;
}

int build_fstream(Layout& L, std::string& err) {
  L.fstream = false;
  L.fs_blocks.clear(); L.fs_t.clear(); L.fs_tmpl.clear(); L.fs_ws.clear(); L.fs_iee.clear(); L.fs_irow.clear(); L.fs_iblk.clear(); L.fs_tmpl_max = 0;
  if (!L.gait || L.fdisc_motion) return TOWR_OK;
  std::vector<FsBlock> blocks;
  std::vector<double> ts;
  std::vector<int32_t> tmpl, wsv, iee, irow;
  int lmax = 0;
  for (const ConsInfo& cs : L.cons) {
    if (cs.kind != TOWR_C_FORCE_DISCRETIZED) continue;
    const int ee = cs.ee, fs = sp_force(ee);
    const SchedInfo& si = L.sched[ee];
    const SplineMeta& m = L.spl[fs];
    if (si.col0 < 0 || m.ee != ee) return TOWR_OK;
    const int r0 = cs.row0, nrow = cs.rows, K = nrow / 5;
    const int64_t L0 = L.row_ptr[r0 + 1] - L.row_ptr[r0];
    for (int r = r0; r < r0 + nrow; ++r) {
      if (L.row_ptr[r + 1] - L.row_ptr[r] != L0) return TOWR_OK;
      if (!std::equal(L.col.begin() + L.row_ptr[r], L.col.begin() + L.row_ptr[r + 1], L.col.begin() + L.row_ptr[r0])) return TOWR_OK;
    }
    const int toff = (int)tmpl.size();
    int js0 = -1, nsch = 0;
    std::vector<int> pos_of_pcol(L.pcols.size(), -1);
    for (int64_t j = 0; j < L0; ++j) {
      const int32_t col = L.col[L.row_ptr[r0] + j];
      if (col >= si.col0 && col < si.col0 + si.n_phases - 1) {
        if (js0 < 0) js0 = (int)j;
        if (col - si.col0 != (int)j - js0) return TOWR_OK;   // schedule columns contiguous, in order
        tmpl.push_back((int32_t)(0x80000000u | (uint32_t)(col - si.col0)));
        ++nsch;
        continue;
      }
      int32_t code = -1;
      for (int e = 0; e < 3 && code < 0; ++e)
        for (int q = 0; q < m.pcol_n[e]; ++q)
          if (L.pcols[m.pcol_off[e] + q].col == col && m.pcol_off[e] + q < (1 << 24)) {
            code = (m.pcol_off[e] + q) | (e << 24);
            pos_of_pcol[m.pcol_off[e] + q] = (int)j;
            break;
          }
      if (code < 0) return TOWR_OK;   // a column the template cannot express
      tmpl.push_back(code);
    }
    if (nsch != si.n_phases - 1) return TOWR_OK;
    if (!spline_dims_coincide(L, fs)) return TOWR_OK;   // the record's one set of window sums (layout.h)
    // window start of each force polynomial: the columns it touches (pact ranges of its 3 dims)
    const int wsoff = (int)wsv.size() / 3;
    for (int p = 0; p < m.n_polys; ++p) {
      int lo = INT32_MAX, hi = -1;
      for (int e = 0; e < 3; ++e) {
        const int32_t* r = L.pact.data() + m.pact_off + 2 * (e * m.n_polys + p);
        for (int q = r[0]; q <= r[1]; ++q) {
          const int pos = pos_of_pcol[m.pcol_off[e] + q];
          if (pos < 0) return TOWR_OK;
          lo = std::min(lo, pos); hi = std::max(hi, pos);
        }
      }
      if (hi >= 0 && hi - lo >= kFsWin) return TOWR_OK;
      const int ws = hi >= 0 ? lo : 0;
      // per window position: its dimension (3: not a PhaseCol active on p, its value is 0) and its slot in the active
      // window of that dimension (the record keeps dimension 0's sums: the dimensions' windows coincide, checked above)
      int32_t wd = 0, wq = 0;
      for (int q = 0; q < kFsWin; ++q) {
        int dim = 3, slot = 0;
        const int32_t te = ws + q < L0 ? tmpl[toff + ws + q] : -1;
        if (te >= 0) {
          const int e = (te >> 24) & 3, li = (te & 0xFFFFFF) - m.pcol_off[e];
          const int32_t* r = L.pact.data() + m.pact_off + 2 * (e * m.n_polys + p);
          if (li >= r[0] && li <= r[1]) { dim = e; slot = li - r[0]; }
        }
        if (slot >= kGsAct) return TOWR_OK;
        wd |= dim << (2 * q);
        wq |= slot << (2 * q);
      }
      wsv.push_back(ws);
      wsv.push_back(wd);
      wsv.push_back(wq);
    }
    lmax = std::max(lmax, (int)L0);
    // the constraint's instants, in row order (one instant per 5 rows)
    std::vector<double> its(K, -1.0);
    for (const ItemDesc& it : L.items)
      if (it.type == IT_FDISC && it.row0 >= r0 && it.row0 < r0 + nrow) its[(it.row0 - r0) / 5] = it.t;
    for (double t : its) if (t < 0) { err = "internal: ForceConstraintDiscretized instant missing"; return TOWR_ERR_INVALID; }
    // instants per block (the stream kernel's LDS records); the composer finds an entry's row by a float
    // division of its position, exact while the block's range stays below kFloatDivMax (layout.h)
    if (5 * L0 >= kFloatDivMax) return TOWR_OK;
    const int cap = std::max(1, std::min(kFsInst, (int)((kFloatDivMax - 1) / (5 * L0))));
    const int nb = (K + cap - 1) / cap;
    for (int q = 0; q < nb; ++q) {
      const int a = (int)((int64_t)q * K / nb), b = (int)((int64_t)(q + 1) * K / nb);
      FsBlock fb{};
      fb.ee = ee; fb.n_inst = b - a; fb.t0 = (int32_t)ts.size() + a; fb.r0 = r0 + 5 * a;
      fb.v0 = (int32_t)L.row_ptr[r0 + 5 * a]; fb.nv = (int32_t)(L.row_ptr[r0 + 5 * b] - L.row_ptr[r0 + 5 * a]);
      fb.L = (int32_t)L0; fb.tmpl = toff; fb.js0 = js0 < 0 ? (int32_t)L0 : js0; fb.ns1 = nsch; fb.wsoff = wsoff;
      if (fb.nv >= kFloatDivMax) { err = "internal: FsBlock past the float-division bound"; return TOWR_ERR_INVALID; }
      blocks.push_back(fb);
    }
    ts.insert(ts.end(), its.begin(), its.end());
    for (int k = 0; k < K; ++k) { iee.push_back(ee); irow.push_back(r0 + 5 * k); }
  }
  if (blocks.empty()) return TOWR_OK;
  L.fstream = true;
  L.fs_blocks.swap(blocks); L.fs_t.swap(ts); L.fs_tmpl.swap(tmpl); L.fs_ws.swap(wsv); L.fs_tmpl_max = lmax;
  L.fs_iee.swap(iee); L.fs_irow.swap(irow);
  L.fs_iblk.assign(L.fs_t.size(), 0);
  for (size_t q = 0; q < L.fs_blocks.size(); ++q)
    for (int k = 0; k < L.fs_blocks[q].n_inst; ++k) L.fs_iblk[(size_t)L.fs_blocks[q].t0 + k] = (int32_t)q;
  return TOWR_OK;
}

// GsGeo / GsBlock tables of the streaming RangeOfMotion and Dynamic paths (layout.h). A class streams
// when every one of its constraints passes the checks below; otherwise it keeps the tile path.
namespace {
struct BaseDec { int8_t s = -1, deriv = 0, dim = 0; int32_t node = 0; };   // base node-set column
struct PhaseDec { int8_t kind = -1, ee = 0, dim = 0; int32_t q = 0; };     // PhaseSpline column (kind 0 motion, 1 force, 2 torque)

bool build_gstream_class(Layout& L, int cls, const std::vector<BaseDec>& bdec, const std::vector<PhaseDec>& pdec,
                         const std::vector<int>& sdec_ee, const std::vector<int>& sdec_j, std::string& why) {
  const int nspl = (int)L.spl.size();
  const int ctype = cls == GS_ROM ? TOWR_C_RANGE_OF_MOTION : cls == GS_TQ ? TOWR_C_TORQUE_DISCRETIZED : TOWR_C_DYNAMIC;
  const int itype = cls == GS_ROM ? IT_ROM : cls == GS_TQ ? IT_TQDISC : IT_DYN;
  const int R = cls == GS_ROM ? 3 : cls == GS_TQ ? 4 : 6;
  const bool per_ee = cls != GS_DYN;   // one endeffector's constraint (RangeOfMotion, TQDISC)
  // TQDISC on curved terrain adds its motion block only where a scale is non-zero (:57): data-dependent, tiles
  if (cls == GS_TQ && L.fdisc_motion) { why = "motion block on curved terrain"; return false; }
  if (cls == GS_TQ)   // one set of window sums per spline in the record
    for (const ConsInfo& cs : L.cons)
      if (cs.kind == TOWR_C_TORQUE_DISCRETIZED && cs.rows > 0 &&
          (!spline_dims_coincide(L, sp_torque(cs.ee)) || !spline_dims_coincide(L, sp_force(cs.ee)))) {
        why = "window structure differs by dimension";
        return false;
      }
  if (cls == GS_DYN)   // one set of force and torque window sums per endeffector
    for (int ee = 0; ee < L.rb.n_ee; ++ee)
      if (!spline_dims_coincide(L, sp_torque(ee)) || !spline_dims_coincide(L, sp_force(ee))) {
        why = "window structure differs by dimension";
        return false;
      }
  std::vector<GsGeo> geos;
  std::vector<GsBlock> blocks;
  std::vector<GsInst> insts;
  std::vector<int32_t> tmpl;
  std::vector<uint8_t> pcode;
  std::vector<GsSeg> segs;
  std::vector<uint8_t> tseg;
  std::vector<uint32_t> vmap;
  std::vector<int16_t> wsv;
  int gmax[3] = {0, 0, 0}, nmax = 0;
  int cap = cls == GS_ROM ? kGsInstRom : cls == GS_TQ ? kGsInstTq : kGsInstDyn;
  cap = std::max(1, std::min(cap, kGsChunkMax / gs_rec_fields(cls, L.rb.n_ee)));   // a block's record chunk fits the prefetch
  if (gs_rec_fields(cls, L.rb.n_ee) > kGsChunkMax) { why = "record larger than the composer's prefetch"; return false; }
  int tmax = 0, pmax = 0;
  for (const ConsInfo& cs : L.cons) {
    if (cs.kind != ctype || cs.rows == 0) continue;
    const int K = cs.rows / R;
    GsGeo g{};
    g.cls = cls; g.ee = per_ee ? cs.ee : -1; g.nrt = R; g.r0 = cs.row0;
    g.rec0 = (int32_t)insts.size();
    // the instants: time and segment row from the items of the set
    std::vector<GsInst> its((size_t)K, GsInst{-1.0, -1, 0, 0, 0, 0, 0, 0.0});
    for (const ItemDesc& it : L.items)
      if (it.type == itype && it.row0 >= cs.row0 && it.row0 < cs.row0 + cs.rows) {
        GsInst& q = its[(it.row0 - cs.row0) / R];
        q.t = it.t; q.seg = it.seg; q.ee = (int16_t)(per_ee ? cs.ee : 0); q.row0 = it.row0; q.p0 = it.p0;
      }
    for (const GsInst& q : its) if (q.seg < 0) { why = "instant without items"; return false; }
    const int toff = (int)tmpl.size();
    int Lsum = 0, Psum = 0;
    for (int r = 0; r < R; ++r) {
      const int64_t b0 = L.row_ptr[cs.row0 + r], len = L.row_ptr[cs.row0 + r + 1] - b0;
      int P = 0;
      while (P < len && bdec[L.col[b0 + P]].s >= 0) ++P;
      for (int k = 0; k < K; ++k) {   // same length and prefix length, same template columns
        const int64_t a = L.row_ptr[cs.row0 + R * k + r], n = L.row_ptr[cs.row0 + R * k + r + 1] - a;
        if (n != len) { why = "row lengths differ between instants"; return false; }
        for (int64_t j = 0; j < n; ++j)
          if ((bdec[L.col[a + j]].s >= 0) != (j < P)) { why = "base columns are not a prefix of constant length"; return false; }
        if (!std::equal(L.col.begin() + a + P, L.col.begin() + a + n, L.col.begin() + b0 + P)) { why = "template differs between instants"; return false; }
      }
      g.L[r] = (int32_t)len; g.P[r] = P; g.T[r] = (int32_t)tmpl.size(); g.poff[r] = Psum;
      for (int64_t j = P; j < len; ++j) {
        const int32_t col = L.col[b0 + j];
        if (sdec_ee[col] >= 0) {
          if (per_ee && sdec_ee[col] != cs.ee) { why = "schedule of another endeffector"; return false; }
          tmpl.push_back((int32_t)(0x80000000u | ((uint32_t)sdec_ee[col] << 16) | (uint32_t)sdec_j[col]));
          continue;
        }
        const PhaseDec& d = pdec[col];
        const bool ok = d.kind >= 0 && (cls == GS_DYN || (d.ee == cs.ee && (cls == GS_ROM ? d.kind == 0 : d.kind == 1 || d.kind == 2)));
        if (!ok) { why = "a column the template cannot express"; return false; }
        tmpl.push_back((int32_t)(((uint32_t)d.kind << 28) | ((uint32_t)d.ee << 25) | ((uint32_t)d.dim << 22) | (uint32_t)d.q));
      }
      Lsum += (int)len; Psum += P;
      tmax = std::max(tmax, (int)tmpl.size() - toff);
    }
    g.Li = Lsum; g.Psum = Psum; g.pc0 = (int32_t)pcode.size(); g.K = K;
    // instants per compose block: the composer finds an entry's instant by a float division of its position,
    // exact while the block's range stays below kFloatDivMax (layout.h)
    const int capg = std::max(1, std::min(cap, (kFloatDivMax - 1) / std::max(1, Lsum)));
    {   // segments (layout.h GsSeg), the position -> segment map, the value map, window starts
      g.seg0 = (int32_t)(L.gs_segs.size() + segs.size());
      g.ts0 = (int32_t)(L.gs_tseg.size() + tseg.size());
      g.vm0 = (int32_t)(L.gs_vmap.size() + vmap.size());
      const int s0 = (int)segs.size();
      int vbase = 0, S = 0;
      std::vector<uint8_t> ts((size_t)Lsum, 0);
      auto key = [&](int32_t t) { return t < 0 ? (int)(0x100 | ((t >> 16) & 7)) : (int)(((t >> 28) & 3) << 3 | ((t >> 25) & 7)); };
      for (int r = 0; r < R; ++r) {
        auto add = [&](GsSeg q) {   // q.p0 row-relative on entry
          q.r = (int8_t)r; q.vbase = (int16_t)vbase; vbase += q.W;
          for (int j = q.p0; j < q.p0 + q.len; ++j) ts[S + j] = (uint8_t)(segs.size() - s0);
          q.toff = q.type == 0 ? g.poff[r] - S : g.T[r] - g.P[r] - S;   // local template offset (rebased at commit)
          q.p0 = (int16_t)(S + q.p0);
          segs.push_back(q);
        };
        if (g.P[r] > 0) add(GsSeg{0, 0, 0, 0, 0, (int16_t)g.P[r], (int16_t)g.P[r], 0, -1, 0});
        for (int j = g.P[r]; j < g.L[r];) {
          auto tr_at = [&](int pos) { return tmpl[(size_t)(g.T[r] + pos - g.P[r])]; };   // code of position pos
          const int k0 = key(tr_at(j));
          int j2 = j;
          while (j2 < g.L[r] && key(tr_at(j2)) == k0) ++j2;
          GsSeg q{};
          q.p0 = (int16_t)j; q.len = (int16_t)(j2 - j); q.wsoff = -1;
          if (tr_at(j) < 0) {
            q.type = 2; q.ee = (int8_t)((tr_at(j) >> 16) & 7); q.W = q.len;
          } else {
            q.type = 1; q.kind = (int8_t)((tr_at(j) >> 28) & 3); q.ee = (int8_t)((tr_at(j) >> 25) & 7);
            const int sp = q.kind == 0 ? sp_motion(q.ee) : q.kind == 1 ? sp_force(q.ee) : sp_torque(q.ee);
            const SplineMeta& m = L.spl[sp];
            q.wsoff = (int32_t)(L.gs_ws.size() + wsv.size());
            int W = 0;
            for (int p = 0; p < m.n_polys; ++p) {   // the polynomial's active positions in the segment
              int first = -1, last = -1;
              for (int pos = j; pos < j2; ++pos) {
                const int e = (tr_at(pos) >> 22) & 3, qq = tr_at(pos) & 0x3FFFFF;
                const int32_t* w = L.pact.data() + m.pact_off + 2 * (e * m.n_polys + p);
                if (qq >= w[0] && qq <= w[1]) { if (first < 0) first = pos; last = pos; }
              }
              wsv.push_back((int16_t)(first >= 0 ? first - j : 0));
              if (first >= 0) W = std::max(W, last - first + 1);
            }
            q.W = (int16_t)W;
          }
          add(q);
          j = j2;
        }
        S += g.L[r];
      }
      g.ns = (int32_t)segs.size() - s0;
      g.vt = vbase;
      // value slots grouped by segment kind (prefix, schedule, then windows by spline kind): the composer's
      // value lanes run in wave-sized runs of one code path
      std::vector<int> order((size_t)g.ns);
      for (int q = 0; q < g.ns; ++q) order[q] = s0 + q;
      auto rank = [&](const GsSeg& q) { return q.type == 0 ? 0 : q.type == 2 ? 1 : 2 + q.kind; };
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return rank(segs[a]) < rank(segs[b]); });
      vbase = 0;
      for (int q : order) { segs[q].vbase = (int16_t)vbase; vbase += segs[q].W; }
      // encodings: GsSeg::p0 / len / W / vbase are int16 positions within an instant (Lsum), the composer's
      // value index kk vt + vbase and the window width share one int (16 bits each), segment ids are bytes
      if (g.ns > 255 || vbase > 4096 || Lsum > INT16_MAX || (int64_t)vbase * capg > 65535) { why = "segment tables exceed their encodings"; return false; }
      for (int sg : order)
        for (int q = 0; q < segs[sg].W; ++q) vmap.push_back((uint32_t)((sg - s0) << 16 | q));
      tseg.insert(tseg.end(), ts.begin(), ts.end());
      gmax[0] = std::max(gmax[0], Lsum); gmax[1] = std::max(gmax[1], g.ns); gmax[2] = std::max(gmax[2], vbase);
    }
    pmax = std::max(pmax, Psum);
    for (int k = 0; k < K; ++k) {   // prefix codes: blk << 4 | dim << 2 | basis of the instant's base polynomials
      const int pl = L.segs[(size_t)its[k].seg * nspl + SP_BASE_LIN].poly, pa = L.segs[(size_t)its[k].seg * nspl + SP_BASE_ANG].poly;
      for (int r = 0; r < R; ++r) {
        const int64_t a = L.row_ptr[cs.row0 + R * k + r];
        for (int j = 0; j < g.P[r]; ++j) {
          const BaseDec& d = bdec[L.col[a + j]];
          const int nb = d.node - (d.s == 0 ? pl : pa);
          if (nb < 0 || nb > 1) { why = "base column outside the active polynomial"; return false; }
          pcode.push_back((uint8_t)((d.s << 4) | (d.dim << 2) | (2 * nb + d.deriv)));
        }
      }
    }
    const int nb = (K + capg - 1) / capg;
    for (int q = 0; q < nb; ++q) {
      const int a = (int)((int64_t)q * K / nb), b = (int)((int64_t)(q + 1) * K / nb);
      GsBlock bl{};
      bl.geo = (int32_t)(L.gs_geo.size() + geos.size()); bl.k0 = a; bl.n_inst = b - a;
      nmax = std::max(nmax, b - a);
      bl.v0 = (int32_t)L.row_ptr[cs.row0 + R * a]; bl.nv = (int32_t)(L.row_ptr[cs.row0 + R * b] - L.row_ptr[cs.row0 + R * a]);
      if ((int64_t)bl.nv != (int64_t)(b - a) * Lsum) { why = "internal: block range"; return false; }
      if (bl.nv >= kFloatDivMax) { why = "internal: compose block past the float-division bound"; return false; }
      for (int k = a; k < b; ++k) { its[k].kk = (int16_t)(k - a); its[k].nb = (int16_t)(b - a); }
      blocks.push_back(bl);
    }
    insts.insert(insts.end(), its.begin(), its.end());
    geos.push_back(g);
  }
  if (geos.empty()) { why = "no constraint"; return false; }
  // commit: geometries, templates and prefix codes are appended to the shared tables
  const int32_t t0 = (int32_t)L.gs_tmpl.size(), p0 = (int32_t)L.gs_pcode.size();
  for (GsGeo& g : geos) {
    for (int r = 0; r < g.nrt; ++r) g.T[r] += t0;
    g.pc0 += p0;
    L.gs_geo.push_back(g);
  }
  L.gs_tmpl.insert(L.gs_tmpl.end(), tmpl.begin(), tmpl.end());
  L.gs_pcode.insert(L.gs_pcode.end(), pcode.begin(), pcode.end());
  for (GsSeg& q : segs) if (q.type != 0) q.toff += t0;
  L.gs_segs.insert(L.gs_segs.end(), segs.begin(), segs.end());
  L.gs_tseg.insert(L.gs_tseg.end(), tseg.begin(), tseg.end());
  L.gs_vmap.insert(L.gs_vmap.end(), vmap.begin(), vmap.end());
  L.gs_ws.insert(L.gs_ws.end(), wsv.begin(), wsv.end());
  for (int q = 0; q < 3; ++q) L.gs_geo_max[cls][q] = gmax[q];
  L.gs_blocks[cls].swap(blocks);
  L.gs_inst[cls].swap(insts);
  L.gs_tmpl_max[cls] = tmax;
  L.gs_nmax[cls] = nmax;
  L.gs_pcode_max[cls] = pmax;
  L.gstream[cls] = true;
  return true;
}
}  // namespace

int build_gstream(Layout& L, std::string& err) {
  for (int c = 0; c < GS_COUNT; ++c) { L.gstream[c] = false; L.gs_blocks[c].clear(); L.gs_inst[c].clear(); L.gs_tmpl_max[c] = L.gs_pcode_max[c] = 0; }
  L.gs_geo.clear(); L.gs_tmpl.clear(); L.gs_pcode.clear(); L.gs_segs.clear(); L.gs_tseg.clear(); L.gs_vmap.clear(); L.gs_ws.clear();
  if (!L.gait || std::getenv("TOWR_GPU_GAIT_TILES")) return TOWR_OK;   // the tile path (A/B and parity of both paths)
  const int E = L.rb.n_ee;
  std::vector<BaseDec> bdec((size_t)L.n);
  for (int s = 0; s < 2; ++s)
    for (int node = 0; node <= L.spl[s].n_polys; ++node)
      for (int deriv = 0; deriv < 2; ++deriv)
        for (int dim = 0; dim < 3; ++dim) {
          const int32_t col = L.nodecol[(size_t)(L.spl[s].node_off + node) * 6 + deriv * 3 + dim];
          if (col >= 0) bdec[col] = BaseDec{(int8_t)s, (int8_t)deriv, (int8_t)dim, node};
        }
  std::vector<PhaseDec> pdec((size_t)L.n);
  for (int ee = 0; ee < E; ++ee)
    for (int kind = 0; kind < 3; ++kind) {
      const int s = kind == 0 ? sp_motion(ee) : kind == 1 ? sp_force(ee) : sp_torque(ee);
      const SplineMeta& m = L.spl[s];
      if (m.ee != ee) return TOWR_OK;
      for (int e = 0; e < 3; ++e) {
        for (int q = 0; q < m.pcol_n[e]; ++q) pdec[L.pcols[m.pcol_off[e] + q].col] = PhaseDec{(int8_t)kind, (int8_t)ee, (int8_t)e, q};
        for (int p = 0; p < m.n_polys; ++p) {   // active window of at most kGsAct PhaseCols
          const int32_t* w = L.pact.data() + m.pact_off + 2 * (e * m.n_polys + p);
          if (w[1] - w[0] + 1 > kGsAct) return TOWR_OK;
        }
      }
    }
  std::vector<int> sdec_ee((size_t)L.n, -1), sdec_j((size_t)L.n, 0);
  for (int ee = 0; ee < E; ++ee) {
    const SchedInfo& si = L.sched[ee];
    if (si.col0 < 0) return TOWR_OK;
    for (int j = 0; j < si.n_phases - 1; ++j) { sdec_ee[si.col0 + j] = ee; sdec_j[si.col0 + j] = j; }
  }
  for (int cls = 0; cls < GS_COUNT; ++cls) {
    std::string why;
    if (!build_gstream_class(L, cls, bdec, pdec, sdec_ee, sdec_j, why) && why.rfind("internal", 0) == 0) {
      err = why;
      return TOWR_ERR_INVALID;
    }
  }
  // the composer blobs (layout.h gs_blob)
  L.gs_blob.clear();
  for (int c = 0; c < GS_COUNT; ++c) L.gs_geo_max[c][3] = 0;
  for (GsGeo& g : L.gs_geo) {
    int ntl = 0;
    for (int r = 0; r < g.nrt; ++r) ntl = std::max(ntl, g.T[r] + g.L[r] - g.P[r] - g.T[0]);
    int nws = 0;
    for (int q = 0; q < g.ns; ++q) {
      const GsSeg& sg = L.gs_segs[g.seg0 + q];
      if (sg.type == 1) nws = std::max(nws, sg.wsoff + L.spl[sg.kind == 0 ? sp_motion(sg.ee) : sg.kind == 1 ? sp_force(sg.ee) : sp_torque(sg.ee)].n_polys);
    }
    int ws0 = INT32_MAX;
    for (int q = 0; q < g.ns; ++q) if (L.gs_segs[g.seg0 + q].type == 1) ws0 = std::min(ws0, L.gs_segs[g.seg0 + q].wsoff);
    if (ws0 == INT32_MAX) { ws0 = 0; nws = 0; }
    auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t o_vmap = al(sizeof(GsSeg) * g.ns), o_tmpl = o_vmap + al(4 * (size_t)g.vt), o_tseg = o_tmpl + al(4 * (size_t)ntl),
                 o_pcode = o_tseg + al((size_t)g.Li), o_ws = o_pcode + al((size_t)g.K * g.Psum), end = o_ws + al(2 * (size_t)(nws - ws0));
    std::vector<uint8_t> b(end, 0);
    for (int q = 0; q < g.ns; ++q) {
      GsSeg sg = L.gs_segs[g.seg0 + q];
      if (sg.type != 0) sg.toff -= g.T[0];
      if (sg.type == 1) sg.wsoff -= ws0;
      std::memcpy(b.data() + sizeof(GsSeg) * q, &sg, sizeof(GsSeg));
    }
    std::memcpy(b.data() + o_vmap, L.gs_vmap.data() + g.vm0, 4 * (size_t)g.vt);
    std::memcpy(b.data() + o_tmpl, L.gs_tmpl.data() + g.T[0], 4 * (size_t)ntl);
    std::memcpy(b.data() + o_tseg, L.gs_tseg.data() + g.ts0, (size_t)g.Li);
    if (g.K * g.Psum > 0) std::memcpy(b.data() + o_pcode, L.gs_pcode.data() + g.pc0, (size_t)g.K * g.Psum);   // TQDISC: no prefix
    if (nws > ws0) std::memcpy(b.data() + o_ws, L.gs_ws.data() + ws0, 2 * (size_t)(nws - ws0));
    g.blob0 = (int32_t)L.gs_blob.size();
    g.blob_n16 = (int32_t)(end / 16);
    g.o_vmap = (int32_t)o_vmap; g.o_tmpl = (int32_t)o_tmpl; g.o_tseg = (int32_t)o_tseg; g.o_pcode = (int32_t)o_pcode; g.o_ws = (int32_t)o_ws;
    L.gs_blob.resize(L.gs_blob.size() + end / 16);
    std::memcpy(L.gs_blob.data() + g.blob0, b.data(), end);
    L.gs_geo_max[g.cls][3] = std::max(L.gs_geo_max[g.cls][3], (int32_t)end);
  }
  (void)err;
  return TOWR_OK;
}

const towr_data_t* find_data(int n_data, const towr_data_t* data, int kind, int index) {
  for (int i = 0; i < n_data; ++i)
    if (data[i].kind == kind && data[i].index == index) return &data[i];
  return nullptr;
}

towr_problem_desc_t soft_desc(const towr_problem_desc_t& d, const Layout& L) {
  towr_problem_desc_t s = d;
  s.n_constraints = (int32_t)L.soft.size();
  for (size_t k = 0; k < L.soft.size(); ++k) {
    s.constraints[k] = d.constraints[L.soft[k].second];
    s.constraints[k].role = TOWR_ROLE_HARD;
  }
  s.n_costs = 0;
  return s;
}

void build_misc_xspan(Layout& L);
int build_layout(const towr_problem_desc_t& d, Layout& L, std::string& err) { return build_layout_ex(d, 0, nullptr, L, err); }

int build_layout_ex(const towr_problem_desc_t& d, int n_data, const towr_data_t* data, Layout& L, std::string& err) {
  if (n_data < 0 || (n_data > 0 && !data)) { err = "bad side data"; return TOWR_ERR_INVALID; }
  if (d.abi_version != TOWR_GPU_ABI_VERSION) { err = "abi version mismatch"; return TOWR_ERR_INVALID; }
  if (d.angular_rep != 0 && d.angular_rep != 1) { err = "angular_rep must be 0 (EulerZYX) or 1 (RotationVector)"; return TOWR_ERR_INVALID; }
  const int E = d.robot.n_ee;
  if (E < 1 || E > TOWR_MAX_EE) { err = "robot.n_ee out of range"; return TOWR_ERR_INVALID; }
  if (!(d.total_time > 0) || !(d.duration_base_polynomial > 0)) { err = "bad total_time / duration_base_polynomial"; return TOWR_ERR_INVALID; }

  std::vector<double> base_d;
  std::vector<NodeSet> sets;
  if (int rc = make_sets(d, base_d, sets, err)) return rc;
  // ---- variable sets in AddVariableSet order
  {
    const int n = assign_columns(d, sets, L.varsets, L.sched, err);
    if (n < 0) return n;
    L.n = n;
    L.gait = d.optimize_timings != 0;
    L.rotvec = d.angular_rep == 1;   // nlp_formulation.cc:113-116
  }

  // ---- node -> column table, spline metadata, polynomial durations
  L.spl.clear(); L.nodecol.clear(); L.dur.clear();
  for (size_t si = 0; si < sets.size(); ++si) {
    NodeSet& s = sets[si];
    SplineMeta m{};
    m.node_off = (int32_t)(L.nodecol.size() / 6);
    m.n_polys = s.n_nodes - 1;
    m.dur_off = (int32_t)L.dur.size();
    std::vector<int32_t> nc((size_t)s.n_nodes * 6, -1);
    for (int idx = 0; idx < s.n_rows; ++idx)
      for (const Nvi& q : s.info(idx)) nc[(q.id * 2 + q.deriv) * 3 + q.dim] = s.col0 + idx;
    L.nodecol.insert(L.nodecol.end(), nc.begin(), nc.end());
    m.ee = -1;
    if (si < 2) L.dur.insert(L.dur.end(), base_d.begin(), base_d.end());
    else {
      const int ee = (int)(si - 2) / 4;
      for (const PolyInfo& p : s.pinfo) L.dur.push_back(d.phase_durations[ee][p.phase] / p.n_polys_in_phase);  // :75-86
      if (L.gait) {   // PhaseSpline (spline_holder.cc:50-66): polynomial phases + full-pattern columns
        m.ee = ee;
        m.pinfo_off = (int32_t)L.pinfo.size();
        for (const PolyInfo& p : s.pinfo)
          L.pinfo.push_back(PolyPhase{(int16_t)p.phase, (int16_t)p.poly_in_phase, (int16_t)p.n_polys_in_phase, (int16_t)si});
        for (int e = 0; e < 3; ++e) {
          m.pcol_off[e] = (int32_t)L.pcols.size();
          for (int idx = 0; idx < s.n_rows; ++idx) {
            const std::vector<Nvi> q = s.info(idx);
            if (q.empty() || q[0].dim != e) continue;
            PhaseCol pc{};
            pc.col = s.col0 + idx;
            pc.n = (int8_t)std::min<size_t>(2, q.size());
            for (int k = 0; k < pc.n; ++k) { pc.id[k] = (int16_t)q[k].id; pc.deriv[k] = (int8_t)q[k].deriv; }
            L.pcols.push_back(pc);
          }
          m.pcol_n[e] = (int32_t)L.pcols.size() - m.pcol_off[e];
        }
        // active window of each (dim, polynomial): the PhaseCol range whose columns the polynomial's
        // two nodes set (node ids grow with the column, so the range is contiguous); empty: qa > qb
        m.pact_off = (int32_t)L.pact.size();
        for (int e = 0; e < 3; ++e)
          for (int p = 0; p < m.n_polys; ++p) {
            int qa = m.pcol_n[e], qb = m.pcol_n[e] - 1;
            for (int q = 0; q < m.pcol_n[e]; ++q) {
              const PhaseCol& pc = L.pcols[m.pcol_off[e] + q];
              bool act = false;
              for (int k = 0; k < pc.n; ++k) act = act || pc.id[k] == p || pc.id[k] == p + 1;
              if (act) { qa = std::min(qa, q); qb = q; }
            }
            for (int q = qa; q <= qb; ++q) {   // contiguity (the kernels rely on it)
              const PhaseCol& pc = L.pcols[m.pcol_off[e] + q];
              bool act = false;
              for (int k = 0; k < pc.n; ++k) act = act || pc.id[k] == p || pc.id[k] == p + 1;
              if (!act) { err = "internal: PhaseSpline active columns not contiguous"; return TOWR_ERR_INVALID; }
            }
            L.pact.push_back(qa);
            L.pact.push_back(qb);
          }
      }
    }
    L.spl.push_back(m);
  }

  if (int rc = init_values(d, d.init, d.terrain, sets, err)) return rc;
  fill_x0(d, sets, L.sched, L.n, L.x0);
  L.desc = d;

  // ---- robot & terrain
  {
    const double* I = d.robot.inertia;
    const double Ib[9] = {I[0], -I[3], -I[4], -I[3], I[1], -I[5], -I[4], -I[5], I[2]};
    std::memcpy(L.rb.Ib, Ib, sizeof Ib);
    L.rb.m = d.robot.mass; L.rb.g = d.robot.gravity; L.rb.n_ee = E;
    L.terrain = d.terrain;
    L.fdisc_motion = ter_has_curvature(d.terrain.id) ? 1 : 0;
  }

  // ---- constraint sets and work items (AddConstraintSet order)
  L.cons.clear(); L.items.clear(); L.eelin.clear(); L.lin.clear(); L.soft.clear();
  std::vector<int> item_inst;   // instance id (items of one instance share rows)
  int row = 0, inst = 0;
  auto dts_of = [](double Tc, double dt) {   // time_discretization_constraint.cc:37-50
    std::vector<double> v; double t = 0.0; v.push_back(t);
    for (int i = 0; i < (int)std::floor(Tc / dt); ++i) { t += dt; v.push_back(t); }
    v.push_back(Tc);
    return v;
  };
  if (d.n_constraints < 0 || d.n_constraints > TOWR_MAX_CONSTRAINTS) { err = "n_constraints out of range"; return TOWR_ERR_INVALID; }
  for (int ci = 0; ci < d.n_constraints; ++ci) {
    const towr_constraint_t& c = d.constraints[ci];
    if (c.role != TOWR_ROLE_HARD && c.role != TOWR_ROLE_SOFT) { err = "bad constraint role"; return TOWR_ERR_INVALID; }
    if (c.role == TOWR_ROLE_SOFT) {   // not a row block of g: only its SoftConstraint term evaluates it
      L.cons.push_back(ConsInfo{-1, c.ee, row, 0});
      continue;
    }
    ConsInfo info{c.kind, c.ee, row, 0};
    auto add = [&](int type, int group, int ee, int k, int row0, double t, int a0, int a1, double p0) {
      ItemDesc it{}; it.type = type; it.group = group; it.ee = ee; it.k = k; it.row0 = row0; it.seg = -1;
      it.t = t; it.a0 = a0; it.a1 = a1; it.p0 = p0;
      const int S = split_rows(type, group, L.gait);   // one lane per row of a PhaseSpline item
      for (int r = 0; r < S; ++r) {
        int first = 0, count = 0;
        if (type == IT_DYN) {   // one row per part, the last part takes the trailing (linear) rows
          first = r < S - 1 ? r : S - 1;
          count = r < S - 1 ? 1 : item_rows(type) - S + 1;
        } else {
          split_part_rows(item_rows(type), S, r, first, count);
        }
        it.rsel = S > 1 ? 1 + first + 16 * count + 256 * r : 0;
        L.items.push_back(it); item_inst.push_back(inst);
      }
    };
    const bool timed = c.kind == TOWR_C_DYNAMIC || c.kind == TOWR_C_RANGE_OF_MOTION ||
                       c.kind == TOWR_C_FORCE_DISCRETIZED || c.kind == TOWR_C_BASE_MOTION ||
                       c.kind == TOWR_C_TORQUE_DISCRETIZED || c.kind == TOWR_C_TERRAIN_HARD || c.kind == TOWR_C_EE_LINEAR;
    if (timed && !(c.dt > 0 && c.T > 0)) { err = "time-discretised constraint needs T > 0 and dt > 0"; return TOWR_ERR_INVALID; }
    const bool ee_c = c.kind == TOWR_C_RANGE_OF_MOTION || c.kind == TOWR_C_FORCE || c.kind == TOWR_C_FORCE_DISCRETIZED ||
                      c.kind == TOWR_C_TERRAIN || c.kind == TOWR_C_SWING || c.kind == TOWR_C_TORQUE_DISCRETIZED ||
                      c.kind == TOWR_C_TORQUE || c.kind == TOWR_C_TERRAIN_HARD;
    if (ee_c && (c.ee < 0 || c.ee >= E)) { err = "constraint endeffector out of range"; return TOWR_ERR_INVALID; }
    switch (c.kind) {
      case TOWR_C_DYNAMIC: {
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst)
          for (int g = 0; g < 2 + E; ++g) {
            if (g == 1 && L.rotvec) {   // RotVec base-angular block: one item per rotation-vector component
              for (int ax = 0; ax < 3; ++ax) add(IT_DYN, g, 0, k, row + 6 * k, ts[k], 0, 1 + ax, 0.0);
            } else {
              add(IT_DYN, g, 0, k, row + 6 * k, ts[k], 0, 0, 0.0);
            }
          }
        info.rows = 6 * (int)ts.size();
        break;
      }
      case TOWR_C_RANGE_OF_MOTION: {
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst)
          for (int g = 0; g < 3; ++g) add(IT_ROM, g, c.ee, k, row + 3 * k, ts[k], 0, 0, 0.0);
        info.rows = 3 * (int)ts.size();
        break;
      }
      case TOWR_C_FORCE_DISCRETIZED: {
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst) add(IT_FDISC, 0, c.ee, k, row + 5 * k, ts[k], 0, 0, 0.0);
        info.rows = 5 * (int)ts.size();
        break;
      }
      case TOWR_C_BASE_MOTION: {
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst) add(IT_BMOT, 0, 0, k, row + 6 * k, ts[k], 0, 0, 0.0);
        info.rows = 6 * (int)ts.size();
        break;
      }
      case TOWR_C_FORCE: {         // force_constraint.cc:50-60
        const NodeSet& fv = sets[4 + 4 * c.ee];
        const NodeSet& mv = sets[2 + 4 * c.ee];
        int k = 0;
        for (int id = 0; id < fv.n_nodes; ++id)
          if (!fv.is_constant_node(id)) {
            const int mn = mv.node_at_start_of_phase(fv.phase_of(id));
            if (mn < 0) { err = "force node phase has no motion node"; return TOWR_ERR_INVALID; }
            add(IT_FNODE, 0, c.ee, k, row + 5 * k, 0.0, id, mn, 0.0); ++k; ++inst;
          }
        info.rows = 5 * k;
        break;
      }
      case TOWR_C_TERRAIN: {       // terrain_constraint.cc:48-59
        const NodeSet& mv = sets[2 + 4 * c.ee];
        for (int id = 1; id < mv.n_nodes; ++id, ++inst) add(IT_TERR, 0, c.ee, id - 1, row + id - 1, 0.0, id, 0, 0.0);
        info.rows = mv.n_nodes - 1;
        break;
      }
      case TOWR_C_BASE_HEIGHT: {   // base_height_constraint.cc:45-56
        const NodeSet& bv = sets[0];
        for (int id = 1; id < bv.n_nodes; ++id, ++inst) add(IT_BHGT, 0, 0, id - 1, row + id - 1, 0.0, id, 0, c.p[0]);
        info.rows = bv.n_nodes - 1;
        break;
      }
      case TOWR_C_SWING: {         // swing_constraint.cc:41-52
        const NodeSet& mv = sets[2 + 4 * c.ee];
        int k = 0;
        for (int id = 0; id < mv.n_nodes; ++id)
          if (!mv.is_constant_node(id)) {
            if (id == 0 || id == mv.n_nodes - 1) { err = "swing node at trajectory boundary (the reference indexes out of range)"; return TOWR_ERR_INVALID; }
            add(IT_SWING, 0, c.ee, k, row + 4 * k, 0.0, id, 0, c.p[0] > 0 ? c.p[0] : 0.3); ++k; ++inst;
          }
        info.rows = 4 * k;
        break;
      }
      case TOWR_C_SPLINE_ACC: {    // spline_acc_constraint.cc:34-46
        if (c.ee != 0 && c.ee != 1) { err = "SplineAcc: ee must be 0 (base-lin) or 1 (base-ang)"; return TOWR_ERR_INVALID; }
        const int nj = L.spl[c.ee].n_polys - 1;
        for (int j = 0; j < nj; ++j, ++inst) add(IT_SACC, 0, c.ee, j, row + 3 * j, 0.0, 0, 0, 0.0);
        info.rows = 3 * (nj > 0 ? nj : 0);
        break;
      }
      case TOWR_C_TORQUE_DISCRETIZED: {   // torque_constraint_discretized.cc:69-93
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst) add(IT_TQDISC, 0, c.ee, k, row + 4 * k, ts[k], 0, 0, c.p[4]);
        info.rows = 4 * (int)ts.size();
        break;
      }
      case TOWR_C_TORQUE: {        // torque_constraint.cc:56-66: non-constant torque nodes
        const NodeSet& tv = sets[5 + 4 * c.ee];
        const NodeSet& mv = sets[2 + 4 * c.ee];
        int k = 0;
        for (int id = 0; id < tv.n_nodes; ++id)
          if (!tv.is_constant_node(id)) {
            const int ph = tv.phase_of(id);
            const int mn = mv.node_at_start_of_phase(ph), tn = tv.node_at_start_of_phase(ph);
            if (mn < 0 || tn < 0) { err = "torque node phase has no start node"; return TOWR_ERR_INVALID; }
            add(IT_TQNODE, 0, c.ee, k, row + 3 * k, 0.0, id, mn, c.p[4]);
            L.items.back().a2 = tn;
            ++k; ++inst;
          }
        info.rows = 3 * k;
        break;
      }
      case TOWR_C_TERRAIN_HARD: {  // terrain_constraint_hard.cc:35-48
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst) add(IT_THARD, 0, c.ee, k, row + k, ts[k], 0, 0, 0.0);
        info.rows = (int)ts.size();
        break;
      }
      case TOWR_C_EE_LINEAR: {     // ee_linear_constraint.cc:5-17
        if (c.ip[2] < 1 || c.ip[2] > 6 || c.ip[0] < 0 || c.ip[0] > 1 || c.ip[1] < 0 || c.ip[1] > 1) { err = "bad EELinear definition"; return TOWR_ERR_INVALID; }
        EELinDef def{};
        def.target = c.ip[0]; def.deriv = c.ip[1];
        for (int q = 0; q < c.ip[2]; ++q) {   // one term per (ee, dim): coefficients of repeats are summed
          const int code = c.ip[3 + q];
          if (code < 0 || code >= 3 * E) { err = "bad EELinear term"; return TOWR_ERR_INVALID; }
          int w = 0;
          while (w < def.n && def.code[w] != code) ++w;
          if (w == def.n) { def.code[def.n] = code; def.coeff[def.n] = 0.0; ++def.n; }
          def.coeff[w] += c.p[q];
        }
        const int di = (int)L.eelin.size();
        L.eelin.push_back(def);
        auto ts = dts_of(c.T, c.dt);
        for (int k = 0; k < (int)ts.size(); ++k, ++inst) add(IT_EELIN, 0, 0, k, row + k, ts[k], di, 0, 0.0);
        info.rows = (int)ts.size();
        break;
      }
      case TOWR_C_LINEAR_EQ: {     // linear_constraint.cc:35-45: one item per row of M
        const int vi = c.ip[0], rows = c.ip[1];
        if (vi < 0 || vi >= (int)L.varsets.size() || rows < 0) { err = "LinearEquality: bad variable set or row count"; return TOWR_ERR_INVALID; }
        const VarSetInfo& vs = L.varsets[vi];
        const towr_data_t* md = find_data(n_data, data, TOWR_DATA_LINEAR_M, ci);
        if (!md || (rows > 0 && !md->data) || md->count != (int64_t)rows * vs.n) { err = "LinearEquality: matrix (side data TOWR_DATA_LINEAR_M) missing or not rows x n_set"; return TOWR_ERR_INVALID; }
        for (int i = 0; i < rows; ++i, ++inst) {
          const int a0 = (int)L.lin.size();
          for (int j = 0; j < vs.n; ++j) {
            const double v = md->data[(size_t)i * vs.n + j];
            if (v != 0.0) L.lin.push_back(LinNz{vs.col0 + j, 0, v});   // M.sparseView(): exact zeros pruned
          }
          add(IT_LINEQ, 0, 0, i, row + i, 0.0, a0, (int)L.lin.size() - a0, 0.0);
        }
        info.rows = rows;
        break;
      }
      case TOWR_C_TOTAL_DURATION:  // total_duration_constraint.cc:36-47
        if (c.ee < 0 || c.ee >= E || L.sched[c.ee].col0 < 0) { err = "TotalDurationConstraint needs the ee's schedule variables"; return TOWR_ERR_INVALID; }
        add(IT_TDUR, 0, c.ee, 0, row, 0.0, 0, 0, 0.0); ++inst;
        info.rows = 1;
        break;
      default: err = "unknown constraint kind"; return TOWR_ERR_INVALID;
    }
    row += info.rows;
    L.cons.push_back(info);
  }
  L.m = row;

  // ---- segment table: the reference's GetLocalTime scan for every (timed instance, spline)
  {
    L.segs.clear();
    int last_inst = -1, last_row = -1;
    for (size_t q = 0; q < L.items.size(); ++q) {
      ItemDesc& it = L.items[q];
      const bool timed = it.type == IT_DYN || it.type == IT_ROM || it.type == IT_FDISC || it.type == IT_BMOT ||
                         it.type == IT_TQDISC || it.type == IT_THARD || it.type == IT_EELIN;
      if (!timed) { it.seg = -1; continue; }
      if (item_inst[q] != last_inst) {
        last_inst = item_inst[q];
        last_row = push_seg_row(L, it.t);
      }
      it.seg = last_row;
    }
  }

  // ---- fixed gait, RotVec: the Dynamic instants of the base-angular coefficient pre-pass (tiles.hip
  // towr_rv_coef_kernel); the three component items of an instant (a1 = 1, 2, 3, consecutive) get its index in a0
  L.rv_inst.clear();
  if (L.rotvec && !L.gait)
    for (ItemDesc& it : L.items) {
      if (it.type != IT_DYN || it.group != 1 || it.a1 <= 0) continue;
      if (it.a1 == 1) {
        for (int bb = 0; bb < 4; ++bb)   // the pre-pass reads x in global memory: no constant node values
          for (int e = 0; e < 3; ++e)
            if (L.segs[(size_t)it.seg * L.spl.size() + SP_BASE_ANG].col[bb][e] >= L.n) { err = "internal: constant base-angular node value"; return TOWR_ERR_INVALID; }
        L.rv_inst.push_back(RvInst{it.t, it.seg, 0});
      }
      it.a0 = (int32_t)L.rv_inst.size() - 1;
    }
  if (!L.rv_inst.empty()) {   // the group-0 lane of each instant: the same index (its base terms, kRvAb)
    std::unordered_map<int32_t, int32_t> at;   // first row of the instant -> pre-pass instant
    for (const ItemDesc& it : L.items)
      if (it.type == IT_DYN && it.group == 1 && it.a1 > 0) at[it.row0] = it.a0;
    for (ItemDesc& it : L.items)
      if (it.type == IT_DYN && it.group == 0) {
        const auto f = at.find(it.row0);
        if (f == at.end()) { err = "internal: a RotVec Dynamic instant without pre-pass coefficients"; return TOWR_ERR_INVALID; }
        it.a0 = f->second;
      }
  }

  // ---- cost terms (their sample times append rows to the segment table)
  if (int rc = build_costs(d, base_d, L, err)) return rc;

  // ---- structure pass at x0: candidate (row, col) of every item
  std::vector<int32_t> crow, ccol; std::vector<uint8_t> cpres;
  std::vector<int32_t> item_cand_begin(L.items.size() + 1, 0);
  {
    Ctx cx{};
    cx.x = L.x0.data(); cx.nodecol = L.nodecol.data(); cx.spl = L.spl.data(); cx.dur = L.dur.data();
    cx.ter = &L.terrain; cx.rb = L.rb; cx.fdisc_motion = L.fdisc_motion;
    cx.gait = L.gait; cx.pinfo = L.pinfo.data(); cx.pcols = L.pcols.data(); cx.sched = L.sched.data(); cx.pact = L.pact.data();
    cx.eelin = L.eelin.data(); cx.lin = L.lin.data(); cx.rotvec = L.rotvec;
    for (size_t i = 0; i < L.items.size(); ++i) {
      item_cand_begin[i] = (int32_t)crow.size();
      RecordEmit em{&crow, &ccol, &cpres};
      em.g_rows_lo = L.items[i].row0; em.g_rows_hi = L.items[i].row0 + item_rows(L.items[i].type);
      if (L.items[i].rsel > 0) { em.flo = L.items[i].row0 + rsel_first(L.items[i].rsel); em.fcnt = rsel_count(L.items[i].rsel); }
      cx.seg = L.items[i].seg >= 0 ? L.segs.data() + (size_t)L.items[i].seg * L.spl.size() : nullptr;
      eval_item(cx, L.items[i], em);
      if (em.bad_g) { err = "internal: item wrote g outside its rows"; return TOWR_ERR_INVALID; }
    }
    item_cand_begin[L.items.size()] = (int32_t)crow.size();
  }

  build_cost_slots(L);

  // ---- pattern watch: x0 presence of the data-dependent motion blocks (curved terrain)
  L.watch.clear();
  if (L.fdisc_motion) {
    Ctx cx = host_ctx(L, L.x0.data(), L.terrain);
    for (const ItemDesc& it : L.items) {
      if ((it.type != IT_FDISC && it.type != IT_TQDISC) || (it.rsel > 0 && rsel_part(it.rsel) != 0)) continue;
      WatchItem w{};
      w.t = it.t; w.kf = it.p0; w.seg = it.seg; w.type = it.type; w.ee = it.ee;
      w.mask = watch_presence(L, cx, w);
      cx.seg = L.segs.data() + (size_t)it.seg * L.spl.size();
      SplinePt P;
      spline_eval(cx, sp_motion(it.ee), it.t, P);
      for (int dim = 0; dim < 2; ++dim) {   // distinct variables of the spline's Jacobian row dim
        const SplineMeta& m = L.spl[sp_motion(it.ee)];
        if (L.gait) { w.cnt[dim] = m.pcol_n[dim]; continue; }   // PhaseSpline: the full pattern
        int cols[4], n = 0;
        for (int bb = 0; bb < 4; ++bb) {
          const int32_t col = basis_col(cx, sp_motion(it.ee), P.poly, bb, dim);
          bool dup = col < 0;
          for (int q = 0; q < n && !dup; ++q) dup = cols[q] == col;
          if (!dup) cols[n++] = col;
        }
        w.cnt[dim] = n;
      }
      L.watch.push_back(w);
    }
  }

  // ---- CSR pattern (setFromTriplets: sorted columns, duplicates merged)
  std::vector<std::vector<int32_t>> rc((size_t)L.m);
  for (size_t q = 0; q < crow.size(); ++q)
    if (cpres[q]) {
      if (crow[q] < 0 || crow[q] >= L.m || ccol[q] < 0 || ccol[q] >= L.n) { err = "internal: candidate out of range"; return TOWR_ERR_INVALID; }
      rc[crow[q]].push_back(ccol[q]);
    }
  L.row_ptr.assign((size_t)L.m + 1, 0);
  L.col.clear();
  for (int r = 0; r < L.m; ++r) {
    auto& v = rc[r];
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    L.col.insert(L.col.end(), v.begin(), v.end());
    L.row_ptr[r + 1] = (int64_t)L.col.size();
  }
  L.nnz = (int64_t)L.col.size();
  if (L.nnz >= (int64_t)INT32_MAX) { err = "too many nonzeros"; return TOWR_ERR_UNSUPPORTED; }

  // ---- slot table: candidate -> CSR position (or -1)
  L.slots.resize(crow.size());
  for (size_t q = 0; q < crow.size(); ++q) {
    if (!cpres[q]) { L.slots[q] = -1; continue; }
    const int r = crow[q];
    const int32_t* b = L.col.data() + L.row_ptr[r];
    const int32_t* e = L.col.data() + L.row_ptr[r + 1];
    L.slots[q] = (int32_t)(L.row_ptr[r] + (std::lower_bound(b, e, ccol[q]) - b));
  }
  for (size_t i = 0; i < L.items.size(); ++i) {
    L.items[i].slot = item_cand_begin[i];
    L.items[i].ncand = item_cand_begin[i + 1] - item_cand_begin[i];
    if (L.items[i].type == IT_DYN && L.items[i].group == 0 && L.items[i].ncand != kDynG0Cand) {
      err = "internal: Dynamic group-0 candidate count (the kernel's phase-B slot preload assumes kDynG0Cand)";
      return TOWR_ERR_INVALID;
    }
    // every present candidate of an item has its own CSR position (see engine_math.h)
    std::vector<int32_t> seen;
    for (int32_t q = item_cand_begin[i]; q < item_cand_begin[i + 1]; ++q) {
      if (L.slots[q] < 0) continue;
      if (std::find(seen.begin(), seen.end(), L.slots[q]) != seen.end()) {
        err = "internal: duplicate candidate in item type " + std::to_string(L.items[i].type);
        return TOWR_ERR_INVALID;
      }
      seen.push_back(L.slots[q]);
    }
  }

  // ---- tiles: consecutive instances of one constraint set, bounded by the LDS caps, one block
  // per (problem, tile); items are laid out per lane so that each wave runs a single code path
  {
    struct Inst { int32_t first, count; };
    std::vector<std::vector<TileDesc>> per_type(IT_COUNT);
    std::vector<std::vector<ItemDesc>> per_type_items(IT_COUNT);
    size_t i = 0;
    while (i < L.items.size()) {
      // maximal run of items of one type (adjacent constraint sets of one kind, e.g. the
      // RangeOfMotion sets of all feet, share tiles: their rows are contiguous)
      const int type = L.items[i].type;
      std::vector<Inst> insts;
      size_t j = i;
      while (j < L.items.size() && L.items[j].type == type) {
        size_t k = j;
        while (k < L.items.size() && item_inst[k] == item_inst[j]) ++k;
        insts.push_back({(int32_t)j, (int32_t)(k - j)});
        j = k;
      }
      const TypeSpec sp = type_spec(type, E, L.gait, L.rotvec);
      const int n_inst = (int)insts.size();
      auto inst_rows = [&](int a, int b) {   // rows of instances [a, b)
        const int r0 = L.items[insts[a].first].row0;
        const ItemDesc& last = L.items[insts[b - 1].first];
        return std::make_pair(r0, last.row0 + item_rows(last.type));
      };
      int n_tiles = (n_inst + sp.max_inst - 1) / sp.max_inst;
      for (;; ++n_tiles) {
        bool ok = true;
        for (int t = 0; t < n_tiles && ok; ++t) {
          const int a = (int)((int64_t)t * n_inst / n_tiles), b = (int)((int64_t)(t + 1) * n_inst / n_tiles);
          if (b <= a) continue;
          auto rr = inst_rows(a, b);
          const int vcap = is_misc_kind(type) ? kMiscValueCap : L.gait ? kTileValueCapGait : kTileValueCap, rcap = is_misc_kind(type) ? kMiscRowCap : kTileRowCap;
          if (L.row_ptr[rr.second] - L.row_ptr[rr.first] > vcap || rr.second - rr.first > rcap) ok = false;
        }
        if (ok) break;
        if (n_tiles >= n_inst) { err = "internal: one instance exceeds the LDS tile"; return TOWR_ERR_UNSUPPORTED; }
      }
      for (int t = 0; t < n_tiles; ++t) {
        const int a = (int)((int64_t)t * n_inst / n_tiles), b = (int)((int64_t)(t + 1) * n_inst / n_tiles);
        if (b <= a) continue;
        auto rr = inst_rows(a, b);
        TileDesc td{};
        td.type = type;
        td.r0 = rr.first; td.r1 = rr.second;
        td.v0 = (int32_t)L.row_ptr[td.r0]; td.v1 = (int32_t)L.row_ptr[td.r1];
        std::vector<ItemDesc> lanes((size_t)sp.block);
        for (auto& it : lanes) { it = ItemDesc{}; it.type = IT_NONE; it.seg = -1; }
        for (int k = a; k < b; ++k)
          for (int q = 0; q < insts[k].count; ++q) {
            const ItemDesc& it = L.items[insts[k].first + q];
            int lane = type_lane(type, it.group, k - a, b - a, E, L.gait, it.rsel > 0 ? rsel_part(it.rsel) : 0);
            if (type == IT_DYN && it.group == 1 && it.a1 > 0) lane = 64 + (it.a1 - 1) * (b - a) + (k - a);   // per-axis items
            // fixed gait, per-axis base-angular items: one tile of up to (block - 64) / (3 + E) instants,
            // the endeffector groups after the three axis groups (one wave may hold the last axis and
            // the first endeffectors); two tiles with whole waves per group measured slower (0.078 vs
            // 0.063 ms: twice the x staging and block overhead)
            if (type == IT_DYN && !L.gait && it.group >= 2 && L.rotvec)
              lane = 64 + 3 * (b - a) + (it.group - 2) * (b - a) + (k - a);
            if (lane < 0 || lane >= sp.block || lanes[lane].type != IT_NONE) { err = "internal: lane assignment"; return TOWR_ERR_INVALID; }
            lanes[lane] = it;
            if (type == IT_DYN) lanes[lane].a2 = k - a;   // instant within the tile (LDS sum terms)
          }
        td.i0 = (int32_t)per_type_items[type].size();   // relative; rebased below
        per_type_items[type].insert(per_type_items[type].end(), lanes.begin(), lanes.end());
        td.i1 = td.i0 + sp.block;
        per_type[type].push_back(td);
      }
      i = j;
    }
    std::vector<ItemDesc> items;
    L.tiles.clear();
    for (int t = 0; t < IT_COUNT; ++t) {
      L.type_tile0[t] = (int32_t)L.tiles.size();
      const int base = (int)items.size();
      int maxv = 0, maxr = 0;
      for (TileDesc td : per_type[t]) {
        td.i0 += base; td.i1 += base;
        maxv = std::max(maxv, td.v1 - td.v0); maxr = std::max(maxr, td.r1 - td.r0);
        L.tiles.push_back(td);
      }
      items.insert(items.end(), per_type_items[t].begin(), per_type_items[t].end());
      L.type_block[t] = type_spec(t, E, L.gait, L.rotvec).block;
      // LDS: [tile values | 64 dummy slots (absent candidates, by wave lane) | g rows]
      L.type_lds_dummy_off[t] = (maxv + 1) & ~1;
      L.type_lds_rows_off[t] = L.type_lds_dummy_off[t] + 64;   // one per wave lane: waves never collide within an instruction
      L.type_lds[t] = L.type_lds_rows_off[t] + ((maxr + 1) & ~1);
      if (L.gait && !is_misc_kind(t)) {   // no LDS tile (TileEmit DIRECT): positions only encode absence
        L.type_lds_rows_off[t] = 0;
        L.type_lds[t] = 0;
      }
      if (t == IT_DYN) {   // + per-instant endeffector sum terms (dyn_g0_a)
        int kmax = 0;   // instants of the largest tile
        for (const TileDesc& td : per_type[t]) kmax = std::max(kmax, (td.r1 - td.r0) / 6);
        if (!L.gait) L.type_lds[t] = L.type_lds_rows_off[t];   // fixed gait: g rows straight to HBM (tiles.hip kGDirect)
        L.dyn_scr_off = L.type_lds[t];
        L.type_lds[t] += kmax * E * 6;
      }
    }
    L.type_tile0[IT_COUNT] = (int32_t)L.tiles.size();
    // the small kinds (one-wave tiles) share one launch: up to 4 tiles per block, one per wave.
    // Each kind has its own per-wave LDS layout [values | 64 dummy slots | g rows], sized for its
    // largest tile; a block's waves are packed back to back (misc_lds), so the block's LDS is the
    // sum of its tiles' kinds, not 4x the largest kind.
    {
      std::vector<int32_t> mt;
      int stride[IT_COUNT] = {}, rows_off[IT_COUNT] = {};
      for (int t = 0; t < IT_COUNT; ++t) {
        if (!is_misc_kind(t)) continue;
        if (type_spec(t, E, L.gait, L.rotvec).block != 64) { err = "internal: small kinds must use one-wave tiles"; return TOWR_ERR_INVALID; }
        int mv = 0, mr = 0;
        for (int ti = L.type_tile0[t]; ti < L.type_tile0[t + 1]; ++ti) {
          mt.push_back(ti);
          mv = std::max(mv, L.tiles[ti].v1 - L.tiles[ti].v0);
          mr = std::max(mr, L.tiles[ti].r1 - L.tiles[ti].r0);
        }
        L.type_lds_dummy_off[t] = (mv + 1) & ~1;
        rows_off[t] = L.type_lds_dummy_off[t] + 64;
        stride[t] = rows_off[t] + ((mr + 1) & ~1);
      }
      L.misc_tiles.clear();
      L.misc_lds.clear();
      L.misc_region = 0;
      for (size_t q = 0; q < mt.size(); q += kMiscWaves) {
        int32_t off = 0;
        for (int w = 0; w < kMiscWaves; ++w) {
          const int32_t ti = q + w < mt.size() ? mt[q + w] : -1;
          L.misc_tiles.push_back(ti);
          const int t = ti >= 0 ? L.tiles[ti].type : -1;
          L.misc_lds.push_back(off);
          L.misc_lds.push_back(ti >= 0 ? rows_off[t] : 0);
          if (ti >= 0) off += stride[t];
        }
        L.misc_region = std::max(L.misc_region, off);
      }
    }
    // slot table per tile: lane l's candidates 8g..8g+7 in group g at base + g * block + l, as
    // tile-relative uint16 positions; four spare groups per lane absorb the kernel's prefetch
    std::vector<SlotGroup> groups;
    L.idirect.assign(L.gait ? items.size() : 0, ItemDirect{});
    for (const TileDesc& td : L.tiles) {
      const int block = td.i1 - td.i0;
      std::vector<int32_t> bslot((size_t)block, -1);   // build-time slot offsets (L.slots) of the lanes
      int maxc = 0;
      for (int l = 0; l < block; ++l) maxc = std::max(maxc, items[td.i0 + l].type == IT_NONE ? 0 : items[td.i0 + l].ncand);
      const int ng = (maxc + 7) / 8 + kSlotSpare;   // + spare groups for the kernels' slot prefetch
      const size_t base = groups.size();
      SlotGroup none; for (uint32_t& w : none.w) w = 0xFFFFFFFFu;
      groups.resize(base + (size_t)ng * block, none);
      for (int l = 0; l < block; ++l) {
        ItemDesc& it = items[td.i0 + l];
        if (it.type != IT_NONE)
          for (int j = 0; j < it.ncand; ++j) {
            const int32_t g = L.slots[it.slot + j];
            // an absent candidate is stored into the lane's own dummy slot (no branch, no LDS conflict)
            const uint32_t rel = g < 0 ? (uint32_t)(L.type_lds_dummy_off[td.type] + (l & 63)) : (uint32_t)(g - td.v0);
            if (rel >= (uint32_t)kSlotAbsent || (g >= 0 && (g < td.v0 || g >= td.v1))) { err = "internal: slot outside its tile"; return TOWR_ERR_INVALID; }
            uint32_t& w = groups[base + (size_t)(j / 8) * block + l].w[(j % 8) / 2];
            const int sh = (j & 1) ? 16 : 0;
            w = (w & ~(0xFFFFu << sh)) | (rel << sh);
          }
        if (L.gait && !is_misc_kind(td.type) && it.type != IT_NONE) {
          // direct ranges: variable sets whose candidates of this lane are all present at position
          // (tile-relative) = col + a constant; the two with the most candidates
          struct Rng { int32_t c0, c1, off, cnt; bool ok; };
          std::vector<Rng> rs;
          for (int j = 0; j < it.ncand; ++j) {
            const int32_t col = ccol[it.slot + j], g = L.slots[it.slot + j];
            if (col < 0) continue;
            int vs = -1;
            for (size_t v = 0; v < L.varsets.size(); ++v)
              if (col >= L.varsets[v].col0 && col < L.varsets[v].col0 + L.varsets[v].n) { vs = (int)v; break; }
            if (vs < 0) continue;
            const int32_t c0 = L.varsets[vs].col0, c1 = c0 + L.varsets[vs].n;
            Rng* r = nullptr;
            for (Rng& q : rs) if (q.c0 == c0) r = &q;
            const int32_t off = g < 0 ? 0 : (g - td.v0) - col;
            if (!r) { rs.push_back({c0, c1, off, 0, g >= 0}); r = &rs.back(); }
            r->ok = r->ok && g >= 0 && off == r->off;
            ++r->cnt;
          }
          std::sort(rs.begin(), rs.end(), [](const Rng& a, const Rng& b) { return a.cnt > b.cnt; });
          ItemDirect& dd = L.idirect[td.i0 + l];
          int k = 0;
          for (const Rng& q : rs)
            if (q.ok && k < 2) { dd.c0[k] = q.c0; dd.c1[k] = q.c1; dd.off[k] = q.off; ++k; }
          if ((td.type == IT_FDISC || td.type == IT_TQDISC) && it.rsel > 0) {   // rows owned whole by this lane
            const int r_lo = it.row0 + rsel_first(it.rsel), r_hi = r_lo + rsel_count(it.rsel);
            dd.z0 = (int32_t)(L.row_ptr[r_lo] - td.v0);
            dd.z1 = (int32_t)(L.row_ptr[r_hi] - td.v0);
          }
        }
        bslot[l] = it.slot;
        it.slot = (int32_t)(base + l);
      }
      if (L.gait && (td.type == IT_FDISC || td.type == IT_TQDISC)) {   // the lanes' owned ranges tile [v0, v1)
        std::vector<std::pair<int32_t, int32_t>> zr;
        for (int l = 0; l < block; ++l)
          if (items[td.i0 + l].type != IT_NONE) zr.push_back({L.idirect[td.i0 + l].z0, L.idirect[td.i0 + l].z1});
        std::sort(zr.begin(), zr.end());
        int32_t at = 0;
        for (auto& z : zr) { if (z.first != at) { err = "internal: row-split lanes do not cover their tile"; return TOWR_ERR_INVALID; } at = z.second; }
        if (at != td.v1 - td.v0) { err = "internal: row-split lanes do not cover their tile"; return TOWR_ERR_INVALID; }
      }
    }
    if (groups.size() >= (size_t)INT32_MAX) { err = "slot table too large"; return TOWR_ERR_UNSUPPORTED; }
    L.slot_groups.swap(groups);
    L.items.swap(items);
    for (int t = 0; t < IT_COUNT; ++t) {
      int64_t nv = 0, nr = 0;
      std::vector<uint8_t> used((size_t)L.n, 0);
      for (int ti = L.type_tile0[t]; ti < L.type_tile0[t + 1]; ++ti) {
        const TileDesc& td = L.tiles[ti];
        nv += td.v1 - td.v0; nr += td.r1 - td.r0;
        for (int32_t k = td.v0; k < td.v1; ++k) used[L.col[k]] = 1;
      }
      int64_t nx = 0;
      for (uint8_t u : used) nx += u;
      L.type_bytes[t] = 8 * (nv + nr + nx);
    }
    if (int rc = build_fstream(L, err)) return rc;
    if (int rc = build_gstream(L, err)) return rc;
    {   // the merged small-kind launch: union of their x columns
      int64_t nv = 0, nr = 0, nx = 0;
      std::vector<uint8_t> used((size_t)L.n, 0);
      for (int32_t ti : L.misc_tiles) {
        if (ti < 0) continue;
        const TileDesc& td = L.tiles[ti];
        nv += td.v1 - td.v0; nr += td.r1 - td.r0;
        for (int32_t k = td.v0; k < td.v1; ++k) used[L.col[k]] = 1;
      }
      for (uint8_t u : used) nx += u;
      L.misc_bytes = 8 * (nv + nr + nx);
    }
    build_misc_xspan(L);
  }
  return TOWR_OK;
}

// The 16-byte spans of x the small-kind launch stages (fixed phase durations): the node columns of every
// spline its items read (eval_height / eval_swing: the foot's motion nodes; eval_bmot, base height: the base
// nodes; eval_sacc: spline it.ee; eval_fnode: the foot's force and motion nodes), merged into runs of 16-byte
// units. Empty (the whole x) when an item kind reads anything else, or under phase-duration optimisation.
void build_misc_xspan(Layout& L) {
  L.misc_xspan.clear();
  if (L.gait || L.misc_tiles.empty()) return;
  std::vector<uint8_t> need((size_t)(L.n + 1) / 2, 0);
  bool all = false;
  auto spline = [&](int s) {
    if (s < 0 || s >= (int)L.spl.size()) { all = true; return; }
    const SplineMeta& m = L.spl[(size_t)s];
    for (int64_t k = (int64_t)m.node_off * 6; k < (int64_t)(m.node_off + m.n_polys + 1) * 6; ++k) {
      if (k >= (int64_t)L.nodecol.size()) { all = true; return; }
      const int32_t c = L.nodecol[(size_t)k];
      if (c >= 0 && c < L.n) need[(size_t)c / 2] = 1;
    }
  };
  for (int32_t ti : L.misc_tiles) {
    if (ti < 0) continue;
    const TileDesc& td = L.tiles[(size_t)ti];
    for (int32_t i = td.i0; i < td.i1 && !all; ++i) {
      const ItemDesc& it = L.items[(size_t)i];
      switch (it.type) {
        case IT_NONE: break;
        case IT_TERR: case IT_SWING: spline(sp_motion(it.ee)); break;
        case IT_BHGT: spline(SP_BASE_LIN); break;
        case IT_BMOT: spline(SP_BASE_LIN); spline(SP_BASE_ANG); break;
        case IT_SACC: spline(it.ee); break;
        case IT_FNODE: spline(sp_force(it.ee)); spline(sp_motion(it.ee)); break;
        default: all = true; break;
      }
    }
    if (all) return;
  }
  for (size_t u = 0; u < need.size();) {
    if (!need[u]) { ++u; continue; }
    size_t v = u;
    while (v < need.size() && need[v]) ++v;
    L.misc_xspan.push_back((int32_t)u);
    L.misc_xspan.push_back((int32_t)(v - u));
    u = v;
  }
}

int split_rows(int type, int group, bool gait) {
  if (!gait) return 1;
  switch (type) {
    case IT_DYN: return group >= 2 ? kDynGaitRowParts : 1;   // the endeffector groups (force / torque / motion PhaseSplines)
    case IT_ROM: return group == 2 ? 3 : 1;   // the endeffector-motion group
    case IT_FDISC: return 5;
    case IT_TQDISC: return 4;
    default: return 1;
  }
}

TypeSpec type_spec(int type, int n_ee, bool gait, bool rotvec) {
  const int E = std::max(1, n_ee);
  const int blk = tile_block(type, gait);
  switch (type) {
    case IT_DYN:   // waves: g0 | g1 | ee, ee (gait: rows); per-axis base-angular items: 3 g1 lanes per instant
      if (rotvec)   // per-component base-angular items
        return {blk, std::max(1, gait ? std::min(64 / 3, 64 / E) : std::min(64, (blk - 64) / (3 + E)))};
      return {blk, std::max(1, std::min(64, gait ? 64 / E : 128 / E))};
    case IT_ROM: return {blk, gait ? 128 : 64};                                         // waves: g0 | g1 | g2 (gait: rows, 2 halves)
    case IT_FDISC: return {blk, gait ? 128 : blk};
    case IT_TQDISC: return {blk, gait ? 64 : blk};
    default: return {64, 64};
  }
}

int type_lane(int type, int group, int k, int n, int n_ee, bool gait, int sub) {
  if (gait) {   // one wave per row range (tile_block); ROM / FDISC: two halves of 64 instants
    const int half = k >> 6, kk = k & 63;
    if (type == IT_DYN && group >= 2) return 64 * (2 + sub) + (group - 2) * n + k;
    if (type == IT_ROM) return 64 * 5 * half + 64 * (group < 2 ? group : 2 + sub) + kk;
    if (type == IT_FDISC) return 64 * (5 * half + sub) + kk;
    if (type == IT_TQDISC) return 64 * sub + k;
  }
  if (type == IT_DYN) return group == 0 ? k : group == 1 ? 64 + k : 128 + (group - 2) * n + k;
  if (type == IT_ROM) return 64 * group + k;
  return k;
}

int initial_x_for(const towr_problem_desc_t& d, const towr_init_t& init, const towr_terrain_t& ter,
                  std::vector<double>& x0, std::string& err) {
  std::vector<double> base_d;
  std::vector<NodeSet> sets;
  if (int rc = make_sets(d, base_d, sets, err)) return rc;
  std::vector<VarSetInfo> vs;
  std::vector<SchedInfo> sched;
  const int n = assign_columns(d, sets, vs, sched, err);   // same column layout as build_layout
  if (n < 0) return n;
  if (int rc = init_values(d, init, ter, sets, err)) return rc;
  fill_x0(d, sets, sched, n, x0);
  return TOWR_OK;
}

}  // namespace tg
