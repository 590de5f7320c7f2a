// nlp_formulation.cc — see nlp_formulation.hpp. Reference file:line per function.
#include "nlp_formulation.hpp"

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace towr_gpu {

// ------------------------------------------------------------------------------ robot models
RobotModel::RobotModel(Robot r) {
  auto four = [](double x, double y, double z) {
    return std::vector<Vector3d>{{x, y, z}, {x, -y, z}, {-x, y, z}, {-x, -y, z}};
  };
  switch (r) {
    case Monoped:   // monoped_model.h:41-60
      kinematic_model = {{{0.0, 0.0, -0.58}}, {{0.30, 0.15, 0.30}}, {{-0.30, -0.15, -0.30}}};
      dynamic_model = {20, {1.2, 5.5, 6.0, 0.0, -0.2, -0.01}, 1};
      break;
    case Biped: {   // biped_model.h:42-69
      const double z = -0.65, y = 0.20;
      kinematic_model = {{{0.0, y, z}, {0.0, -y, z}}, {{0.25, 0.15, 0.40}, {0.25, 0.15, 0.40}},
                         {{-0.25, -0.15, -0.40}, {-0.25, -0.15, -0.40}}};
      dynamic_model = {20, {1.209, 5.583, 6.056, 0.005, -0.190, -0.012}, 2};
      break;
    }
    case Hyq:       // hyq_model.h:42-75
      kinematic_model = {four(0.31, 0.29, -0.58), std::vector<Vector3d>(4, {0.25, 0.20, 0.10}),
                         std::vector<Vector3d>(4, {-0.25, -0.20, -0.10})};
      dynamic_model = {83, {4.26, 8.97, 9.88, -0.0063, 0.193, 0.0126}, 4};
      break;
    case Anymal:    // anymal_model.h:42-76
      kinematic_model = {four(0.34, 0.19, -0.42), std::vector<Vector3d>(4, {0.15, 0.1, 0.10}),
                         std::vector<Vector3d>(4, {-0.15, -0.1, -0.10})};
      dynamic_model = {29.5, {0.946438, 1.94478, 2.01835, 0.000938112, -0.00595386, -0.00146328}, 4};
      break;
    default: throw std::invalid_argument("Robot model not implemented");
  }
}

// ------------------------------------------------------------------------------ terrain
HeightMap HeightMap::MakeTerrain(TerrainID id) {
  HeightMap h;
  h.id = id;
  switch (id) {   // member defaults of height_map_examples.h
    case FlatID: h.params = {0.0}; break;
    case BlockID: h.params = {0.7, 3.5, 0.5, 0.03}; break;
    case StairsID: h.params = {1.0, 0.4, 0.2, 0.4, 1.0}; break;
    case GapID: h.params = {1.0, 0.5, 1.5}; break;
    case SlopeID: h.params = {1.0, 1.0, 1.0, 0.7}; break;
    case ChimneyID: h.params = {1.0, 1.5, 0.5, 3.0}; break;
    case ChimneyLRID: h.params = {0.5, 1.0, 0.5, 2.0}; break;
    case StepsID: h.params = {0.5, 0.3, 0.15, 5.0}; break;   // hopper_example.cc:53-86
    default: throw std::invalid_argument("terrain not implemented");
  }
  return h;
}

HeightMap HeightMap::Flat(double height) {
  HeightMap h;
  h.id = FlatID;
  h.params = {height};
  return h;
}

double HeightMap::GetHeight(double x, double y) const {   // height_map_examples.cc:35-211
  const auto& p = params;
  switch (id) {
    case FlatID: return p[0];
    case BlockID: {
      double h = 0.0;
      if (p[0] <= x && x <= p[0] + p[3]) h = p[2] / p[3] * (x - p[0]);
      if (p[0] + p[3] <= x && x <= p[0] + p[1]) h = p[2];
      return h;
    }
    case StairsID: {
      double h = 0.0;
      if (x >= p[0]) h = p[2];
      if (x >= p[0] + p[1]) h = p[3];
      if (x >= p[0] + p[1] + p[4]) h = 0.0;
      return h;
    }
    case GapID: {
      const double gs = p[0], w = p[1], hh = p[2], xc = gs + w / 2.0;
      const double a = (4 * hh) / (w * w), b = -(8 * hh * xc) / (w * w), c = -(hh * (w - 2 * xc) * (w + 2 * xc)) / (w * w);
      return (gs <= x && x <= gs + w) ? a * x * x + b * x + c : 0.0;
    }
    case SlopeID: {
      const double ss = p[0], xd = ss + p[1], xf = xd + p[2], sl = p[3] / p[1];
      double z = 0.0;
      if (x >= ss) z = sl * (x - ss);
      if (x >= xd) z = p[3] - sl * (x - xd);
      if (x >= xf) z = 0.0;
      return z;
    }
    case ChimneyID: return (p[0] <= x && x <= p[0] + p[1]) ? p[3] * (y - p[2]) : 0.0;
    case ChimneyLRID: {
      double z = 0.0;
      if (p[0] <= x && x <= p[0] + p[1]) z = p[3] * (y - p[2]);
      if (p[0] + p[1] <= x && x <= p[0] + 2 * p[1]) z = -p[3] * (y + p[2]);
      return z;
    }
    case StepsID: {
      if (x < p[0]) return 0.0;
      const int step = (int)((x - p[0]) / p[1]);
      return step >= (int)p[3] ? p[3] * p[2] : (step + 1) * p[2];
    }
  }
  throw std::invalid_argument("unknown terrain");
}

towr_terrain_t HeightMap::ToC() const {
  towr_terrain_t t;
  std::memset(&t, 0, sizeof(t));
  t.id = id;
  t.friction_coeff = friction_coeff;
  for (int i = 0; i < 8; ++i) t.p[i] = params[i];
  return t;
}

// ------------------------------------------------------------------------------ gaits
GaitGenerator GaitGenerator::MakeGaitGenerator(int leg_count) {
  if (leg_count != 1 && leg_count != 2 && leg_count != 4) throw std::invalid_argument("gait generator not implemented");
  GaitGenerator g(leg_count);
  g.SetGaits({"Stand"});
  return g;
}

void GaitGenerator::SetCombo(Combos c) {
  static const std::vector<std::string> mono[5] = {
      {"Stand", "Hop1", "Hop1", "Hop1", "Hop1", "Stand"}, {"Stand", "Hop1", "Hop1", "Hop1", "Stand"},
      {"Stand", "Hop1", "Hop1", "Hop1", "Hop1", "Stand"}, {"Stand", "Hop2", "Hop2", "Hop2", "Stand"},
      {"Stand", "Hop2", "Hop2", "Hop2", "Hop2", "Hop2", "Stand"}};                 // monoped_gait_generator.cc
  static const std::vector<std::string> bi[5] = {
      {"Stand", "Walk1", "Walk1", "Walk1", "Walk1", "Stand"}, {"Stand", "Run1", "Run1", "Run1", "Run1", "Stand"},
      {"Stand", "Hop1", "Hop1", "Hop1", "Stand"}, {"Stand", "Hop1", "Hop2", "Hop2", "Stand"},
      {"Stand", "Hop5", "Hop5", "Hop5", "Stand"}};                                 // biped_gait_generator.cc
  static const std::vector<std::string> quad[5] = {
      {"Stand", "Walk2", "Walk2", "Walk2", "Walk2E", "Stand"}, {"Stand", "Run2", "Run2", "Run2", "Run2E", "Stand"},
      {"Stand", "Run3", "Run3", "Run3", "Run3E", "Stand"}, {"Stand", "Hop1", "Hop1", "Hop1", "Hop1E", "Stand"},
      {"Stand", "Hop3", "Hop3", "Hop3", "Hop3E", "Stand"}};                        // quadruped_gait_generator.cc
  SetGaits(legs_ == 1 ? mono[c] : legs_ == 2 ? bi[c] : quad[c]);
}

void GaitGenerator::SetGaits(const std::vector<std::string>& gaits) {
  times_.clear();
  contacts_.clear();
  for (const auto& name : gaits) {
    Gait g = GetGait(name);
    times_.insert(times_.end(), g.first.begin(), g.first.end());
    contacts_.insert(contacts_.end(), g.second.begin(), g.second.end());
  }
}

namespace {
GaitGenerator::Gait RemoveTransition(GaitGenerator::Gait g) {   // gait_generator.cc:130-144
  const double last = g.first.back();
  g.first.pop_back();
  g.first.back() += last;
  g.second.pop_back();
  return g;
}
}  // namespace

GaitGenerator::Gait GaitGenerator::GetGait(const std::string& n) const {
  using C = Contacts;
  if (legs_ == 1) {
    const C o{true}, x{false};
    if (n == "Stand") return {{0.5}, {o}};
    if (n == "Flight") return {{0.5}, {x}};
    if (n == "Hop1") return {{0.3, 0.3}, {o, x}};
    if (n == "Hop2") return {{0.2, 0.3}, {o, x}};
  } else if (legs_ == 2) {
    const C I{false, false}, b{false, true}, P{true, false}, B{true, true};
    if (n == "Stand") return {{0.2}, {B}};
    if (n == "Flight") return {{0.5}, {I}};
    if (n == "Walk1" || n == "Walk2") return {{0.3, 0.05, 0.3, 0.05}, {b, B, P, B}};
    if (n == "Run1" || n == "Run3") return {{0.15, 0.4, 0.15 + 0.15, 0.4, 0.15}, {b, I, P, I, b}};
    if (n == "Hop1") return {{0.15, 0.5, 0.15}, {B, I, B}};
    if (n == "Hop2") return {{0.15, 0.4, 0.15}, {b, I, b}};
    if (n == "Hop3") return {{0.2, 0.2, 0.2}, {P, I, P}};
    if (n == "Hop5") return {{0.2, 0.3, 0.2, 0.2}, {P, I, b, B}};
  } else {
    auto f = [](std::initializer_list<int> on) { C c(4, false); for (int i : on) c[i] = true; return c; };
    const C II = f({}), PI = f({LH}), bI = f({RH}), IP = f({LF}), Ib = f({RF});
    const C Pb = f({LH, RF}), bP = f({RH, LF}), BI = f({LH, RH}), IB = f({LF, RF}), PP = f({LH, LF}), bb = f({RH, RF});
    const C Bb = f({LH, RH, RF}), BP = f({LH, RH, LF}), bB = f({RH, LF, RF}), PB = f({LH, LF, RF}), BB = f({0, 1, 2, 3});
    (void)PI; (void)bI; (void)Ib;
    if (n == "Stand") return {{0.3}, {BB}};
    if (n == "Flight") return {{0.3}, {Bb}};
    if (n == "Walk1") return {{0.3, 0.2, 0.3, 0.2, 0.3, 0.2, 0.3, 0.2}, {bB, BB, Bb, BB, PB, BB, BP, BB}};
    if (n == "Walk2" || n == "Walk2E") {
      Gait g{{0.25, 0.13, 0.25, 0.13, 0.25, 0.13, 0.25, 0.13}, {bB, bb, Bb, Pb, PB, PP, BP, bP}};
      return n == "Walk2E" ? RemoveTransition(g) : g;
    }
    if (n == "Run1") return {{0.3, 0.2, 0.3, 0.2}, {bP, BB, Pb, BB}};
    if (n == "Run2") return {{0.4, 0.1, 0.4, 0.1}, {bP, II, Pb, II}};
    if (n == "Run2E") return {{0.4}, {bP}};
    if (n == "Run3") return {{0.3, 0.1, 0.3, 0.1}, {PP, II, bb, II}};
    if (n == "Run3E") return {{0.3}, {PP}};
    if (n == "Hop1") return {{0.3, 0.1, 0.3, 0.1}, {BI, II, IB, II}};
    if (n == "Hop1E") return {{0.3}, {BI}};
    if (n == "Hop2") return {{0.3, 0.4, 0.3}, {BB, II, BB}};
    if (n == "Hop3" || n == "Hop3E") {
      Gait g{{0.2, 0.3, 0.2, 0.2, 0.2, 0.3, 0.2, 0.2}, {Bb, BI, BP, bP, bB, IB, PB, Pb}};
      return n == "Hop3E" ? RemoveTransition(g) : g;
    }
    if (n == "Hop5") return {{0.1, 0.2, 0.1, 0.1, 0.2, 0.1}, {Bb, BB, IP, Bb, BB, IP}};
  }
  throw std::invalid_argument("gait not defined: " + n);
}

std::vector<std::vector<double>> GaitGenerator::GetPhaseDurationsAll() const {
  const int n_ee = (int)contacts_.front().size();
  std::vector<double> acc(n_ee, 0.0);
  std::vector<std::vector<double>> out(n_ee);
  for (size_t ph = 0; ph + 1 < contacts_.size(); ++ph)
    for (int ee = 0; ee < n_ee; ++ee) {
      acc[ee] += times_[ph];
      if (contacts_[ph][ee] != contacts_[ph + 1][ee]) { out[ee].push_back(acc[ee]); acc[ee] = 0.0; }
    }
  for (int ee = 0; ee < n_ee; ++ee) out[ee].push_back(acc[ee] + times_.back());
  return out;
}

std::vector<double> GaitGenerator::GetPhaseDurations(double T, int ee) const {
  std::vector<double> v = GetPhaseDurationsAll().at(ee);
  double total = 0.0;
  for (double d : v) total += d;   // std::accumulate
  for (double& d : v) d = d / total * T;
  return v;
}

// ------------------------------------------------------------------------------ parameters
bool Parameters::IsOptimizeTimings() const {
  for (auto c : constraints_) if (c == TotalTime) return true;
  return false;
}

double Parameters::GetTotalTime() const {
  if (ee_phase_durations_.empty()) return 0.0;
  double T = 0.0;
  for (double d : ee_phase_durations_.front()) T += d;
  return T;
}

// ------------------------------------------------------------------------------ formulation
std::vector<VarSet> NlpFormulation::GetVariableSets() const {
  const int E = params_.GetEECount();
  std::vector<VarSet> vs{{TOWR_VAR_BASE_LIN, 0}, {TOWR_VAR_BASE_ANG, 0}};
  for (int k : {TOWR_VAR_EE_MOTION, TOWR_VAR_EE_ANG, TOWR_VAR_EE_FORCE, TOWR_VAR_EE_TORQUE})
    for (int ee = 0; ee < E; ++ee) vs.push_back({k, ee});
  if (params_.IsOptimizeTimings())
    for (int ee = 0; ee < E; ++ee) vs.push_back({TOWR_VAR_EE_SCHEDULE, ee});
  return vs;
}

std::vector<ConstraintSpec> NlpFormulation::GetConstraints() const {
  const Parameters& P = params_;
  const int E = P.GetEECount();
  const double T = P.GetTotalTime();
  std::vector<ConstraintSpec> out;
  for (auto name : P.constraints_) {
    switch (name) {
      case Parameters::Dynamic: out.push_back({TOWR_C_DYNAMIC, 0, T, P.dt_constraint_dynamic_}); break;
      case Parameters::EndeffectorRom:
        for (int ee = 0; ee < E; ++ee) out.push_back({TOWR_C_RANGE_OF_MOTION, ee, T, P.dt_constraint_range_of_motion_});
        break;
      case Parameters::BaseRom: {
        ConstraintSpec c{TOWR_C_BASE_MOTION, 0, T, P.dt_constraint_base_motion_};
        c.p = P.base_rom_;
        out.push_back(c);
        break;
      }
      case Parameters::TotalTime:
        for (int ee = 0; ee < E; ++ee) out.push_back({TOWR_C_TOTAL_DURATION, ee, T, 0.0});
        break;
      case Parameters::Terrain:
        for (int ee = 0; ee < E; ++ee) {   // nlp_formulation.cc:464-481
          const double mn = ee < (int)P.ee_swing_height_min_.size() ? P.ee_swing_height_min_[ee] : 0.02;
          const double mx = ee < (int)P.ee_swing_height_max_.size() ? P.ee_swing_height_max_[ee] : INFINITY;
          if (mn < 0.0) throw std::runtime_error("Swing height minimum must be >= 0.0");
          if (mx <= mn) throw std::runtime_error("Swing height maximum must be > minimum");
          ConstraintSpec c{TOWR_C_TERRAIN, ee, T, 0.0};
          c.p[0] = mn; c.p[1] = mx;
          out.push_back(c);
        }
        break;
      case Parameters::Force:
        for (int ee = 0; ee < E; ++ee) {
          ConstraintSpec c = P.dt_constraint_force_ > 0.0 ? ConstraintSpec{TOWR_C_FORCE_DISCRETIZED, ee, T, P.dt_constraint_force_}
                                                          : ConstraintSpec{TOWR_C_FORCE, ee, T, 0.0};
          c.p[0] = P.force_limit_in_normal_direction_;
          out.push_back(c);
        }
        break;
      case Parameters::Swing:
        for (int ee = 0; ee < E; ++ee) { ConstraintSpec c{TOWR_C_SWING, ee, T, 0.0}; c.p[0] = 0.3; out.push_back(c); }
        break;
      case Parameters::BaseAcc:
        out.push_back({TOWR_C_SPLINE_ACC, 0, T, 0.0});
        out.push_back({TOWR_C_SPLINE_ACC, 1, T, 0.0});
        break;
      case Parameters::BaseHeight: { ConstraintSpec c{TOWR_C_BASE_HEIGHT, 0, T, 0.0}; c.p[0] = 0.4; out.push_back(c); break; }   // nlp_formulation.cc:597
      case Parameters::TerrainHard:   // nlp_formulation.cc:492-506
        for (int ee = 0; ee < E; ++ee) out.push_back({TOWR_C_TERRAIN_HARD, ee, T, P.dt_constraint_range_of_motion_});
        break;
      case Parameters::Torque:        // nlp_formulation.cc:533-558
        for (int ee = 0; ee < E; ++ee) {
          ConstraintSpec c = P.dt_constraint_torque_ > 0.0 ? ConstraintSpec{TOWR_C_TORQUE_DISCRETIZED, ee, T, P.dt_constraint_torque_}
                                                           : ConstraintSpec{TOWR_C_TORQUE, ee, T, 0.0};
          c.p[0] = P.torque_tx_min_; c.p[1] = P.torque_tx_max_; c.p[2] = P.torque_ty_min_; c.p[3] = P.torque_ty_max_;
          c.p[4] = P.torque_k_friction_;
          out.push_back(c);
        }
        break;
      default: throw std::runtime_error("constraint not defined!");
    }
  }
  for (const auto& def : P.ee_linear_constraints_) {   // GetConstraints, nlp_formulation.cc:373-375
    if (def.terms.empty() || def.terms.size() > 6) throw std::invalid_argument("EELinear: 1..6 terms supported");
    ConstraintSpec c{TOWR_C_EE_LINEAR, 0, T, def.dt};
    c.ip[0] = def.target; c.ip[1] = def.deriv; c.ip[2] = (int32_t)def.terms.size();
    for (size_t q = 0; q < def.terms.size(); ++q) {
      c.p[q] = def.terms[q].coeff;
      c.ip[3 + q] = def.terms[q].ee * 3 + def.terms[q].dim;
    }
    out.push_back(c);
  }
  return out;
}

// NlpFormulation::GetCosts (nlp_formulation.cc:604-680): MakeForcesCost (:646-664) and
// MakeEEMotionCost (:666-678) expand into NodeCosts; the swing ee-base tracking terms (:613-626) follow
std::vector<CostSpec> NlpFormulation::GetCosts() const {
  const Parameters& P = params_;
  const int E = P.GetEECount();
  std::vector<CostSpec> out;
  auto node = [&](int ee, double w, int kind, int deriv, int dim) {
    CostSpec c{TOWR_COST_NODE, ee, w, 0.0};
    c.ip[0] = kind; c.ip[1] = deriv; c.ip[2] = dim;
    out.push_back(c);
  };
  for (const auto& [name, w] : P.costs_) {
    switch (name) {
      case Parameters::ForcesCostID:
        for (int ee = 0; ee < E; ++ee)
          for (int dim = 0; dim < 3; ++dim) {
            node(ee, w, TOWR_VAR_EE_FORCE, 0, dim);
            node(ee, w, TOWR_VAR_EE_TORQUE, 0, dim);
            node(ee, 0.1 * w, TOWR_VAR_EE_FORCE, 1, dim);
            node(ee, 0.1 * w, TOWR_VAR_EE_TORQUE, 1, dim);
          }
        break;
      case Parameters::EEMotionCostID:
        for (int ee = 0; ee < E; ++ee) {
          node(ee, w, TOWR_VAR_EE_MOTION, 1, 0);
          node(ee, w, TOWR_VAR_EE_MOTION, 1, 1);
          node(ee, 0.5 * w, TOWR_VAR_EE_MOTION, 1, 2);
        }
        break;
      case Parameters::EnergyCostID: {
        CostSpec c{TOWR_COST_ENERGY, 0, w, P.dt_cost_energy_};
        c.p[0] = P.energy_cost_torque_weight_;
        out.push_back(c);
        break;
      }
      case Parameters::AngMomCostID: out.push_back(CostSpec{TOWR_COST_ANG_MOMENTUM, 0, w, P.dt_cost_ang_mom_}); break;
      default: throw std::runtime_error("cost not defined!");
    }
  }
  if (P.enable_swing_ee_base_pos_tracking && P.swing_ee_base_pos_tracking_weight_ > 0.0) {
    // reference ee positions in the base frame at the initial state
    double R[3][3];
    {
      const auto& a = initial_base_.ang_p;
      const double sx = std::sin(a[0]), cx = std::cos(a[0]), sy = std::sin(a[1]), cy = std::cos(a[1]), sz = std::sin(a[2]), cz = std::cos(a[2]);
      const double m[3][3] = {{cy * cz, cz * sx * sy - cx * sz, sx * sz + cx * cz * sy},
                              {cy * sz, cx * cz + sx * sy * sz, cx * sy * sz - cz * sx},
                              {-sy, cy * sx, cx * cy}};
      std::memcpy(R, m, sizeof R);
    }
    for (int ee = 0; ee < E; ++ee) {
      double rW[3];
      for (int k = 0; k < 3; ++k) rW[k] = initial_ee_W_.at(ee)[k] - initial_base_.lin_p[k];
      CostSpec c{TOWR_COST_EE_BASE_POS, ee, P.swing_ee_base_pos_tracking_weight_, P.dt_cost_swing_ee_base_pos_tracking_};
      for (int i = 0; i < 3; ++i) c.p[i] = R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2];
      out.push_back(c);
    }
  }
  return out;
}

towr_problem_desc_t NlpFormulation::MakeDesc() const {
  return MakeDesc(GetVariableSets(), GetConstraints(), TOWR_INIT_FORMULATION, {}, params_.GetTotalTime());
}

towr_problem_desc_t NlpFormulation::MakeDesc(const std::vector<VarSet>& vs, const std::vector<ConstraintSpec>& cs,
                                             int init_mode, const std::vector<Vector3d>& ee_goal, double total_time) const {
  const Parameters& P = params_;
  const KinematicModel& km = model_.kinematic_model;
  const DynamicModel& dm = model_.dynamic_model;
  const int E = P.GetEECount();
  if (E != dm.ee_count) throw std::invalid_argument("params ee count does not match robot");
  if (E > TOWR_MAX_EE || (int)vs.size() > TOWR_MAX_VARSETS || (int)cs.size() > TOWR_MAX_CONSTRAINTS)
    throw std::invalid_argument("problem exceeds the engine's fixed limits");
  towr_problem_desc_t d;
  std::memset(&d, 0, sizeof(d));
  d.abi_version = TOWR_GPU_ABI_VERSION;
  d.angular_rep = P.angular_rep_ == Parameters::RotationVector ? 1 : 0;   // nlp_formulation.cc:113-116
  d.robot.mass = dm.m;
  d.robot.gravity = dm.g;
  for (int i = 0; i < 6; ++i) d.robot.inertia[i] = dm.inertia[i];
  d.robot.n_ee = E;
  for (int ee = 0; ee < E; ++ee)
    for (int k = 0; k < 3; ++k) {
      d.robot.nominal_stance[ee][k] = km.nominal_stance[ee][k];
      d.robot.max_dev[ee][k] = km.max_dev[ee][k];
      d.robot.min_dev[ee][k] = km.min_dev[ee][k];
    }
  d.terrain = terrain_.ToC();
  d.total_time = total_time;
  d.duration_base_polynomial = P.duration_base_polynomial_;
  d.ee_polynomials_per_swing_phase = P.ee_polynomials_per_swing_phase_;
  d.force_polynomials_per_stance_phase = P.force_polynomials_per_stance_phase_;
  d.torque_polynomials_per_stance_phase = P.torque_polynomials_per_stance_phase_;
  d.optimize_timings = P.IsOptimizeTimings() ? 1 : 0;
  d.bound_phase_duration[0] = P.bound_phase_duration_[0];
  d.bound_phase_duration[1] = P.bound_phase_duration_[1];
  for (int ee = 0; ee < E; ++ee) {
    const auto& ph = P.ee_phase_durations_.at(ee);
    if ((int)ph.size() > TOWR_MAX_PHASES) throw std::invalid_argument("too many phases");
    d.n_phases[ee] = (int)ph.size();
    d.contact_at_start[ee] = P.ee_in_contact_at_start_.at(ee) ? 1 : 0;
    for (size_t i = 0; i < ph.size(); ++i) d.phase_durations[ee][i] = ph[i];
  }
  d.n_varsets = (int)vs.size();
  for (size_t i = 0; i < vs.size(); ++i) { d.varsets[i].kind = vs[i].kind; d.varsets[i].ee = vs[i].ee; }
  d.n_constraints = (int)cs.size();
  for (size_t i = 0; i < cs.size(); ++i) {
    d.constraints[i].kind = cs[i].kind;
    d.constraints[i].ee = cs[i].ee;
    d.constraints[i].T = cs[i].T;
    d.constraints[i].dt = cs[i].dt;
    for (int j = 0; j < 6; ++j) d.constraints[i].p[j] = cs[i].p[j];
    for (int j = 0; j < 9; ++j) d.constraints[i].ip[j] = cs[i].ip[j];
  }
  const std::vector<CostSpec> costs = GetCosts();
  if ((int)costs.size() > TOWR_MAX_COSTS) throw std::invalid_argument("too many cost terms");
  d.n_costs = (int)costs.size();
  for (size_t i = 0; i < costs.size(); ++i) {
    towr_cost_t& c = d.costs[i];
    c.kind = costs[i].kind; c.ee = costs[i].ee; c.weight = costs[i].weight; c.dt = costs[i].dt;
    for (int j = 0; j < 4; ++j) { c.p[j] = costs[i].p[j]; c.ip[j] = costs[i].ip[j]; }
  }
  towr_init_t& it = d.init;
  it.mode = init_mode;
  for (int k = 0; k < 3; ++k) {
    it.base_lin_p0[k] = initial_base_.lin_p[k]; it.base_lin_v0[k] = initial_base_.lin_v[k];
    it.base_ang_p0[k] = initial_base_.ang_p[k]; it.base_ang_v0[k] = initial_base_.ang_v[k];
    it.base_lin_p1[k] = final_base_.lin_p[k];   it.base_lin_v1[k] = final_base_.lin_v[k];
    it.base_ang_p1[k] = final_base_.ang_p[k];   it.base_ang_v1[k] = final_base_.ang_v[k];
  }
  for (int ee = 0; ee < E && ee < (int)initial_ee_W_.size(); ++ee)
    for (int k = 0; k < 3; ++k) {
      it.ee_p0[ee][k] = initial_ee_W_[ee][k];
      if (ee < (int)ee_goal.size()) it.ee_p1[ee][k] = ee_goal[ee][k];
    }
  return d;
}

// ------------------------------------------------------------------------------ canned configs
NlpFormulation AnymalTrot(double total_duration, Vector3d goal) {
  // BASELINE config 3: towr_user_interface.cc:66-73 (T = 2.4, goal x = 2.1), RobotModel::Anymal,
  // quadruped combo C1, the initial state of TowrRosApp::SetTowrInitialState (towr_ros_app.cc:47-58)
  NlpFormulation f;
  f.model_ = RobotModel(RobotModel::Anymal);
  f.terrain_ = HeightMap::MakeTerrain(HeightMap::FlatID);
  const auto& nominal = f.model_.kinematic_model.nominal_stance;
  for (const auto& p : nominal) f.initial_ee_W_.push_back({p[0], p[1], 0.0});
  f.initial_base_.lin_p = {0.0, 0.0, -nominal[0][2] + 0.0};
  f.final_base_.lin_p = goal;
  GaitGenerator gg = GaitGenerator::MakeGaitGenerator(4);
  gg.SetCombo(GaitGenerator::C1);
  for (int ee = 0; ee < 4; ++ee) {
    f.params_.ee_phase_durations_.push_back(gg.GetPhaseDurations(total_duration, ee));
    f.params_.ee_in_contact_at_start_.push_back(gg.IsInContactAtStart(ee));
  }
  return f;
}

NlpFormulation BipedWalk(double total_duration, Vector3d goal) {
  NlpFormulation f;
  f.model_ = RobotModel(RobotModel::Biped);
  f.terrain_ = HeightMap::Flat();
  const auto& nominal = f.model_.kinematic_model.nominal_stance;
  for (const auto& p : nominal) f.initial_ee_W_.push_back({p[0], p[1], 0.0});
  f.initial_base_.lin_p = {0.0, 0.0, -nominal[0][2]};
  f.final_base_.lin_p = goal;
  GaitGenerator gg = GaitGenerator::MakeGaitGenerator(2);
  gg.SetCombo(GaitGenerator::C0);
  for (int ee = 0; ee < 2; ++ee) {
    f.params_.ee_phase_durations_.push_back(gg.GetPhaseDurations(total_duration, ee));
    f.params_.ee_in_contact_at_start_.push_back(gg.IsInContactAtStart(ee));
  }
  return f;
}

NlpFormulation MonopedHopper() {   // hopper_example.cc:105-113 phase durations, flat (BASELINE config 1)
  NlpFormulation f;
  f.model_ = RobotModel(RobotModel::Monoped);
  f.terrain_ = HeightMap::Flat();
  f.params_.ee_phase_durations_.push_back({0.5, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4});
  f.initial_base_.lin_p = {0.0, 0.0, 0.6};
  f.initial_ee_W_.push_back({0.0, 0.0, 0.0});
  f.final_base_.lin_p = {0.0, 0.0, 0.6};
  f.params_.ee_in_contact_at_start_.push_back(true);
  return f;
}

}  // namespace towr_gpu
