"""Host-side problem description, mirroring the reference's setup API.

Names and defaults follow the reference so a towr user finds the same knobs:
  Parameters          towr/src/parameters.cc:40-167, towr/include/towr/parameters.h:135-336
  RobotModel          towr/src/models/robot_model.cc:40-63, include/towr/models/examples/*.h
  HeightMap           towr/include/towr/terrain/height_map.h:79-86, examples/height_map_examples.h
  GaitGenerator       towr/src/initialization/{gait,monoped,biped,quadruped}_gait_generator.cc
  NlpFormulation      towr/src/nlp_formulation.cc:76-378 (variable-set and constraint-set order)

This layer only fills the POD `towr_problem_desc_t` of include/towr_gpu.h. Nothing here
evaluates g or J; that is the HIP engine's job.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

from . import _capi as capi

# ------------------------------------------------------------------ robot models ------------
LF, RF, LH, RH = 0, 1, 2, 3   # endeffector_mappings.h:44
L, R = 0, 1                   # endeffector_mappings.h:43


@dataclass
class KinematicModel:
    nominal_stance: List[Tuple[float, float, float]]
    max_dev: List[Tuple[float, float, float]]
    min_dev: List[Tuple[float, float, float]]


@dataclass
class DynamicModel:
    mass: float
    inertia: Tuple[float, float, float, float, float, float]  # Ixx Iyy Izz Ixy Ixz Iyz
    ee_count: int
    g: float = 9.80665  # dynamic_model.cc:37


class RobotModel:
    """RobotModel(Robot) factory, robot_model.cc:40-63."""
    Monoped, Biped, Hyq, Anymal = range(4)
    names = {0: "Monoped", 1: "Biped", 2: "Hyq", 3: "Anymal"}

    def __init__(self, robot: int):
        self.robot = robot
        if robot == RobotModel.Monoped:      # monoped_model.h:41-60
            self.kinematic_model = KinematicModel([(0.0, 0.0, -0.58)], [(0.30, 0.15, 0.30)],
                                                  [(-0.30, -0.15, -0.30)])
            self.dynamic_model = DynamicModel(20, (1.2, 5.5, 6.0, 0.0, -0.2, -0.01), 1)
        elif robot == RobotModel.Biped:      # biped_model.h:42-69
            z, y = -0.65, 0.20
            self.kinematic_model = KinematicModel([(0.0, y, z), (0.0, -y, z)],
                                                  [(0.25, 0.15, 0.40)] * 2,
                                                  [(-0.25, -0.15, -0.40)] * 2)
            self.dynamic_model = DynamicModel(20, (1.209, 5.583, 6.056, 0.005, -0.190, -0.012), 2)
        elif robot == RobotModel.Hyq:        # hyq_model.h:42-75
            x, y, z = 0.31, 0.29, -0.58
            self.kinematic_model = KinematicModel([(x, y, z), (x, -y, z), (-x, y, z), (-x, -y, z)],
                                                  [(0.25, 0.20, 0.10)] * 4,
                                                  [(-0.25, -0.20, -0.10)] * 4)
            self.dynamic_model = DynamicModel(83, (4.26, 8.97, 9.88, -0.0063, 0.193, 0.0126), 4)
        elif robot == RobotModel.Anymal:     # anymal_model.h:42-76
            x, y, z = 0.34, 0.19, -0.42
            self.kinematic_model = KinematicModel([(x, y, z), (x, -y, z), (-x, y, z), (-x, -y, z)],
                                                  [(0.15, 0.1, 0.10)] * 4,
                                                  [(-0.15, -0.1, -0.10)] * 4)
            self.dynamic_model = DynamicModel(
                29.5, (0.946438, 1.94478, 2.01835, 0.000938112, -0.00595386, -0.00146328), 4)
        else:
            raise ValueError("Robot model not implemented")


# ------------------------------------------------------------------ terrain -----------------
class HeightMap:
    """HeightMap::TerrainID and the example terrains' default parameters."""
    FlatID, BlockID, StairsID, GapID, SlopeID, ChimneyID, ChimneyLRID = range(7)
    StepsID = capi.TERRAIN_STEPS  # FiveStepStairs of towr/test/hopper_example.cc:53-86

    def __init__(self, tid: int, params: Sequence[float] = (), friction_coeff: float = 0.5):
        self.id = tid
        self.params = list(params) + [0.0] * (8 - len(params))
        self.friction_coeff = friction_coeff

    @staticmethod
    def MakeTerrain(tid: int) -> "HeightMap":
        """height_map.cc:37-50 with the member defaults of height_map_examples.h."""
        defaults = {
            HeightMap.FlatID: (0.0,),                          # FlatGround(height=0.0)
            HeightMap.BlockID: (0.7, 3.5, 0.5, 0.03),          # block_start, length, height, eps
            HeightMap.StairsID: (1.0, 0.4, 0.2, 0.4, 1.0),     # first_step_start, width, h1, h2, width_top
            HeightMap.GapID: (1.0, 0.5, 1.5),                  # gap_start, w, h
            HeightMap.SlopeID: (1.0, 1.0, 1.0, 0.7),           # slope_start, up, down, height_center
            HeightMap.ChimneyID: (1.0, 1.5, 0.5, 3.0),         # x_start, length, y_start, slope
            HeightMap.ChimneyLRID: (0.5, 1.0, 0.5, 2.0),
            HeightMap.StepsID: (0.5, 0.3, 0.15, 5.0),          # stairs_start, depth, height, n
        }
        return HeightMap(tid, defaults[tid])

    @staticmethod
    def Flat(height: float = 0.0) -> "HeightMap":
        return HeightMap(HeightMap.FlatID, (height,))

    def GetHeight(self, x: float, y: float) -> float:
        """Host-side restatement used only for the initial guess (NlpFormulation uses
        terrain_->GetHeight for final base/foothold heights, nlp_formulation.cc:130-135, 209)."""
        p = self.params
        if self.id == HeightMap.FlatID:
            return p[0]
        if self.id == HeightMap.BlockID:
            bs, ln, hh, eps = p[0], p[1], p[2], p[3]
            h = 0.0
            if bs <= x <= bs + eps:
                h = hh / eps * (x - bs)
            if bs + eps <= x <= bs + ln:
                h = hh
            return h
        if self.id == HeightMap.StairsID:
            h = 0.0
            if x >= p[0]:
                h = p[2]
            if x >= p[0] + p[1]:
                h = p[3]
            if x >= p[0] + p[1] + p[4]:
                h = 0.0
            return h
        if self.id == HeightMap.GapID:
            gs, w, hh = p[0], p[1], p[2]
            xc = gs + w / 2.0
            a, b = (4 * hh) / (w * w), -(8 * hh * xc) / (w * w)
            c = -(hh * (w - 2 * xc) * (w + 2 * xc)) / (w * w)
            return a * x * x + b * x + c if gs <= x <= gs + w else 0.0
        if self.id == HeightMap.SlopeID:
            ss, xd = p[0], p[0] + p[1]
            xf, slope = xd + p[2], p[3] / p[1]
            z = 0.0
            if x >= ss:
                z = slope * (x - ss)
            if x >= xd:
                z = p[3] - slope * (x - xd)
            if x >= xf:
                z = 0.0
            return z
        if self.id == HeightMap.ChimneyID:
            return p[3] * (y - p[2]) if p[0] <= x <= p[0] + p[1] else 0.0
        if self.id == HeightMap.ChimneyLRID:
            z = 0.0
            if p[0] <= x <= p[0] + p[1]:
                z = p[3] * (y - p[2])
            if p[0] + p[1] <= x <= p[0] + 2 * p[1]:
                z = -p[3] * (y + p[2])
            return z
        if self.id == HeightMap.StepsID:
            if x < p[0]:
                return 0.0
            step = int((x - p[0]) / p[1])
            return p[3] * p[2] if step >= int(p[3]) else (step + 1) * p[2]
        raise ValueError("unknown terrain")

    def to_c(self) -> capi.Terrain:
        t = capi.Terrain()
        t.id = self.id
        t.friction_coeff = self.friction_coeff
        for i, v in enumerate(self.params[:8]):
            t.p[i] = v
        return t


# ------------------------------------------------------------------ gait generators ---------
class GaitGenerator:
    """GaitGenerator (gait_generator.cc:43-144) + the monoped/biped/quadruped combos."""
    C0, C1, C2, C3, C4 = range(5)

    def __init__(self, n_ee: int):
        self.n_ee = n_ee
        self.times: List[float] = []
        self.contacts: List[List[bool]] = []

    @staticmethod
    def MakeGaitGenerator(leg_count: int) -> "GaitGenerator":
        if leg_count == 1:
            return MonopedGaitGenerator()
        if leg_count == 2:
            return BipedGaitGenerator()
        if leg_count == 4:
            return QuadrupedGaitGenerator()
        raise ValueError("gait generator not implemented")

    def _gait(self, name):
        raise NotImplementedError

    def SetGaits(self, gaits: Sequence[str]):
        self.times, self.contacts = [], []
        for g in gaits:
            t, c = self._gait(g)
            self.times += list(t)
            self.contacts += [list(x) for x in c]

    @staticmethod
    def RemoveTransition(g):
        t, c = list(g[0]), list(g[1])
        last = t[-1]
        t.pop()
        t[-1] += last
        c.pop()
        return t, c

    def GetPhaseDurationsAll(self) -> List[List[float]]:
        """GaitGenerator::GetPhaseDurations(), gait_generator.cc:76-105."""
        n_ee = len(self.contacts[0])
        acc = [0.0] * n_ee
        out: List[List[float]] = [[] for _ in range(n_ee)]
        for ph in range(len(self.contacts) - 1):
            cur, nxt = self.contacts[ph], self.contacts[ph + 1]
            for ee in range(n_ee):
                acc[ee] += self.times[ph]
                if cur[ee] != nxt[ee]:
                    out[ee].append(acc[ee])
                    acc[ee] = 0.0
        for ee in range(n_ee):
            out[ee].append(acc[ee] + self.times[-1])
        return out

    def GetNormalizedPhaseDurations(self, ee: int) -> List[float]:
        v = self.GetPhaseDurationsAll()[ee]
        total = 0.0
        for d in v:           # std::accumulate
            total += d
        return [d / total for d in v]

    def GetPhaseDurations(self, t_total: float, ee: int) -> List[float]:
        """gait_generator.cc:54-63"""
        return [d * t_total for d in self.GetNormalizedPhaseDurations(ee)]

    def IsInContactAtStart(self, ee: int) -> bool:
        return self.contacts[0][ee]


class MonopedGaitGenerator(GaitGenerator):
    """monoped_gait_generator.cc:37-120"""

    def __init__(self):
        super().__init__(1)
        self.SetGaits(["Stand"])

    def SetCombo(self, combo):
        c = {0: ["Stand", "Hop1", "Hop1", "Hop1", "Hop1", "Stand"],
             1: ["Stand", "Hop1", "Hop1", "Hop1", "Stand"],
             2: ["Stand", "Hop1", "Hop1", "Hop1", "Hop1", "Stand"],
             3: ["Stand", "Hop2", "Hop2", "Hop2", "Stand"],
             4: ["Stand", "Hop2", "Hop2", "Hop2", "Hop2", "Hop2", "Stand"]}[combo]
        self.SetGaits(c)

    def _gait(self, g):
        o, x = [True], [False]
        return {"Stand": ([0.5], [o]), "Flight": ([0.5], [x]),
                "Hop1": ([0.3, 0.3], [o, x]), "Hop2": ([0.2, 0.3], [o, x])}[g]


class BipedGaitGenerator(GaitGenerator):
    """biped_gait_generator.cc:39-215"""

    def __init__(self):
        super().__init__(2)
        self.SetGaits(["Stand"])

    def SetCombo(self, combo):
        c = {0: ["Stand", "Walk1", "Walk1", "Walk1", "Walk1", "Stand"],
             1: ["Stand", "Run1", "Run1", "Run1", "Run1", "Stand"],
             2: ["Stand", "Hop1", "Hop1", "Hop1", "Stand"],
             3: ["Stand", "Hop1", "Hop2", "Hop2", "Stand"],
             4: ["Stand", "Hop5", "Hop5", "Hop5", "Stand"]}[combo]
        self.SetGaits(c)

    def _gait(self, g):
        I_, b_, P_, B_ = [False, False], [False, True], [True, False], [True, True]
        if g == "Stand":
            return [0.2], [B_]
        if g == "Flight":
            return [0.5], [I_]
        if g in ("Walk1", "Walk2"):
            step, stance = 0.3, 0.05
            return [step, stance, step, stance], [b_, B_, P_, B_]
        if g in ("Run1", "Run3"):
            flight, pushoff, landing = 0.4, 0.15, 0.15
            return [pushoff, flight, landing + pushoff, flight, landing], [b_, I_, P_, I_, b_]
        if g == "Hop1":
            return [0.15, 0.5, 0.15], [B_, I_, B_]
        if g == "Hop2":
            return [0.15, 0.4, 0.15], [b_, I_, b_]
        if g == "Hop3":
            return [0.2, 0.2, 0.2], [P_, I_, P_]
        if g == "Hop5":
            push, flight, land = 0.2, 0.3, 0.2
            return [push, flight, land, land], [P_, I_, b_, B_]
        raise ValueError(g)


class QuadrupedGaitGenerator(GaitGenerator):
    """quadruped_gait_generator.cc:39-365"""

    def __init__(self):
        super().__init__(4)
        f = lambda *on: [i in on for i in range(4)]
        self.II = f()
        self.PI, self.bI, self.IP, self.Ib = f(LH), f(RH), f(LF), f(RF)
        self.Pb, self.bP, self.BI, self.IB = f(LH, RF), f(RH, LF), f(LH, RH), f(LF, RF)
        self.PP, self.bb = f(LH, LF), f(RH, RF)
        self.Bb, self.BP, self.bB, self.PB = f(LH, RH, RF), f(LH, RH, LF), f(RH, LF, RF), f(LH, LF, RF)
        self.BB = f(0, 1, 2, 3)
        self.SetGaits(["Stand"])

    def SetCombo(self, combo):
        c = {0: ["Stand", "Walk2", "Walk2", "Walk2", "Walk2E", "Stand"],
             1: ["Stand", "Run2", "Run2", "Run2", "Run2E", "Stand"],
             2: ["Stand", "Run3", "Run3", "Run3", "Run3E", "Stand"],
             3: ["Stand", "Hop1", "Hop1", "Hop1", "Hop1E", "Stand"],
             4: ["Stand", "Hop3", "Hop3", "Hop3", "Hop3E", "Stand"]}[combo]
        self.SetGaits(c)

    def _gait(self, g):
        s = self
        if g == "Stand":
            return [0.3], [s.BB]
        if g == "Flight":
            return [0.3], [s.Bb]
        if g == "Walk1":
            step, stand = 0.3, 0.2
            return [step, stand] * 4, [s.bB, s.BB, s.Bb, s.BB, s.PB, s.BB, s.BP, s.BB]
        if g in ("Walk2", "Walk2E"):
            three, lateral, diagonal = 0.25, 0.13, 0.13
            gi = ([three, lateral, three, diagonal, three, lateral, three, diagonal],
                  [s.bB, s.bb, s.Bb, s.Pb, s.PB, s.PP, s.BP, s.bP])
            return GaitGenerator.RemoveTransition(gi) if g == "Walk2E" else gi
        if g == "Run1":
            return [0.3, 0.2, 0.3, 0.2], [s.bP, s.BB, s.Pb, s.BB]
        if g == "Run2":
            stand, flight = 0.4, 0.1
            return [stand, flight, stand, flight], [s.bP, s.II, s.Pb, s.II]
        if g == "Run2E":
            return [0.4], [s.bP]
        if g == "Run3":
            return [0.3, 0.1, 0.3, 0.1], [s.PP, s.II, s.bb, s.II]
        if g == "Run3E":
            return [0.3], [s.PP]
        if g == "Hop1":
            return [0.3, 0.1, 0.3, 0.1], [s.BI, s.II, s.IB, s.II]
        if g == "Hop1E":
            return [0.3], [s.BI]
        if g == "Hop2":
            return [0.3, 0.4, 0.3], [s.BB, s.II, s.BB]
        if g in ("Hop3", "Hop3E"):
            A, B, Cc = 0.3, 0.2, 0.2
            gi = ([B, A, B, Cc, B, A, B, Cc], [s.Bb, s.BI, s.BP, s.bP, s.bB, s.IB, s.PB, s.Pb])
            return GaitGenerator.RemoveTransition(gi) if g == "Hop3E" else gi
        if g == "Hop5":
            return [0.1, 0.2, 0.1] * 2, [s.Bb, s.BB, s.IP, s.Bb, s.BB, s.IP]
        raise ValueError(g)


# ------------------------------------------------------------------ parameters --------------
class Parameters:
    """Parameters, parameters.cc:40-167 (defaults) and parameters.h:141-152 (constraint names)."""
    (Dynamic, EndeffectorRom, TotalTime, Terrain, TerrainHard, Force, Torque, Swing, BaseRom,
     BaseAcc, BaseHeight) = range(11)
    ForcesCostID, EEMotionCostID, EnergyCostID, AngMomCostID = range(4)   # parameters.h:157-161

    def __init__(self):
        self.duration_base_polynomial_ = 0.1
        self.force_polynomials_per_stance_phase_ = 3
        self.torque_polynomials_per_stance_phase_ = 3
        self.ee_polynomials_per_swing_phase_ = 2
        self.force_limit_in_normal_direction_ = 1000.0
        self.dt_constraint_range_of_motion_ = 0.08
        self.dt_constraint_dynamic_ = 0.1
        self.dt_constraint_base_motion_ = self.duration_base_polynomial_ / 4.
        self.dt_constraint_force_ = 0.02
        self.dt_constraint_torque_ = 0.02           # 0 => node-based TorqueConstraint
        self.torque_tx_min_, self.torque_tx_max_ = -100.0, 100.0
        self.torque_ty_min_, self.torque_ty_max_ = -100.0, 100.0
        self.torque_k_friction_ = 2.0 / 3.0
        self.ee_linear_constraints_: List["EELinearConstraintDef"] = []
        # costs (parameters.h:157-247): (CostName, weight) pairs; none by default (parameters.cc:90)
        self.costs_: List[Tuple[int, float]] = []
        self.energy_cost_torque_weight_ = 1.0
        self.dt_cost_energy_ = 0.02
        self.dt_cost_ang_mom_ = 0.02
        self.enable_swing_ee_base_pos_tracking = False
        self.swing_ee_base_pos_tracking_weight_ = 1e-2
        self.dt_cost_swing_ee_base_pos_tracking_ = 0.05
        self.dt_constraint_torque_ = 0.02
        self.bound_phase_duration_ = (0.2, 1.0)
        self.constraints_ = [Parameters.Terrain, Parameters.Dynamic, Parameters.BaseAcc,
                             Parameters.EndeffectorRom, Parameters.Force, Parameters.Swing,
                             Parameters.BaseHeight]
        self.ee_phase_durations_: List[List[float]] = []
        self.ee_in_contact_at_start_: List[bool] = []
        self.ee_swing_height_min_: List[float] = []
        self.ee_swing_height_max_: List[float] = []
        self.base_rom_ax = (-1e20, 1e20)
        self.base_rom_ay = (-1e20, 1e20)
        self.base_rom_lz = (-1e20, 1e20)
        self.angular_rep_ = 0  # EulerZYX

    def OptimizePhaseDurations(self):
        self.constraints_.append(Parameters.TotalTime)

    def IsOptimizeTimings(self) -> bool:
        return Parameters.TotalTime in self.constraints_

    def GetEECount(self) -> int:
        return len(self.ee_in_contact_at_start_)

    def GetPhaseCount(self, ee: int) -> int:
        return len(self.ee_phase_durations_[ee])

    def GetTotalTime(self) -> float:
        """parameters.cc:144-158 (std::accumulate of the first foot)."""
        if not self.ee_phase_durations_:
            return 0.0
        T = 0.0
        for d in self.ee_phase_durations_[0]:
            T += d
        return T

    def GetBasePolyDurations(self) -> List[float]:
        """parameters.cc:114-130"""
        out, dt, t_left, eps = [], self.duration_base_polynomial_, self.GetTotalTime(), 1e-10
        while t_left > eps:
            out.append(dt if t_left > dt else t_left)
            t_left -= dt
        return out


def _euler_zyx(a):
    """EulerConverter::GetRotationMatrixBaseToWorld (euler_converter.cc:207-221)."""
    sx, cx, sy, cy, sz, cz = math.sin(a[0]), math.cos(a[0]), math.sin(a[1]), math.cos(a[1]), math.sin(a[2]), math.cos(a[2])
    return [[cy * cz, cz * sx * sy - cx * sz, sx * sz + cx * cz * sy],
            [cy * sz, cx * cz + sx * sy * sz, cx * sy * sz - cz * sx],
            [-sy, cy * sx, cx * cy]]


@dataclass
class EELinearConstraintDef:
    """Parameters::EELinearConstraintDef (parameters.h:317-325): |sum_i coeff_i * ee_i[dim_i]| <= tolerance
    at discretised times, on the ee motion (target 0) or ee angle (target 1) splines, position
    (deriv 0) or velocity (deriv 1). terms: (ee, dim, coeff) triples (at most 6)."""
    terms: List[Tuple[int, int, float]]
    target: int = 0
    deriv: int = 0
    tolerance: float = 0.0
    dt: float = 0.1


@dataclass
class BaseState:
    lin_p: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    lin_v: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    ang_p: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    ang_v: Tuple[float, float, float] = (0.0, 0.0, 0.0)


class NlpFormulation:
    """NlpFormulation (nlp_formulation.cc): builds the ProblemDesc with the same variable-set
    order (GetVariableSets, :76-119) and constraint-set expansion (GetConstraints, :365-398)."""

    def __init__(self):
        self.terrain_ = HeightMap.Flat()
        self.model_ = RobotModel(RobotModel.Monoped)
        self.params_ = Parameters()
        self.initial_base_ = BaseState()
        self.final_base_ = BaseState()
        self.initial_ee_W_: List[Tuple[float, float, float]] = []

    # variable sets in NlpFormulation::GetVariableSets order
    def variable_sets(self) -> List[Tuple[int, int]]:
        E = self.params_.GetEECount()
        vs = [(capi.VAR_BASE_LIN, 0), (capi.VAR_BASE_ANG, 0)]
        vs += [(capi.VAR_EE_MOTION, ee) for ee in range(E)]
        vs += [(capi.VAR_EE_ANG, ee) for ee in range(E)]
        vs += [(capi.VAR_EE_FORCE, ee) for ee in range(E)]
        vs += [(capi.VAR_EE_TORQUE, ee) for ee in range(E)]
        if self.params_.IsOptimizeTimings():
            vs += [(capi.VAR_EE_SCHEDULE, ee) for ee in range(E)]
        return vs

    # constraint sets in NlpFormulation::GetConstraints order
    def constraint_sets(self) -> List[dict]:
        P, E, T = self.params_, self.params_.GetEECount(), self.params_.GetTotalTime()
        out = []
        for name in P.constraints_:
            if name == Parameters.Dynamic:
                out.append(dict(kind=capi.C_DYNAMIC, ee=0, T=T, dt=P.dt_constraint_dynamic_))
            elif name == Parameters.EndeffectorRom:
                out += [dict(kind=capi.C_RANGE_OF_MOTION, ee=ee, T=T, dt=P.dt_constraint_range_of_motion_)
                        for ee in range(E)]
            elif name == Parameters.BaseRom:
                p = list(P.base_rom_ax) + list(P.base_rom_ay) + list(P.base_rom_lz)
                out.append(dict(kind=capi.C_BASE_MOTION, ee=0, T=T, dt=P.dt_constraint_base_motion_, p=p))
            elif name == Parameters.TotalTime:
                out += [dict(kind=capi.C_TOTAL_DURATION, ee=ee, T=T) for ee in range(E)]
            elif name == Parameters.Terrain:
                for ee in range(E):
                    mn = P.ee_swing_height_min_[ee] if ee < len(P.ee_swing_height_min_) else 0.02
                    mx = P.ee_swing_height_max_[ee] if ee < len(P.ee_swing_height_max_) else math.inf
                    if mn < 0.0:
                        raise ValueError("Swing height minimum must be >= 0.0")
                    if mx <= mn:
                        raise ValueError("Swing height maximum must be > minimum")
                    out.append(dict(kind=capi.C_TERRAIN, ee=ee, p=[mn, mx]))
            elif name == Parameters.Force:
                for ee in range(E):
                    if P.dt_constraint_force_ > 0.0:
                        out.append(dict(kind=capi.C_FORCE_DISCRETIZED, ee=ee, T=T, dt=P.dt_constraint_force_,
                                        p=[P.force_limit_in_normal_direction_]))
                    else:
                        out.append(dict(kind=capi.C_FORCE, ee=ee, p=[P.force_limit_in_normal_direction_]))
            elif name == Parameters.Swing:
                out += [dict(kind=capi.C_SWING, ee=ee, p=[0.3]) for ee in range(E)]
            elif name == Parameters.BaseAcc:
                out += [dict(kind=capi.C_SPLINE_ACC, ee=0), dict(kind=capi.C_SPLINE_ACC, ee=1)]
            elif name == Parameters.BaseHeight:
                out.append(dict(kind=capi.C_BASE_HEIGHT, ee=0, p=[0.4]))  # nlp_formulation.cc:597
            elif name == Parameters.TerrainHard:     # nlp_formulation.cc:492-506
                out += [dict(kind=capi.C_TERRAIN_HARD, ee=ee, T=T, dt=P.dt_constraint_range_of_motion_)
                        for ee in range(E)]
            elif name == Parameters.Torque:          # nlp_formulation.cc:533-558
                tp = [P.torque_tx_min_, P.torque_tx_max_, P.torque_ty_min_, P.torque_ty_max_, P.torque_k_friction_]
                for ee in range(E):
                    if P.dt_constraint_torque_ > 0.0:
                        out.append(dict(kind=capi.C_TORQUE_DISCRETIZED, ee=ee, T=T, dt=P.dt_constraint_torque_, p=tp))
                    else:
                        out.append(dict(kind=capi.C_TORQUE, ee=ee, p=tp))
            else:
                raise ValueError("constraint not defined!")
        for dfn in P.ee_linear_constraints_:        # GetConstraints, nlp_formulation.cc:373-375
            if not 1 <= len(dfn.terms) <= 6:
                raise ValueError("EELinear: 1..6 terms supported")
            out.append(dict(kind=capi.C_EE_LINEAR, ee=0, T=T, dt=dfn.dt, p=[c for _, _, c in dfn.terms],
                            ip=[dfn.target, dfn.deriv, len(dfn.terms)] + [e * 3 + d for e, d, _ in dfn.terms]))
        return out

    # cost terms in NlpFormulation::GetCosts order (nlp_formulation.cc:604-680)
    def cost_terms(self) -> List[dict]:
        P, E = self.params_, self.params_.GetEECount()
        out = []
        for name, w in P.costs_:
            if name == Parameters.ForcesCostID:      # MakeForcesCost (:646-664)
                for ee in range(E):
                    for dim in range(3):
                        out.append(dict(kind=capi.COST_NODE, ee=ee, weight=w, ip=[capi.VAR_EE_FORCE, 0, dim]))
                        out.append(dict(kind=capi.COST_NODE, ee=ee, weight=w, ip=[capi.VAR_EE_TORQUE, 0, dim]))
                        out.append(dict(kind=capi.COST_NODE, ee=ee, weight=0.1 * w, ip=[capi.VAR_EE_FORCE, 1, dim]))
                        out.append(dict(kind=capi.COST_NODE, ee=ee, weight=0.1 * w, ip=[capi.VAR_EE_TORQUE, 1, dim]))
            elif name == Parameters.EEMotionCostID:  # MakeEEMotionCost (:666-678)
                for ee in range(E):
                    out.append(dict(kind=capi.COST_NODE, ee=ee, weight=w, ip=[capi.VAR_EE_MOTION, 1, 0]))
                    out.append(dict(kind=capi.COST_NODE, ee=ee, weight=w, ip=[capi.VAR_EE_MOTION, 1, 1]))
                    out.append(dict(kind=capi.COST_NODE, ee=ee, weight=0.5 * w, ip=[capi.VAR_EE_MOTION, 1, 2]))
            elif name == Parameters.EnergyCostID:
                out.append(dict(kind=capi.COST_ENERGY, weight=w, dt=P.dt_cost_energy_, p=[P.energy_cost_torque_weight_]))
            elif name == Parameters.AngMomCostID:
                out.append(dict(kind=capi.COST_ANG_MOMENTUM, weight=w, dt=P.dt_cost_ang_mom_))
            else:
                raise ValueError("cost not defined!")
        if P.enable_swing_ee_base_pos_tracking and P.swing_ee_base_pos_tracking_weight_ > 0.0:   # :613-626
            b0 = self.initial_base_
            R = _euler_zyx(b0.ang_p)
            for ee in range(E):
                rW = [self.initial_ee_W_[ee][k] - b0.lin_p[k] for k in range(3)]
                rB = [R[0][i] * rW[0] + R[1][i] * rW[1] + R[2][i] * rW[2] for i in range(3)]
                out.append(dict(kind=capi.COST_EE_BASE_POS, ee=ee, weight=P.swing_ee_base_pos_tracking_weight_,
                                dt=P.dt_cost_swing_ee_base_pos_tracking_, p=rB))
        return out

    def to_desc(self, varsets=None, constraints=None, init_mode=capi.INIT_FORMULATION,
                ee_goal=None, total_time=None, costs=None) -> capi.ProblemDesc:
        """The engine's problem description. varsets / constraints / costs override the lists
        GetVariableSets / GetConstraints / GetCosts would build (a hand-assembled ifopt::Problem,
        as towr/test/procedural_example.cc and backflip_example.cc do)."""
        P = self.params_
        d = capi.ProblemDesc()
        d.abi_version = capi.ABI_VERSION
        d.angular_rep = P.angular_rep_
        km, dm = self.model_.kinematic_model, self.model_.dynamic_model
        E = P.GetEECount()
        if E != dm.ee_count:
            raise ValueError("params ee count does not match robot")
        d.robot.mass, d.robot.gravity = dm.mass, dm.g
        for i, v in enumerate(dm.inertia):
            d.robot.inertia[i] = v
        d.robot.n_ee = E
        for ee in range(E):
            for k in range(3):
                d.robot.nominal_stance[ee][k] = km.nominal_stance[ee][k]
                d.robot.max_dev[ee][k] = km.max_dev[ee][k]
                d.robot.min_dev[ee][k] = km.min_dev[ee][k]
        d.terrain = self.terrain_.to_c()
        d.total_time = P.GetTotalTime() if total_time is None else total_time
        d.duration_base_polynomial = P.duration_base_polynomial_
        d.ee_polynomials_per_swing_phase = P.ee_polynomials_per_swing_phase_
        d.force_polynomials_per_stance_phase = P.force_polynomials_per_stance_phase_
        d.torque_polynomials_per_stance_phase = P.torque_polynomials_per_stance_phase_
        d.optimize_timings = int(P.IsOptimizeTimings())
        d.bound_phase_duration[0], d.bound_phase_duration[1] = P.bound_phase_duration_
        for ee in range(E):
            ph = P.ee_phase_durations_[ee]
            if len(ph) > capi.MAX_PHASES:
                raise ValueError("too many phases")
            d.n_phases[ee] = len(ph)
            d.contact_at_start[ee] = int(P.ee_in_contact_at_start_[ee])
            for i, v in enumerate(ph):
                d.phase_durations[ee][i] = v
        vs = self.variable_sets() if varsets is None else varsets
        d.n_varsets = len(vs)
        for i, (k, ee) in enumerate(vs):
            d.varsets[i].kind, d.varsets[i].ee = k, ee
        cs = self.constraint_sets() if constraints is None else constraints
        d.n_constraints = len(cs)
        for i, c in enumerate(cs):
            d.constraints[i].kind = c["kind"]
            d.constraints[i].ee = c.get("ee", 0)
            d.constraints[i].T = c.get("T", d.total_time)
            d.constraints[i].dt = c.get("dt", 0.0)
            for j, v in enumerate(c.get("p", [])):
                d.constraints[i].p[j] = v
            for j, v in enumerate(c.get("ip", [])):
                d.constraints[i].ip[j] = v
            d.constraints[i].role = c.get("role", capi.ROLE_HARD)
        cts = self.cost_terms() if costs is None else costs
        if len(cts) > capi.MAX_COSTS:
            raise ValueError("too many cost terms")
        d.n_costs = len(cts)
        for i, c in enumerate(cts):
            d.costs[i].kind, d.costs[i].ee = c["kind"], c.get("ee", 0)
            d.costs[i].weight, d.costs[i].dt = c["weight"], c.get("dt", 0.0)
            for j, v in enumerate(c.get("p", [])):
                d.costs[i].p[j] = v
            for j, v in enumerate(c.get("ip", [])):
                d.costs[i].ip[j] = v
        it = d.init
        it.mode = init_mode
        b0, b1 = self.initial_base_, self.final_base_
        for k in range(3):
            it.base_lin_p0[k], it.base_lin_v0[k] = b0.lin_p[k], b0.lin_v[k]
            it.base_ang_p0[k], it.base_ang_v0[k] = b0.ang_p[k], b0.ang_v[k]
            it.base_lin_p1[k], it.base_lin_v1[k] = b1.lin_p[k], b1.lin_v[k]
            it.base_ang_p1[k], it.base_ang_v1[k] = b1.ang_p[k], b1.ang_v[k]
        for ee in range(min(E, len(self.initial_ee_W_))):
            for k in range(3):
                it.ee_p0[ee][k] = self.initial_ee_W_[ee][k]
                if ee_goal is not None:
                    it.ee_p1[ee][k] = ee_goal[ee][k]
        return d


# ------------------------------------------------------------------ canned configurations ----
def anymal_trot(total_duration=2.4, goal=(2.1, 0.0, 0.0), terrain=None, optimize_timings=False,
                start_xy=(0.0, 0.0), start_yaw=0.0, goal_yaw=0.0) -> NlpFormulation:
    """BASELINE config 3 (and 4/5 variants): towr_ros defaults (towr_user_interface.cc:66-73:
    T=2.4, goal x=2.1) with RobotModel::Anymal, quadruped combo C1 (fly trot), the initial state of
    TowrRosApp::SetTowrInitialState (towr_ros_app.cc:47-58)."""
    f = NlpFormulation()
    f.model_ = RobotModel(RobotModel.Anymal)
    f.terrain_ = terrain if terrain is not None else HeightMap.MakeTerrain(HeightMap.FlatID)
    nominal = f.model_.kinematic_model.nominal_stance
    z_ground = 0.0
    f.initial_ee_W_ = [(p[0] + start_xy[0], p[1] + start_xy[1], z_ground) for p in nominal]
    f.initial_base_ = BaseState(lin_p=(start_xy[0], start_xy[1], -nominal[0][2] + z_ground),
                                ang_p=(0.0, 0.0, start_yaw))
    f.final_base_ = BaseState(lin_p=tuple(goal), ang_p=(0.0, 0.0, goal_yaw))
    gg = GaitGenerator.MakeGaitGenerator(4)
    gg.SetCombo(GaitGenerator.C1)
    for ee in range(4):
        f.params_.ee_phase_durations_.append(gg.GetPhaseDurations(total_duration, ee))
        f.params_.ee_in_contact_at_start_.append(gg.IsInContactAtStart(ee))
    if optimize_timings:
        f.params_.OptimizePhaseDurations()
    return f


def biped_walk(total_duration=2.0, goal=(1.0, 0.0, 0.0)) -> NlpFormulation:
    """BASELINE config 2: Biped, BipedGaitGenerator C0 scaled to T=2.0."""
    f = NlpFormulation()
    f.model_ = RobotModel(RobotModel.Biped)
    f.terrain_ = HeightMap.Flat()
    nominal = f.model_.kinematic_model.nominal_stance
    f.initial_ee_W_ = [(p[0], p[1], 0.0) for p in nominal]
    f.initial_base_ = BaseState(lin_p=(0.0, 0.0, -nominal[0][2]))
    f.final_base_ = BaseState(lin_p=tuple(goal))
    gg = GaitGenerator.MakeGaitGenerator(2)
    gg.SetCombo(GaitGenerator.C0)
    for ee in range(2):
        f.params_.ee_phase_durations_.append(gg.GetPhaseDurations(total_duration, ee))
        f.params_.ee_in_contact_at_start_.append(gg.IsInContactAtStart(ee))
    return f


def monoped_hopper() -> NlpFormulation:
    """BASELINE config 1: monoped with the phase durations of towr/test/hopper_example.cc:105-113,
    flat terrain as BASELINE states (the fork's example uses FiveStepStairs; pass
    terrain=HeightMap.MakeTerrain(HeightMap.StepsID) for that)."""
    f = NlpFormulation()
    f.model_ = RobotModel(RobotModel.Monoped)
    f.terrain_ = HeightMap.Flat()
    f.params_.ee_phase_durations_.append([0.5, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4, 0.3, 0.4])
    f.initial_base_ = BaseState(lin_p=(0.0, 0.0, 0.6))
    f.initial_ee_W_ = [(0.0, 0.0, 0.0)]
    f.final_base_ = BaseState(lin_p=(0.0, 0.0, 0.6))
    f.params_.ee_in_contact_at_start_.append(True)
    return f


def hopper_example():
    """The fork's own hopper driver exactly as towr/test/hopper_example.cc:95-171 builds it: monoped on the
    FiveStepStairs terrain (:53-86), its 13 phase durations, Parameters::Torque added to the default
    constraints (:145), costs ForcesCost 1e-9 and EEMotionCost 1e-4 (:147-148), OptimizePhaseDurations
    (:150), then NodeCosts 1e-4 on the base-linear and base-angular position and velocity nodes of every
    dimension, added after GetCosts (:163-168). The stance-position bounds (:114-122) are variable bounds,
    not evaluation inputs. Returns (formulation, cost terms in ifopt AddCostSet order)."""
    f = monoped_hopper()
    f.terrain_ = HeightMap.MakeTerrain(HeightMap.StepsID)
    P = f.params_
    P.constraints_.append(Parameters.Torque)
    P.costs_ = [(Parameters.ForcesCostID, 1e-9), (Parameters.EEMotionCostID, 1e-4)]
    P.OptimizePhaseDurations()
    # final base: z = 0.6 + FiveStepStairs().GetHeight(0, 0) (:131), 0.6 in front of the stairs
    f.final_base_ = BaseState(lin_p=(0.0, 0.0, 0.6 + f.terrain_.GetHeight(0.0, 0.0)))
    costs = f.cost_terms()
    for dim in range(3):
        for var in (capi.VAR_BASE_LIN, capi.VAR_BASE_ANG):
            costs.append(dict(kind=capi.COST_NODE, weight=1e-4, ip=[var, 0, dim]))
            costs.append(dict(kind=capi.COST_NODE, weight=1e-4, ip=[var, 1, dim]))
    return f, costs


def hopper_example_desc() -> capi.ProblemDesc:
    f, costs = hopper_example()
    return f.to_desc(costs=costs)


def procedural_monoped():
    """towr/test/procedural_example.cc:54-242: manual variable order and constraint list, node-based
    ForceConstraint, plain linear initialisation. Returns (formulation, varsets, constraints, goal)."""
    f = NlpFormulation()
    f.model_ = RobotModel(RobotModel.Monoped)
    f.terrain_ = HeightMap.Flat(0.0)
    f.params_.ee_phase_durations_.append([0.3, 0.2, 0.3, 0.2, 0.3])
    f.params_.ee_in_contact_at_start_.append(True)
    f.initial_base_ = BaseState(lin_p=(0.0, 0.0, 0.58))
    f.final_base_ = BaseState(lin_p=(1.0, 0.0, 0.58))
    f.initial_ee_W_ = [(0.0, 0.0, 0.0)]
    T = 1.3
    vs = [(capi.VAR_BASE_LIN, 0), (capi.VAR_BASE_ANG, 0), (capi.VAR_EE_MOTION, 0),
          (capi.VAR_EE_ANG, 0), (capi.VAR_EE_FORCE, 0), (capi.VAR_EE_TORQUE, 0)]
    cs = [dict(kind=capi.C_DYNAMIC, ee=0, T=T, dt=0.1),
          dict(kind=capi.C_RANGE_OF_MOTION, ee=0, T=T, dt=0.08),
          dict(kind=capi.C_TERRAIN, ee=0, p=[0.02, 0.5]),
          dict(kind=capi.C_FORCE, ee=0, p=[1000.0]),
          dict(kind=capi.C_SWING, ee=0, p=[0.3]),
          dict(kind=capi.C_SPLINE_ACC, ee=0),
          dict(kind=capi.C_SPLINE_ACC, ee=1),
          dict(kind=capi.C_BASE_HEIGHT, ee=0, p=[0.3])]
    goal = [(1.0, 0.0, 0.0)]
    return f, vs, cs, goal, T


def procedural_desc() -> capi.ProblemDesc:
    f, vs, cs, goal, T = procedural_monoped()
    return f.to_desc(varsets=vs, constraints=cs, init_mode=capi.INIT_PROCEDURAL, ee_goal=goal,
                     total_time=T)


def backflip_monoped():
    """towr/test/backflip_example.cc:43-192: monoped backflip with the RotVecConverter (rotation vector
    0 -> (0, -2 pi, 0)), phases 0.5 / 0.8 / 0.6 s, 3 swing / 4 force and torque polynomials, manual
    constraint list and NodeCosts on force and torque. Returns (formulation, varsets, constraints,
    goal, T, costs). The procedural initialisation interpolates the ee angle like the base angle
    (the example sets it to zero); x0 is only the starting point."""
    f = NlpFormulation()
    f.model_ = RobotModel(RobotModel.Monoped)
    f.terrain_ = HeightMap.Flat(0.0)
    P = f.params_
    P.angular_rep_ = 1
    P.ee_phase_durations_.append([0.5, 0.8, 0.6])
    P.ee_in_contact_at_start_.append(True)
    P.ee_polynomials_per_swing_phase_ = 3
    P.force_polynomials_per_stance_phase_ = 4
    P.torque_polynomials_per_stance_phase_ = 4
    f.initial_base_ = BaseState(lin_p=(0.0, 0.0, 0.58))
    f.final_base_ = BaseState(lin_p=(0.0, 0.0, 0.58), ang_p=(0.0, -2.0 * math.pi, 0.0))
    f.initial_ee_W_ = [(0.0, 0.0, 0.0)]
    T = 1.9
    vs = [(capi.VAR_BASE_LIN, 0), (capi.VAR_BASE_ANG, 0), (capi.VAR_EE_MOTION, 0),
          (capi.VAR_EE_ANG, 0), (capi.VAR_EE_FORCE, 0), (capi.VAR_EE_TORQUE, 0)]
    cs = [dict(kind=capi.C_DYNAMIC, ee=0, T=T, dt=0.1),
          dict(kind=capi.C_RANGE_OF_MOTION, ee=0, T=T, dt=0.08),
          dict(kind=capi.C_TERRAIN, ee=0, p=[0.02, 1e20]),
          dict(kind=capi.C_FORCE, ee=0, p=[2000.0]),
          dict(kind=capi.C_SWING, ee=0, p=[0.3]),
          dict(kind=capi.C_SPLINE_ACC, ee=0),
          dict(kind=capi.C_SPLINE_ACC, ee=1)]
    costs = []
    for d in range(3):
        costs.append(dict(kind=capi.COST_NODE, ee=0, weight=1e-5, ip=[capi.VAR_EE_FORCE, 0, d]))
        costs.append(dict(kind=capi.COST_NODE, ee=0, weight=1e-5, ip=[capi.VAR_EE_TORQUE, 0, d]))
    return f, vs, cs, [(0.0, 0.0, 0.0)], T, costs


def backflip_desc() -> capi.ProblemDesc:
    f, vs, cs, goal, T, costs = backflip_monoped()
    return f.to_desc(varsets=vs, constraints=cs, init_mode=capi.INIT_PROCEDURAL, ee_goal=goal, total_time=T,
                     costs=costs)


def with_costs(f: "NlpFormulation", costs=None, ee_base_pos=True, torque_weight=None) -> "NlpFormulation":
    """Enables cost terms (Parameters::costs_, parameters.h:157-247) on a formulation; by default every
    kind: Forces 1e-3, EEMotion 0.5, Energy 1e-4, AngularMomentum 0.1 and the swing ee-base tracking."""
    P = f.params_
    P.costs_ = costs if costs is not None else [(Parameters.ForcesCostID, 1e-3), (Parameters.EEMotionCostID, 0.5),
                                                 (Parameters.EnergyCostID, 1e-4), (Parameters.AngMomCostID, 0.1)]
    P.enable_swing_ee_base_pos_tracking = ee_base_pos
    if torque_weight is not None:
        P.energy_cost_torque_weight_ = torque_weight
    return f
