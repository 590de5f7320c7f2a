"""The BASELINE.json configurations as ProblemDescs (+ extra parity cases)."""
import math

from towr2025_amd import formulation as F


def config_descs():
    """name -> ProblemDesc: BASELINE.json configs[0..3] plus cases covering every kind and terrain."""
    return {
        "monoped_hopper_flat": F.monoped_hopper().to_desc(),                       # configs[0]
        "monoped_procedural": F.procedural_desc(),                                 # procedural_example.cc
        "biped_walk_2s": F.biped_walk().to_desc(),                                 # configs[1]
        "anymal_trot_2p4s": F.anymal_trot().to_desc(),                             # configs[2]
        "anymal_trot_stairs": F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID)).to_desc(),
        "hopper_five_steps": _hopper_steps(),
        "anymal_slope_yaw": F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.SlopeID),
                                          goal=(1.8, 0.3, 0.0), goal_yaw=0.3).to_desc(),
        "hyq_chimney": _hyq(F.HeightMap.ChimneyID),
        "hyq_chimney_lr": _hyq(F.HeightMap.ChimneyLRID),                          # height_map_examples.cc:186-211
        "hyq_gap": _hyq(F.HeightMap.GapID),
        "anymal_block_baserom": _anymal_baserom(),
        # configs[3]: ANYmal on stairs with phase-duration (gait) optimisation
        "anymal_stairs_gaitopt": F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID),
                                               optimize_timings=True).to_desc(),
        "biped_walk_gaitopt": _gaitopt(F.biped_walk()),
        "hyq_gap_gaitopt": _gaitopt_hyq_gap(),
        # Torque (discretized and node-based), TerrainHard, EELinear
        "biped_torque_hard_eelin": _with_next_tier(F.biped_walk()),
        "hopper_torque_node": _with_next_tier(F.monoped_hopper(), node_torque=True, eelin=False),
        # the fork's hopper driver (hopper_example.cc:95-171): FiveStepStairs, Torque, phase-duration optimisation
        "hopper_gait_torque": F.hopper_example_desc(),
        "anymal_gait_torque": _with_next_tier(F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID),
                                                            optimize_timings=True), hard=False),
        "hyq_gap_torque": _with_next_tier(_hyq_formulation(F.HeightMap.GapID)),
        # RotVecConverter base orientation
        "anymal_trot_rotvec": _rotvec(F.anymal_trot()).to_desc(),
        "biped_gaitopt_rotvec": _rotvec(_gaitopt_f(F.biped_walk())).to_desc(),
        "hopper_next_rotvec": _with_next_tier(_rotvec(F.monoped_hopper()), eelin=False),
        "monoped_backflip_rotvec": F.backflip_desc(),                            # backflip_example.cc
    }


def _rotvec(f):
    f.params_.angular_rep_ = 1
    return f


def _hyq_formulation(tid):
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(tid))
    f.model_ = F.RobotModel(F.RobotModel.Hyq)
    nominal = f.model_.kinematic_model.nominal_stance
    f.initial_ee_W_ = [(p[0], p[1], 0.0) for p in nominal]
    f.initial_base_ = F.BaseState(lin_p=(0.0, 0.0, -nominal[0][2]))
    return f


def _with_next_tier(f, node_torque=False, hard=True, eelin=True):
    P = f.params_
    P.constraints_.append(F.Parameters.Torque)
    if node_torque:
        P.dt_constraint_torque_ = 0.0
    if hard:
        P.constraints_.append(F.Parameters.TerrainHard)
    E = P.GetEECount()
    if eelin and E >= 2:   # symmetric lateral foot positions; yaw-rate of the first foot's angle
        P.ee_linear_constraints_.append(F.EELinearConstraintDef(terms=[(0, 1, 1.0), (1, 1, 1.0)], tolerance=0.5))
        P.ee_linear_constraints_.append(F.EELinearConstraintDef(terms=[(0, 2, 0.5), (E - 1, 0, -1.0), (0, 2, 0.5)],
                                                                target=1, deriv=1, tolerance=1.0, dt=0.05))
    return f.to_desc()


def _gaitopt(f):
    f.params_.OptimizePhaseDurations()
    return f.to_desc()


def _gaitopt_hyq_gap():
    d = _hyq(F.HeightMap.GapID)
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.GapID), optimize_timings=True)
    f.model_ = F.RobotModel(F.RobotModel.Hyq)
    nominal = f.model_.kinematic_model.nominal_stance
    f.initial_ee_W_ = [(p[0], p[1], 0.0) for p in nominal]
    f.initial_base_ = F.BaseState(lin_p=(0.0, 0.0, -nominal[0][2]))
    del d
    return f.to_desc()


def _hopper_steps():
    f = F.monoped_hopper()
    f.terrain_ = F.HeightMap.MakeTerrain(F.HeightMap.StepsID)
    return f.to_desc()


def _hyq(tid):
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(tid))
    f.model_ = F.RobotModel(F.RobotModel.Hyq)
    nominal = f.model_.kinematic_model.nominal_stance
    f.initial_ee_W_ = [(p[0], p[1], 0.0) for p in nominal]
    f.initial_base_ = F.BaseState(lin_p=(0.0, 0.0, -nominal[0][2]))
    return f.to_desc()


def _anymal_baserom():
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.BlockID))
    f.params_.constraints_.append(F.Parameters.BaseRom)
    f.params_.dt_constraint_force_ = 0.0   # node-based ForceConstraint instead of the discretised one
    return f.to_desc()


_with_costs = F.with_costs


def cost_descs():
    """name -> ProblemDesc with cost terms (eval_f / eval_grad_f)."""
    C = F.Parameters
    return {
        "anymal_all_costs": _with_costs(F.anymal_trot()).to_desc(),
        "anymal_stairs_gaitopt_costs": _with_costs(F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID),
                                                                 optimize_timings=True)).to_desc(),
        "biped_energy_angmom": _with_costs(F.biped_walk(), costs=[(C.EnergyCostID, 1e-3), (C.AngMomCostID, 1.0)],
                                           ee_base_pos=True, torque_weight=0.0).to_desc(),
        "biped_gaitopt_costs": _with_costs(_gaitopt_f(F.biped_walk()), torque_weight=2.0).to_desc(),
        "hopper_forces_motion": _with_costs(F.monoped_hopper(), costs=[(C.ForcesCostID, 1.0), (C.EEMotionCostID, 1.0)],
                                            ee_base_pos=False).to_desc(),
        "anymal_rotvec_costs": _with_costs(_rotvec(F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID),
                                                                 optimize_timings=True))).to_desc(),
        "monoped_backflip_rotvec": F.backflip_desc(),
        "hopper_gait_torque": F.hopper_example_desc(),
        "anymal_slope_yaw_costs": _with_costs(F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.SlopeID),
                                                            goal=(1.8, 0.3, 0.0), goal_yaw=0.3)).to_desc(),
    }


def _gaitopt_f(f):
    f.params_.OptimizePhaseDurations()
    return f


# ---- LinearEqualityConstraint, BaseHeightCost, SoftConstraint (VERDICT r1 "missing" 1-2) ----------
def _varset_cols(desc):
    """[(col0, n)] of the description's variable sets (a layout-only handle: no GPU)."""
    from towr2025_amd import TowrGpuProblem
    p = TowrGpuProblem(desc, device=-1)
    return [(c0, n) for (_, _, c0, n) in p.varset_info()]


def _sparse_matrix(rows, cols, seed, density=0.3, zero_row=None):
    import numpy as np
    rng = np.random.default_rng(seed)
    M = rng.standard_normal((rows, cols)) * (rng.random((rows, cols)) < density)
    if zero_row is not None:
        M[zero_row] = 0.0
    return M


def _soft_bounds(rows, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    lo = -rng.random(rows)
    return np.concatenate([lo, lo + 2.0 * rng.random(rows)])


def _biped_example_costs(f, target, with_nodes=True):
    """The cost list of towr/test/biped_example.cc:196-215: BaseHeightCost(target, 1e-1, dt 0.01) and
    NodeCosts on the base motion."""
    from towr2025_amd import _capi as capi
    costs = [dict(kind=capi.COST_BASE_HEIGHT, weight=1e-1, dt=0.01, p=[target])]
    if with_nodes:
        for dim, w in ((0, 1e-4), (1, 1e-2), (2, 1e-3)):
            costs.append(dict(kind=capi.COST_NODE, weight=w, ip=[capi.VAR_BASE_LIN, 1, dim]))
        for dim in range(3):
            costs.append(dict(kind=capi.COST_NODE, weight=1e-3, ip=[capi.VAR_BASE_ANG, 0, dim]))
            costs.append(dict(kind=capi.COST_NODE, weight=1e-4, ip=[capi.VAR_BASE_ANG, 1, dim]))
    return costs


def ext_cases():
    """name -> (ProblemDesc, side data [(towr_data_kind, index, array)]) for the LinearEquality
    constraint, the fork's BaseHeightCost and SoftConstraint terms."""
    from towr2025_amd import _capi as capi
    out = {}
    # LinearEqualityConstraint on base-lin (a zero row of M) and on an ee-motion set, procedural monoped
    f, vs, cs, goal, T = F.procedural_monoped()
    d0 = f.to_desc(varsets=vs, constraints=cs, init_mode=capi.INIT_PROCEDURAL, ee_goal=goal, total_time=T)
    cols = _varset_cols(d0)
    M0 = _sparse_matrix(6, cols[0][1], 11, zero_row=2)
    M1 = _sparse_matrix(3, cols[2][1], 12, density=0.5)
    cs2 = cs + [dict(kind=capi.C_LINEAR_EQ, ip=[0, 6]), dict(kind=capi.C_LINEAR_EQ, ip=[2, 3])]
    d = f.to_desc(varsets=vs, constraints=cs2, init_mode=capi.INIT_PROCEDURAL, ee_goal=goal, total_time=T)
    out["procedural_lineq"] = (d, [(capi.DATA_LINEAR_M, len(cs), M0), (capi.DATA_LINEAR_M, len(cs) + 1, M1)])
    # ... on the schedule set of a phase-duration-optimisation problem (ANYmal stairs, configs[3])
    fg = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True)
    cols_g = _varset_cols(fg.to_desc())
    vsg = fg.variable_sets()
    si = [i for i, (k, ee) in enumerate(vsg) if k == capi.VAR_EE_SCHEDULE][0]
    csg = fg.constraint_sets() + [dict(kind=capi.C_LINEAR_EQ, ip=[si, 2])]
    dg = fg.to_desc(constraints=csg)
    out["anymal_gait_lineq"] = (dg, [(capi.DATA_LINEAR_M, len(csg) - 1,
                                      _sparse_matrix(2, cols_g[si][1], 13, density=0.7))])
    # BaseHeightCost: the fork's biped driver (fixed gait), its phase-duration-optimisation variant, and
    # ANYmal's flying trot on stairs (no foot in contact: the terrain height under the base)
    fb = F.biped_walk()
    z0 = fb.initial_base_.lin_p[2]
    out["biped_base_height_cost"] = (fb.to_desc(costs=_biped_example_costs(fb, z0)), [])
    fbg = _gaitopt_f(F.biped_walk())
    out["biped_gait_base_height_cost"] = (fbg.to_desc(costs=_biped_example_costs(fbg, z0)), [])
    fa = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID))
    out["anymal_stairs_base_height_cost"] = (fa.to_desc(costs=_biped_example_costs(fa, 0.5, with_nodes=False)), [])
    # SoftConstraint: a soft-only BaseMotion set and a wrapped hard Dynamic set, procedural monoped
    f, vs, cs, goal, T = F.procedural_monoped()
    cs3 = cs + [dict(kind=capi.C_BASE_MOTION, T=T, dt=0.1, role=capi.ROLE_SOFT)]
    costs = [dict(kind=capi.COST_SOFT, weight=1.0, ip=[len(cs3) - 1]), dict(kind=capi.COST_SOFT, weight=1.0, ip=[0]),
             dict(kind=capi.COST_NODE, weight=1e-3, ip=[capi.VAR_EE_FORCE, 0, 2])]
    d = f.to_desc(varsets=vs, constraints=cs3, init_mode=capi.INIT_PROCEDURAL, ee_goal=goal, total_time=T, costs=costs)
    rows_bm = 6 * (math.floor(T / 0.1) + 2)     # TimeDiscretizationConstraint instants (time_discretization_constraint.cc:41-49)
    rows_dyn = 6 * (math.floor(T / 0.1) + 2)
    out["procedural_soft"] = (d, [(capi.DATA_SOFT_BOUNDS, 0, _soft_bounds(rows_bm, 21)),
                                  (capi.DATA_SOFT_BOUNDS, 1, _soft_bounds(rows_dyn, 22))])
    # ... under phase-duration optimisation: a soft ForceConstraintDiscretized (the streaming path in the
    # soft child) and a soft LinearEquality set (its matrix re-indexed for the child)
    fg = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True)
    P = fg.params_
    cols_g = _varset_cols(fg.to_desc())
    csg = fg.constraint_sets()
    nfd = 5 * (math.floor(P.GetTotalTime() / P.dt_constraint_force_) + 2)
    csg = csg + [dict(kind=capi.C_FORCE_DISCRETIZED, ee=1, T=P.GetTotalTime(), dt=P.dt_constraint_force_,
                      p=[P.force_limit_in_normal_direction_], role=capi.ROLE_SOFT),
                 dict(kind=capi.C_LINEAR_EQ, ip=[0, 4], role=capi.ROLE_SOFT)]
    costs = [dict(kind=capi.COST_SOFT, weight=1.0, ip=[len(csg) - 2]), dict(kind=capi.COST_SOFT, weight=1.0, ip=[len(csg) - 1])]
    dg = fg.to_desc(constraints=csg, costs=costs)
    out["anymal_gait_soft"] = (dg, [(capi.DATA_LINEAR_M, len(csg) - 1, _sparse_matrix(4, cols_g[0][1], 14)),
                                    (capi.DATA_SOFT_BOUNDS, 0, _soft_bounds(nfd, 23)),
                                    (capi.DATA_SOFT_BOUNDS, 1, _soft_bounds(4, 24))])
    return out


def anymal_long_gait(n_phases=17, phase=0.2):
    """ANYmal on stairs with phase-duration optimisation over a longer horizon (n_phases phases of `phase` s per
    foot, every foot in contact at the start and the end). At 17 phases the FDISC record launch's LDS (staging +
    its FsBlock / window / template tables, towr_gpu.hip rec_launch_lds) is past 64 kB."""
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True,
                      total_duration=phase * n_phases)
    for ee in range(4):
        f.params_.ee_phase_durations_[ee] = [phase] * n_phases
        f.params_.ee_in_contact_at_start_[ee] = True
    return f.to_desc()
