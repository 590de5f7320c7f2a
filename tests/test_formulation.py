"""The reference-shaped setup layer: gait generators, Parameters defaults, NlpFormulation order."""
import numpy as np

from towr2025_amd import _capi as capi
from towr2025_amd import formulation as F


def test_quadruped_fly_trot_durations():
    """SURVEY §8 ANYmal C1 at T = 2.4: LF/RH and RF/LH phase durations."""
    g = F.GaitGenerator.MakeGaitGenerator(4)
    g.SetCombo(F.GaitGenerator.C1)
    lf = g.GetPhaseDurations(2.4, F.LF)
    rf = g.GetPhaseDurations(2.4, F.RF)
    np.testing.assert_allclose(lf, [0.42, 0.36, 0.24, 0.36, 0.24, 0.36, 0.42], atol=1e-12)
    np.testing.assert_allclose(rf, [0.18, 0.30, 0.24, 0.36, 0.24, 0.36, 0.24, 0.30, 0.18], atol=1e-12)
    np.testing.assert_allclose(g.GetPhaseDurations(2.4, F.RH), lf, atol=0)
    assert all(g.IsInContactAtStart(e) for e in range(4))


def test_biped_walk_has_204_force_instants():
    f = F.biped_walk()
    d = f.to_desc()
    fd = [d.constraints[i] for i in range(d.n_constraints) if d.constraints[i].kind == capi.C_FORCE_DISCRETIZED]
    assert len(fd) == 2
    n = int(np.floor(fd[0].T / fd[0].dt)) + 2
    assert 2 * n == 204


def test_parameters_defaults_and_base_polys():
    p = F.Parameters()
    assert p.constraints_ == [F.Parameters.Terrain, F.Parameters.Dynamic, F.Parameters.BaseAcc,
                              F.Parameters.EndeffectorRom, F.Parameters.Force, F.Parameters.Swing,
                              F.Parameters.BaseHeight]
    p.ee_phase_durations_ = [[0.5, 0.3, 0.4]]
    p.ee_in_contact_at_start_ = [True]
    assert len(p.GetBasePolyDurations()) == 12
    assert not p.IsOptimizeTimings()
    p.OptimizePhaseDurations()
    assert p.IsOptimizeTimings()


def test_formulation_order():
    f = F.anymal_trot()
    vs = f.variable_sets()
    assert vs[:2] == [(capi.VAR_BASE_LIN, 0), (capi.VAR_BASE_ANG, 0)]
    assert [k for k, _ in vs[2:]] == [capi.VAR_EE_MOTION] * 4 + [capi.VAR_EE_ANG] * 4 + [capi.VAR_EE_FORCE] * 4 + [capi.VAR_EE_TORQUE] * 4
    kinds = [c["kind"] for c in f.constraint_sets()]
    assert kinds == [capi.C_TERRAIN] * 4 + [capi.C_DYNAMIC] + [capi.C_SPLINE_ACC] * 2 + \
        [capi.C_RANGE_OF_MOTION] * 4 + [capi.C_FORCE_DISCRETIZED] * 4 + [capi.C_SWING] * 4 + [capi.C_BASE_HEIGHT]
