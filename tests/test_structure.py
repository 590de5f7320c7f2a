"""Host-side structure checks of the product (layout-only handles, no GPU): Jacobian pattern
bit-exact vs the oracle, starting point equal, sizes as in SURVEY §8, error behaviour."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from tests.configs import config_descs
from towr2025_amd import TowrGpuError, TowrGpuProblem
from towr2025_amd import _capi as capi
from towr2025_amd import formulation as F

CONFIGS = config_descs()


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_pattern_and_x0_match_oracle(name):
    desc = CONFIGS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=-1)
    assert (p.n, p.m) == (o.n, o.m)
    x0 = o.initial_x()
    np.testing.assert_array_equal(p.initial_x(), x0)
    r, c, _ = o.eval_jac(x0)
    pr, pc = p.jac_structure()
    np.testing.assert_array_equal(pr, r)
    np.testing.assert_array_equal(pc, c)
    rp, cc = p.jac_csr()
    assert rp[-1] == p.nnz and np.array_equal(cc, pc)
    assert np.array_equal(np.repeat(np.arange(p.m), np.diff(rp)), pr)


def test_sizes_match_survey_table():
    """SURVEY §8 problem sizes (n, m) computed from the reference's setup arithmetic."""
    expect = {"anymal_trot_2p4s": (1090, 3238), "biped_walk_2s": (688, 1506),
              "monoped_hopper_flat": (876, 2025), "monoped_procedural": (304, 284)}
    for name, (n, m) in expect.items():
        p = TowrGpuProblem(CONFIGS[name], device=-1)
        assert (p.n, p.m) == (n, m), name


def test_initial_x_for_matches_fresh_layout():
    base = F.anymal_trot()
    p = TowrGpuProblem(base.to_desc(), device=-1)
    other = F.anymal_trot(goal=(2.3, 0.2, 0.0), start_xy=(0.1, -0.2), start_yaw=0.2, goal_yaw=0.25,
                          terrain=F.HeightMap(F.HeightMap.StairsID, (1.1, 0.4, 0.15, 0.2, 1.0)))
    d = other.to_desc()
    np.testing.assert_array_equal(p.initial_x_for(d.init, d.terrain), Oracle(d).initial_x())


def test_unsupported_and_invalid():
    d = F.anymal_trot().to_desc()
    d.angular_rep = 2                      # neither EulerZYX (0) nor RotationVector (1)
    with pytest.raises(TowrGpuError, match="-1"):
        TowrGpuProblem(d, device=-1)
    d = F.anymal_trot(optimize_timings=True).to_desc()
    d.n_varsets -= 1                       # drop a schedule set while optimising timings
    with pytest.raises(TowrGpuError, match="-1"):
        TowrGpuProblem(d, device=-1)
    d = F.anymal_trot().to_desc()
    d.abi_version = 99
    with pytest.raises(TowrGpuError, match="-1"):
        TowrGpuProblem(d, device=-1)
    d = F.anymal_trot().to_desc()
    d.n_varsets -= 1                       # drop a node variable set
    with pytest.raises(TowrGpuError):
        TowrGpuProblem(d, device=-1)


def test_layout_only_handle_cannot_evaluate():
    p = TowrGpuProblem(CONFIGS["monoped_procedural"], device=-1)
    with pytest.raises(TowrGpuError, match="-4"):
        p.eval_g(p.initial_x())


def test_kernel_bytes_cover_the_call():
    p = TowrGpuProblem(CONFIGS["anymal_trot_2p4s"], device=-1)
    ks = {k[0]: k for k in p.kernels()}
    assert {k[1] for k in ks.values() if k[0] < 5} == {"dynamic", "range_of_motion", "force_discretized", "small_kinds"}
    # every value and row is written by exactly one launch class, and by exactly one launch of a step
    assert sum(k[3] for k in ks.values() if k[0] < 5) >= 8 * (p.m + p.nnz)
    steps = p.step_launches()
    assert sum(ks[k][3] for k in steps) >= 8 * (p.m + p.nnz)
    # default fusion: RangeOfMotion + ForceConstraintDiscretized in one launch, x columns counted once
    assert [ks[k][1] for k in steps] == ["range_of_motion+force_discretized", "dynamic", "small_kinds"]
    assert ks[steps[0]][3] <= ks[1][3] + ks[2][3]
    assert ks[steps[0]][2] == ks[1][2] + ks[2][2]   # units = both classes' tiles


@pytest.mark.parametrize("spec,launches", [
    ("none", ["dynamic", "range_of_motion", "force_discretized", "small_kinds"]),
    ("rf,dm", ["range_of_motion+force_discretized", "dynamic+small_kinds"]),
    ("drftm", ["dynamic+range_of_motion+force_discretized+small_kinds"]),
    ("rt", ["dynamic", "range_of_motion", "force_discretized", "small_kinds"]),   # no torque sets: no group
])
def test_fusion_groups_from_environment(monkeypatch, spec, launches):
    monkeypatch.setenv("TOWR_GPU_FUSE", spec)
    p = TowrGpuProblem(CONFIGS["anymal_trot_2p4s"], device=-1)
    names = dict((k[0], k[1]) for k in p.kernels())
    assert [names[k] for k in p.step_launches()] == launches
