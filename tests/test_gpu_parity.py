"""GPU parity: the HIP engine through the C-ABI vs the CPU oracle (pattern bit-exact, values within
BASELINE.md's gate, tests/parity.py), on every configuration and on seeded perturbations of x0.

The gate is row-scaled everywhere; only the phase-duration columns of gait-optimisation configs get
the column-scaled floor (tests/parity.py). Each test prints the largest relative error it saw."""
import numpy as np
import pytest

from oracle.oracle import Oracle
from tests.configs import config_descs, cost_descs
from tests.parity import assert_close, assert_cost_close, residue_cols
from tests.gap_frozen import frozen_reference, is_gap
from towr2025_amd import TowrGpuProblem
from towr2025_amd import formulation as F

pytestmark = pytest.mark.gpu

CONFIGS = config_descs()


def _perturb(x0, seed, scale=0.05):
    return x0 + scale * np.random.default_rng(seed).standard_normal(x0.shape)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_pattern_and_values(name):
    desc = CONFIGS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    x0 = o.initial_x()
    np.testing.assert_array_equal(p.initial_x(), x0)
    r, c, _ = o.eval_jac(x0)
    pr, pc = p.jac_structure()
    np.testing.assert_array_equal(pr, r)
    np.testing.assert_array_equal(pc, c)
    fc = residue_cols(desc, o.n)
    worst = {"max_rel": 0.0, "worst": 0.0, "widened": 0}
    for seed in (0, 1, 2):
        x = x0 if seed == 0 else _perturb(x0, 20261015 + seed)
        g_ref = o.eval_g(x)
        rr, cc, v_ref = o.eval_jac(x)
        moved = len(rr) != len(r) or not (np.array_equal(rr, r) and np.array_equal(cc, c))
        outside = 0
        if moved:
            # only curved terrain moves the reference's pattern; compare on the frozen pattern
            assert is_gap(desc), f"{name} seed {seed}: the reference pattern moved on a non-Gap terrain"
            v_ref, outside = frozen_reference(o, r, c, x)
            print(f"{name} seed {seed}: reference pattern moved, {outside} reference entries outside the frozen pattern")
        # the engine reports exactly the reference entries its frozen pattern cannot deliver
        assert p.pattern_outside(x) == outside, f"{name} seed {seed}: pattern_outside {p.pattern_outside(x)} != {outside}"
        g = p.eval_g(x)
        v = p.eval_jac_values(x)
        st = assert_close(g_ref, g, r, v_ref, v, o.m, f"{name} seed {seed} (separate calls)", cols_ref=c, floor_cols=fc)
        worst = {k: max(worst[k], st[k]) for k in worst}
        g2, v2 = p.eval_g_jac(x)
        np.testing.assert_array_equal(g2, g)
        np.testing.assert_array_equal(v2, v)
    print(f"{name}: max relative error {worst['max_rel']:.3e}, worst |err|/tol {worst['worst']:.3f}, "
          f"schedule-column floor widened {worst['widened']} entries")


def test_batch_host_matches_single():
    desc = CONFIGS["anymal_trot_2p4s"]
    o = Oracle(desc)
    p = TowrGpuProblem(desc)
    x0 = o.initial_x()
    X = np.stack([_perturb(x0, 100 + b) for b in range(7)])
    G, V = p.eval_batch(X)
    r, _, _ = o.eval_jac(x0)
    for b in range(7):
        assert_close(o.eval_g(X[b]), G[b], r, o.eval_jac(X[b])[2], V[b], o.m, f"batch {b}")


def test_batch_device_per_problem_terrain():
    import torch
    from towr2025_amd import formulation as F
    base = F.anymal_trot()
    desc = base.to_desc()
    p = TowrGpuProblem(desc)
    B = 33
    rng = np.random.default_rng(7)
    terrains, X = [], []
    for b in range(B):
        if b % 2:
            t = F.HeightMap.Flat(rng.uniform(0, 0.3))
        else:
            t = F.HeightMap(F.HeightMap.StairsID, (rng.uniform(0.8, 1.4), 0.4, rng.uniform(0.1, 0.25), rng.uniform(0.1, 0.25), 1.0))
        f = F.anymal_trot(terrain=t)
        terrains.append(f.terrain_.to_c())
        o = Oracle(f.to_desc())
        X.append(_perturb(o.initial_x(), 500 + b))
    X = np.stack(X)
    p.set_batch_terrain(terrains)
    ldv = (p.nnz + 15) // 16 * 16
    dev = torch.device("cuda:0")
    Xd = torch.from_numpy(X).to(dev)
    Gd = torch.full((B, p.m), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
    p.eval_batch_device(Xd, Gd, Vd)
    torch.cuda.synchronize()
    G, V = Gd.cpu().numpy(), Vd.cpu().numpy()[:, :p.nnz]
    for b in range(B):
        d = F.anymal_trot(terrain=None).to_desc()
        d.terrain = terrains[b]
        o = Oracle(d)
        rr, _, v_ref = o.eval_jac(X[b])
        assert_close(o.eval_g(X[b]), G[b], rr, v_ref, V[b], o.m, f"device batch {b}")
    assert np.isnan(Vd.cpu().numpy()[:, p.nnz:]).all()   # padding untouched


COSTS = cost_descs()


@pytest.mark.parametrize("name", sorted(COSTS))
def test_costs_objective_and_gradient(name):
    """eval_f / eval_grad_f through the C-ABI vs the oracle (tests/parity.py assert_cost_close)."""
    desc = COSTS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    x0 = o.initial_x()
    for seed in (0, 1, 2):
        x = x0 if seed == 0 else _perturb(x0, 777 + seed)
        f = p.eval_f(x)
        g = p.eval_grad_f(x)
        assert_cost_close(o.eval_f(x), f, o.eval_grad_f(x), g, f"{name} seed {seed}")


def test_costs_batch_device_matches_single():
    import torch
    desc = COSTS["anymal_stairs_gaitopt_costs"]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    x0 = o.initial_x()
    B = 37
    X = np.stack([_perturb(x0, 300 + b, 0.02) for b in range(B)])
    Xd = torch.zeros((B, o.n + 5), dtype=torch.float64, device="cuda")   # padded leading dimensions
    Xd[:, :o.n] = torch.from_numpy(X).cuda()
    Fd = torch.zeros(B, dtype=torch.float64, device="cuda")
    Gd = torch.full((B, o.n + 3), float("nan"), dtype=torch.float64, device="cuda")
    p.eval_cost_batch_device(Xd, Fd, Gd)
    F0 = torch.zeros(B, dtype=torch.float64, device="cuda")
    p.eval_cost_batch_device(Xd, F0)   # objective only
    torch.cuda.synchronize()
    Fh, Gh, F0h = Fd.cpu().numpy(), Gd.cpu().numpy(), F0.cpu().numpy()
    for b in range(0, B, 6):
        assert_cost_close(o.eval_f(X[b]), Fh[b], o.eval_grad_f(X[b]), Gh[b, :o.n], f"batch {b}")
    np.testing.assert_array_equal(F0h, Fh)
    assert np.all(np.isnan(Gh[:, o.n:]))   # nothing written past n


@pytest.mark.parametrize("name", ["anymal_all_costs", "anymal_stairs_gaitopt_costs", "anymal_rotvec_costs",
                                  "biped_energy_angmom"])
def test_costs_gradient_bit_reproducible(name):
    """The objective and gradient do not depend on scheduling: 512 copies of one x in a batch (blocks on
    every CU at once) and a second call give identical bits in every row (cost_traj.hip: slots summed in
    a fixed order, or exact fixed-point limbs), and the single-problem entry point gives the same bits."""
    import torch
    desc = COSTS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    x = _perturb(o.initial_x(), 4242, 0.03)
    B = 512
    Xd = torch.from_numpy(np.tile(x, (B, 1))).cuda()
    runs = []
    for _ in range(2):
        Fd = torch.zeros(B, dtype=torch.float64, device="cuda")
        Gd = torch.zeros((B, o.n), dtype=torch.float64, device="cuda")
        p.eval_cost_batch_device(Xd, Fd, Gd)
        torch.cuda.synchronize()
        runs.append((Fd.cpu().numpy(), Gd.cpu().numpy()))
    for Fh, Gh in runs:
        assert (Fh == Fh[0]).all()
        assert (Gh.view(np.uint64) == Gh[0].view(np.uint64)).all(), f"rows differ: {np.unique(np.nonzero(Gh != Gh[0])[0])[:8]}"
    np.testing.assert_array_equal(runs[0][1].view(np.uint64), runs[1][1].view(np.uint64))
    g1 = p.eval_grad_f(x)
    np.testing.assert_array_equal(g1.view(np.uint64), runs[0][1][0].view(np.uint64))
    assert_cost_close(o.eval_f(x), runs[0][0][0], o.eval_grad_f(x), runs[0][1][0], name)


# every launch arrangement (TOWR_GPU_FUSE) on configurations covering all launch classes: the
# default fusion group, per-class launches, and the fused groups measured slower (kept selectable)
@pytest.mark.parametrize("spec", ["none", "rf,dm", "drftm", "rftm,d"])
@pytest.mark.parametrize("name", ["anymal_trot_2p4s", "biped_torque_hard_eelin", "anymal_stairs_gaitopt", "anymal_trot_rotvec", "anymal_gait_torque"])
def test_fusion_groups(monkeypatch, spec, name):
    monkeypatch.setenv("TOWR_GPU_FUSE", spec)
    desc = CONFIGS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    x = _perturb(o.initial_x(), 77)
    r, c, v_ref = o.eval_jac(x)
    g, v = p.eval_g_jac(x)
    assert_close(o.eval_g(x), g, r, v_ref, v, o.m, f"{name} fuse {spec}", cols_ref=c, floor_cols=residue_cols(desc, o.n))


# Phase-duration optimisation: the streaming record + compose path (default) and the tile path it
# replaced (TOWR_GPU_GAIT_TILES, read at handle creation) both against the oracle, and against each other;
# one and two launch streams (TOWR_GPU_STREAMS: the record scratch is per class, the classes overlap)
@pytest.mark.parametrize("name", ["anymal_stairs_gaitopt", "biped_gaitopt_rotvec", "anymal_gait_torque", "hyq_gap_gaitopt",
                                  "hopper_gait_torque"])
def test_gait_paths(monkeypatch, name):
    from towr2025_amd import _capi as capi
    desc = CONFIGS[name]
    torque = any(desc.constraints[i].kind == capi.C_TORQUE_DISCRETIZED for i in range(desc.n_constraints))
    o = Oracle(desc)
    x = _perturb(o.initial_x(), 91)
    r, c, _ = o.eval_jac(o.initial_x())   # the pattern is frozen at x0 (Gap: the reference's moves with x)
    v_ref = frozen_reference(o, r, c, x)[0] if is_gap(desc) else o.eval_jac(x)[2]
    fc = residue_cols(desc, o.n)
    outs = {}
    for tiles, streams in ((None, None), ("1", None), (None, "1"), (None, "3")):
        for var, val in (("TOWR_GPU_GAIT_TILES", tiles), ("TOWR_GPU_STREAMS", streams)):
            if val is None:
                monkeypatch.delenv(var, raising=False)
            else:
                monkeypatch.setenv(var, val)
        p = TowrGpuProblem(desc, device=0)
        assert p.kernel_path(0) == (0 if tiles else 1) and p.kernel_path(1) == (0 if tiles else 1)
        if torque:   # TorqueConstraintDiscretized: record + compose except on curved terrain (data-dependent motion block)
            assert p.kernel_path(3) == (0 if tiles or is_gap(desc) else 1)
        g, v = p.eval_g_jac(x)
        assert_close(o.eval_g(x), g, r, v_ref, v, o.m, f"{name} tiles={tiles} streams={streams}", cols_ref=c, floor_cols=fc)
        outs[(tiles, streams)] = (g, v)
        p.close()
    for k in ((None, "1"), (None, "3")):   # the stream count changes only the launch order
        np.testing.assert_array_equal(outs[k][0], outs[(None, None)][0])
        np.testing.assert_array_equal(outs[k][1], outs[(None, None)][1])


@pytest.mark.parametrize("tiles", [None, "1"])
def test_long_gait_record_lds_past_64k(monkeypatch, tiles):
    """A longer gait horizon (tests/configs.py anymal_long_gait: 17 phases per foot) whose FDISC record launch needs
    more than 64 kB of LDS for its staging and FsBlock / window / template tables. With RangeOfMotion / Dynamic on
    the tile path (TOWR_GPU_GAIT_TILES) no record launch has a Dynamic part, so the FDISC launch's LDS alone sets
    the kernel's dynamic-LDS attribute (towr_gpu.hip rec_launch_lds, used at creation and at the launch); the
    default path streams every class. Both against the oracle, single call and a B = 70 batch."""
    import torch
    from tests.configs import anymal_long_gait
    if tiles is None:
        monkeypatch.delenv("TOWR_GPU_GAIT_TILES", raising=False)
    else:
        monkeypatch.setenv("TOWR_GPU_GAIT_TILES", tiles)
    desc = anymal_long_gait()
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    assert p.kernel_path(2) == 1 and p.kernel_path(0) == (0 if tiles else 1)
    x0 = o.initial_x()
    r, c, _ = o.eval_jac(x0)
    fc = residue_cols(desc, o.n)
    x = _perturb(x0, 1717, 0.02)
    g, v = p.eval_g_jac(x)
    assert_close(o.eval_g(x), g, r, o.eval_jac(x)[2], v, o.m, f"long gait tiles={tiles}", cols_ref=c, floor_cols=fc)
    B = 70
    X = np.stack([_perturb(x0, 1800 + b, 0.02) for b in range(B)])
    dev = torch.device("cuda:0")
    Gd = torch.full((B, p.m), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, p.nnz), np.nan, dtype=torch.float64, device=dev)
    p.eval_batch_device(torch.from_numpy(X).to(dev), Gd, Vd)
    torch.cuda.synchronize()
    G, V = Gd.cpu().numpy(), Vd.cpu().numpy()
    for b in (0, 41, B - 1):
        assert_close(o.eval_g(X[b]), G[b], r, o.eval_jac(X[b])[2], V[b], o.m, f"long gait batch {b} tiles={tiles}",
                     cols_ref=c, floor_cols=fc)


@pytest.mark.parametrize("name", ["hyq_gap", "hyq_gap_gaitopt"])
def test_gap_batch(name):
    """Gap batches (one handle, per-problem Gap terrains): every problem's values on the frozen pattern are
    its reference's (the oracle with that problem's terrain), and the batch's frozen-pattern counts equal
    the oracle's count of its reference entries outside the frozen pattern."""
    import torch
    from towr2025_amd import formulation as F
    desc = CONFIGS[name]
    o0 = Oracle(desc)
    x0 = o0.initial_x()
    r, c, _ = o0.eval_jac(x0)
    p = TowrGpuProblem(desc, device=0)
    B = 10
    rng = np.random.default_rng(11)
    terrains, X = [], []
    for b in range(B):
        t = F.HeightMap(F.HeightMap.GapID, (rng.uniform(0.9, 1.1), rng.uniform(0.45, 0.55), rng.uniform(1.2, 1.6)))
        terrains.append(t.to_c())
        X.append(_perturb(x0, 7000 + b, 0.02 + 0.02 * (b % 3)))
    X = np.stack(X)
    p.set_batch_terrain(terrains)
    dev = torch.device("cuda:0")
    Xd = torch.from_numpy(X).to(dev)
    ldv = (p.nnz + 15) // 16 * 16
    Gd = torch.full((B, p.m), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
    p.eval_batch_device(Xd, Gd, Vd)
    counts = np.full(B, -1, dtype=np.int32)
    p.pattern_outside_batch(Xd, counts)
    torch.cuda.synchronize()
    G, V = Gd.cpu().numpy(), Vd.cpu().numpy()[:, :p.nnz]
    for b in range(B):
        d = type(desc).from_buffer_copy(desc)   # the shared description stays untouched
        d.terrain = terrains[b]
        o = Oracle(d)
        v_ref, outside = frozen_reference(o, r, c, X[b])
        assert counts[b] == outside, f"{name} problem {b}: {counts[b]} != {outside}"
        assert_close(o.eval_g(X[b]), G[b], r, v_ref, V[b], o.m, f"{name} gap batch {b}", cols_ref=c, floor_cols=residue_cols(d, o.n))
    assert np.isnan(Vd.cpu().numpy()[:, p.nnz:]).all()


def test_bench_workload_full_size(monkeypatch):
    """The bench's workload at its full size (B = 4096 randomised ANYmal problems, bench.make_batch):
    a seeded sample of problems against the oracle; every problem bit-identical between the default
    launch arrangement and per-class launches and between two evaluations (idempotence); no NaN, and
    the padding of the leading dimensions untouched."""
    import torch
    import bench
    from towr2025_amd import formulation as F
    B = 4096
    desc = F.anymal_trot().to_desc()
    p = TowrGpuProblem(desc)
    monkeypatch.setenv("TOWR_GPU_FUSE", "none")
    q = TowrGpuProblem(desc)
    Xh, terrains = bench.make_batch(p, B, first_id=0)
    p.set_batch_terrain(terrains)
    q.set_batch_terrain(terrains)
    dev = torch.device("cuda:0")
    ldg, ldv = (p.m + 15) // 16 * 16, (p.nnz + 15) // 16 * 16
    X = torch.from_numpy(np.ascontiguousarray(Xh[1])).to(dev)
    outs = []
    for prob in (p, p, q):
        G = torch.full((B, ldg), np.nan, dtype=torch.float64, device=dev)
        V = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
        prob.eval_batch_device(X, G, V)
        torch.cuda.synchronize()
        outs.append((G.cpu().numpy(), V.cpu().numpy()))
    (G, V), (G2, V2), (G3, V3) = outs
    assert np.isnan(G[:, p.m:]).all() and np.isnan(V[:, p.nnz:]).all()
    G, V = G[:, :p.m], V[:, :p.nnz]
    assert np.isfinite(G).all() and np.isfinite(V).all()
    np.testing.assert_array_equal(G2[:, :p.m], G)
    np.testing.assert_array_equal(V2[:, :p.nnz], V)
    np.testing.assert_array_equal(G3[:, :p.m], G)
    np.testing.assert_array_equal(V3[:, :p.nnz], V)
    rng = np.random.default_rng(4096)
    for b in sorted(rng.choice(B, 12, replace=False)):
        d = F.anymal_trot().to_desc()
        d.terrain = terrains[b]
        o = Oracle(d)
        r, _, v_ref = o.eval_jac(Xh[1, b])
        assert_close(o.eval_g(Xh[1, b]), G[b], r, v_ref, V[b], o.m, f"bench problem {b}")


def _batch_vs_single(base_f, name, B=64, optimize_timings=False):
    """B randomised problems of one layout (bench.make_batch: start/goal, per-problem Flat/Stairs terrain,
    x = x0 + seeded noise, durations +-3 % with phase-duration optimisation) through the device batch
    entry point with padded leading dimensions and NaN-prefilled outputs:
      * every problem bit-identical to its own B = 1 evaluation (a handle whose base terrain is the
        problem's, towr_gpu_eval_g_jac);
      * a seeded sample against the oracle (BASELINE.md's gate);
      * the padding of G and V still NaN (nothing written past m / nnz)."""
    import torch
    import bench
    desc = base_f.to_desc()
    p = TowrGpuProblem(desc)
    Xh, terrains = bench.make_batch(p, B, first_id=9000, optimize_timings=optimize_timings)
    X = np.ascontiguousarray(Xh[0])
    p.set_batch_terrain(terrains)
    dev = torch.device("cuda:0")
    ldx, ldg, ldv = p.n + 7, p.m + 9, p.nnz + 13          # deliberately unaligned leading dimensions
    Xd = torch.zeros((B, ldx), dtype=torch.float64, device=dev)
    Xd[:, :p.n] = torch.from_numpy(X).to(dev)
    Gd = torch.full((B, ldg), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
    p.eval_batch_device(Xd, Gd, Vd)
    torch.cuda.synchronize()
    G, V = Gd.cpu().numpy(), Vd.cpu().numpy()
    assert np.isnan(G[:, p.m:]).all() and np.isnan(V[:, p.nnz:]).all(), "write past m / nnz"
    G, V = G[:, :p.m], V[:, :p.nnz]
    assert np.isfinite(G).all() and np.isfinite(V).all(), "unwritten or non-finite outputs"
    r, c = p.jac_structure()
    sample = set(np.random.default_rng(B).choice(B, 6, replace=False).tolist())
    worst = 0.0
    for b in range(B):
        d = base_f.to_desc()
        d.terrain = terrains[b]
        q = TowrGpuProblem(d)
        g1, v1 = q.eval_g_jac(X[b])
        np.testing.assert_array_equal(G[b], g1, err_msg=f"{name} problem {b}: g differs from its B = 1 evaluation")
        np.testing.assert_array_equal(V[b], v1, err_msg=f"{name} problem {b}: J differs from its B = 1 evaluation")
        if b in sample:
            o = Oracle(d)
            rr, cc, v_ref = o.eval_jac(X[b])
            np.testing.assert_array_equal(rr, r)
            np.testing.assert_array_equal(cc, c)
            st = assert_close(o.eval_g(X[b]), G[b], r, v_ref, V[b], o.m, f"{name} problem {b}", cols_ref=c,
                              floor_cols=residue_cols(d, o.n))
            worst = max(worst, st["max_rel"])
        q.close()
    print(f"{name}: B = {B}, every problem bit-identical to B = 1; sample max relative error {worst:.3e}")


def test_batch_device_gait_optimization():
    """BASELINE configs[3]'s formulation (phase-duration optimisation: GAIT kernels, direct HBM
    emission into per-wave zero-filled rows) as a randomised device batch."""
    _batch_vs_single(F.anymal_trot(optimize_timings=True), "anymal_gaitopt_batch", B=64, optimize_timings=True)


def test_batch_device_gait_two_chains(monkeypatch):
    """The phase-duration path at B >= kSplitBatch (64) runs two chains (FDISC records + compose on the
    high-priority side stream 0, RangeOfMotion / Dynamic records + composes on the caller's stream), below it one
    serial chain (towr_gpu.hip launch_stream_path). B = 601 (odd: a compose block's problem pair is ragged) against the same problems
    as batches of 37 and 1 (37 < 64: the serial chain): bit-identical, nothing written past m / nnz, a
    sample against the oracle."""
    import torch
    import bench
    f = F.anymal_trot(optimize_timings=True)
    desc = f.to_desc()
    p = TowrGpuProblem(desc)
    B = 601
    Xh, terrains = bench.make_batch(p, B, first_id=7100, optimize_timings=True)
    X = np.ascontiguousarray(Xh[0])
    dev = torch.device("cuda:0")
    ldg, ldv = p.m + 3, p.nnz + 5
    Xd = torch.from_numpy(X).to(dev)
    Gd = torch.full((B, ldg), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
    p.set_batch_terrain(terrains)
    p.eval_batch_device(Xd, Gd, Vd)
    torch.cuda.synchronize()
    G, V = Gd.cpu().numpy(), Vd.cpu().numpy()
    assert np.isnan(G[:, p.m:]).all() and np.isnan(V[:, p.nnz:]).all(), "write past m / nnz"
    for s, e in [(k, min(B, k + 37)) for k in range(0, B, 37)] + [(300, 301)]:
        g = torch.full((e - s, p.m), np.nan, dtype=torch.float64, device=dev)
        v = torch.full((e - s, p.nnz), np.nan, dtype=torch.float64, device=dev)
        p.set_batch_terrain(terrains[s:e])
        p.eval_batch_device(Xd[s:e].contiguous(), g, v)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(G[s:e, :p.m], g.cpu().numpy(), err_msg=f"g of problems [{s}, {e})")
        np.testing.assert_array_equal(V[s:e, :p.nnz], v.cpu().numpy(), err_msg=f"J of problems [{s}, {e})")
    # one launch stream (TOWR_GPU_STREAMS=1, read at handle creation): the two chains one after the other
    for var, val in (("TOWR_GPU_STREAMS", "1"),):
        monkeypatch.setenv(var, val)
        q = TowrGpuProblem(desc)
        monkeypatch.delenv(var)
        q.set_batch_terrain(terrains)
        g1 = torch.full((B, ldg), np.nan, dtype=torch.float64, device=dev)
        v1 = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
        q.eval_batch_device(Xd, g1, v1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(g1.cpu().numpy(), G, err_msg=f"g: {var}={val} vs the default")
        np.testing.assert_array_equal(v1.cpu().numpy(), V, err_msg=f"J: {var}={val} vs the default")
        q.close()
    r, c = p.jac_structure()
    for b in (0, 255, 256, 600):
        d = f.to_desc()
        d.terrain = terrains[b]
        o = Oracle(d)
        _, _, v_ref = o.eval_jac(X[b])
        assert_close(o.eval_g(X[b]), G[b, :p.m], r, v_ref, V[b, :p.nnz], o.m, f"gait chunk problem {b}", cols_ref=c,
                     floor_cols=residue_cols(d, o.n))


@pytest.mark.parametrize("streams", [None, "1", "2"])
def test_batch_device_gait_torque(monkeypatch, streams):
    """ANYmal phase-duration optimisation + TorqueConstraintDiscretized as a randomised B = 64 device batch, every
    problem bit-identical to its B = 1 (single-chain) evaluation, on each big-batch launch arrangement of
    launch_stream_path (TOWR_GPU_STREAMS, read at handle creation):
      * default (two side streams): TQDISC records + compose as a third chain (`tq3`);
      * "2" (one side stream): the TQDISC records in the FDISC record launch (towr_gait_frec_kernel<5>) and its
        compose blocks in the FDISC compose launch (mask 17) on side stream 0 (`tqf`);
      * "1" (no side stream): the same chains one after the other on the caller's stream."""
    if streams is None:
        monkeypatch.delenv("TOWR_GPU_STREAMS", raising=False)
    else:
        monkeypatch.setenv("TOWR_GPU_STREAMS", streams)
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True)
    f.params_.constraints_.append(F.Parameters.Torque)
    _batch_vs_single(f, f"anymal_gait_torque_batch streams={streams}", B=64, optimize_timings=True)


@pytest.mark.parametrize("streams", [None, "1"])
def test_batch_device_rotvec(monkeypatch, streams):
    """RotVecConverter base orientation (ROTVEC kernels) as a randomised device batch, every problem bit-identical to
    its B = 1 evaluation: by default the coefficient pre-pass, Dynamic and the small kinds on side stream 0 beside
    RangeOfMotion and FDISC; TOWR_GPU_STREAMS=1 (read at handle creation): every launch on the caller's stream."""
    if streams is None:
        monkeypatch.delenv("TOWR_GPU_STREAMS", raising=False)
    else:
        monkeypatch.setenv("TOWR_GPU_STREAMS", streams)
    f = F.anymal_trot()
    f.params_.angular_rep_ = 1
    _batch_vs_single(f, f"anymal_rotvec_batch streams={streams}", B=64)


def test_batch_terrain_count_must_match():
    """Per-problem terrains apply to batch entry points only, and only with exactly B problems;
    single-problem entry points keep the description's terrain (include/towr_gpu.h)."""
    import torch
    from towr2025_amd.problem import TowrGpuError
    desc = F.anymal_trot().to_desc()
    p = TowrGpuProblem(desc)
    o = Oracle(desc)
    x = _perturb(o.initial_x(), 5)
    ter = [F.HeightMap.Flat(0.2).to_c() for _ in range(4)]
    p.set_batch_terrain(ter)
    dev = torch.device("cuda:0")
    X = torch.from_numpy(np.stack([x] * 3)).to(dev)
    G = torch.zeros((3, p.m), dtype=torch.float64, device=dev)
    V = torch.zeros((3, p.nnz), dtype=torch.float64, device=dev)
    with pytest.raises(TowrGpuError, match="batch terrains are set for 4"):
        p.eval_batch_device(X, G, V)
    with pytest.raises(TowrGpuError, match="batch terrains are set for 4"):
        p.eval_batch(np.stack([x] * 3))
    g, v = p.eval_g_jac(x)   # single problem: the description's (flat, h = 0) terrain
    r, _, v_ref = o.eval_jac(x)
    assert_close(o.eval_g(x), g, r, v_ref, v, o.m, "single call with batch terrains set")
    p.set_batch_terrain([])
    p.eval_batch_device(X, G, V)   # cleared: the description's terrain again
    torch.cuda.synchronize()
    np.testing.assert_array_equal(G.cpu().numpy()[1], g)


def test_host_batch_chunks_and_registered_buffers():
    """towr_gpu_eval_batch over several output chunks (kernels of chunk i overlap the D2H of chunk
    i - 1, per-problem terrains offset per chunk), through the pinned staging and in place into
    registered G / V, and the B = 1 host calls with registered g / values: all bit-identical to the
    device batch of the same problems."""
    import torch
    import bench
    desc = F.anymal_trot().to_desc()
    p = TowrGpuProblem(desc)
    B = 600                                   # ~64 MB of output per chunk: 3 chunks
    Xh, terrains = bench.make_batch(p, B, first_id=123)
    X = np.ascontiguousarray(Xh[2])
    p.set_batch_terrain(terrains)
    dev = torch.device("cuda:0")
    Gd = torch.zeros((B, p.m), dtype=torch.float64, device=dev)
    Vd = torch.zeros((B, p.nnz), dtype=torch.float64, device=dev)
    p.eval_batch_device(torch.from_numpy(X).to(dev), Gd, Vd)
    torch.cuda.synchronize()
    G_ref, V_ref = Gd.cpu().numpy(), Vd.cpu().numpy()
    G1, V1 = p.eval_batch(X)                                   # staged
    np.testing.assert_array_equal(G1, G_ref)
    np.testing.assert_array_equal(V1, V_ref)
    G2, V2 = np.full((B, p.m), np.nan), np.full((B, p.nnz), np.nan)
    p.register_host(G2)
    p.register_host(V2)
    p.eval_batch(X, G2, V2)                                    # in place
    np.testing.assert_array_equal(G2, G_ref)
    np.testing.assert_array_equal(V2, V_ref)
    p.unregister_host(G2)
    p.unregister_host(V2)
    # B = 1 host calls (one launch of every class) with registered outputs vs staged
    q = TowrGpuProblem(desc)
    o = Oracle(desc)
    xs = [_perturb(o.initial_x(), 31 + k) for k in range(3)]
    staged = [q.eval_g_jac(x) for x in xs]
    for k, x in enumerate(xs):   # the zero-copy single launch vs the device batch's launches
        Xd1 = torch.from_numpy(x.reshape(1, -1).copy()).to(dev)
        Gd1 = torch.zeros((1, q.m), dtype=torch.float64, device=dev)
        Vd1 = torch.zeros((1, q.nnz), dtype=torch.float64, device=dev)
        q.eval_batch_device(Xd1, Gd1, Vd1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(staged[k][0], Gd1.cpu().numpy()[0])
        np.testing.assert_array_equal(staged[k][1], Vd1.cpu().numpy()[0])
    g, v = np.full(q.m, np.nan), np.full(q.nnz, np.nan)
    q.register_host(g)
    q.register_host(v)
    xr = np.zeros(q.n)
    q.register_host(xr)
    for rep in range(2):   # alternating x: every call's zero-copy outputs are that call's, none stale
        for k, x in enumerate(xs):
            if rep:
                xr[:] = x                     # x from registered memory too
                q.eval_g_jac_into(xr, g, v)
            else:
                q.eval_g_jac_into(np.ascontiguousarray(x), g, v)
            np.testing.assert_array_equal(g, staged[k][0])
            np.testing.assert_array_equal(v, staged[k][1])
    r, c, v_ref = o.eval_jac(xs[2])
    assert_close(o.eval_g(xs[2]), g, r, v_ref, v, o.m, "registered single call")
    q.close()   # destroy unregisters


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["anymal_trot_2p4s", "anymal_trot_rotvec", "anymal_stairs_gaitopt", "anymal_gait_torque"])
def test_batch_device_g_or_jac_only(name):
    """g alone and the Jacobian alone over a batch of 80 (B >= 64: Dynamic and the small kinds beside the fused
    launch for the Euler layout; for RotVec the coefficient pre-pass runs without the Jacobian too, for the base
    terms the g rows need): each equals the full call's output bit for bit and leaves the other output untouched."""
    import torch
    desc = CONFIGS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc)
    B = 80
    X = np.stack([_perturb(o.initial_x(), 900 + b) for b in range(B)])
    ldv = (p.nnz + 15) // 16 * 16
    dev = torch.device("cuda:0")
    Xd = torch.from_numpy(X).to(dev)

    def run(want_g, want_jac):
        Gd = torch.full((B, p.m), np.nan, dtype=torch.float64, device=dev)
        Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
        p.eval_batch_device(Xd, Gd, Vd, want_g=want_g, want_jac=want_jac)
        torch.cuda.synchronize()
        return Gd.cpu().numpy(), Vd.cpu().numpy()[:, :p.nnz]

    G, V = run(True, True)
    fc = residue_cols(desc, o.n)
    for b in (0, B - 1):
        r, c, v_ref = o.eval_jac(X[b])
        assert_close(o.eval_g(X[b]), G[b], r, v_ref, V[b], o.m, f"{name} full batch {b}", cols_ref=c, floor_cols=fc)
    Gg, Vg = run(True, False)
    assert np.array_equal(Gg, G) and np.isnan(Vg).all()
    Gj, Vj = run(False, True)
    assert np.array_equal(Vj, V) and np.isnan(Gj).all()
    # the output that is not wanted may be NULL
    Gd = torch.full((B, p.m), np.nan, dtype=torch.float64, device=dev)
    Vd = torch.full((B, ldv), np.nan, dtype=torch.float64, device=dev)
    p.eval_batch_device(Xd, Gd, None, want_g=True, want_jac=False)
    p.eval_batch_device(Xd, None, Vd, want_g=False, want_jac=True)
    torch.cuda.synchronize()
    assert np.array_equal(Gd.cpu().numpy(), G) and np.array_equal(Vd.cpu().numpy()[:, :p.nnz], V)


@pytest.mark.parametrize("name", ["anymal_trot_2p4s", "anymal_stairs_gaitopt"])
def test_keep_jacobian_pair(name):
    """IPOPT's pair through towr_gpu_eval_g_keep_jac + towr_gpu_eval_jac_values_kept: bit-identical to the one-call
    evaluation at the same x; at another x (or after another host-pointer evaluation dropped the kept values) the
    values are evaluated afresh, never served from the kept x."""
    desc = CONFIGS[name]
    o = Oracle(desc)
    p = TowrGpuProblem(desc, device=0)
    xa, xb = _perturb(o.initial_x(), 61), _perturb(o.initial_x(), 62)
    ga, va = p.eval_g_jac(xa)
    gb, vb = p.eval_g_jac(xb)
    np.testing.assert_array_equal(p.eval_g_keep_jac(xa), ga)
    np.testing.assert_array_equal(p.eval_jac_values_kept(xa), va)
    np.testing.assert_array_equal(p.eval_jac_values_kept(xa), va)   # served again from the kept values
    np.testing.assert_array_equal(p.eval_jac_values_kept(xb), vb)   # another x: evaluated
    np.testing.assert_array_equal(p.eval_g_keep_jac(xb), gb)
    p.eval_g(xa)                                                       # any other evaluation drops the kept values
    np.testing.assert_array_equal(p.eval_jac_values_kept(xb), vb)
    xc = xb.copy()
    xc[7] = np.nextafter(xc[7], np.inf)                               # one ulp away: not the kept x
    np.testing.assert_array_equal(p.eval_g_keep_jac(xb), gb)
    np.testing.assert_array_equal(p.eval_jac_values_kept(xc), p.eval_jac_values(xc))
