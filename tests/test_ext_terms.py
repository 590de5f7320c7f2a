"""LinearEqualityConstraint, the fork's BaseHeightCost and SoftConstraint (VERDICT r1 "missing" 1-2).

CPU (no GPU):
  * the oracle restatements against independent forms of the same quantity:
      - LinearEquality: g = M x_set and J = the nonzeros of M (linear_constraint.cc:47-76);
      - SoftConstraint: its cost / gradient against 0.5 |g - b|^2 and J^T (g - b) built from a HARD copy
        of the wrapped set (soft_constraint.cc:52-69), and central differences;
      - BaseHeightCost: central differences on the base-linear columns, and the reference's partial
        gradient elsewhere (base_height_cost.cc:70-86 differentiates only p_z of the base);
  * engine_math.h through the host emulation against the oracle (LinearEquality rows, BaseHeightCost);
  * sizes, pattern and description validation on layout-only handles.
GPU (-m gpu): the HIP path through the C-ABI against the oracle, single problem and batched.
Parity is "pinned by the oracle and FD only": the reference's tests hold no fixtures for these terms
(SURVEY §8c)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle.oracle import Oracle
from tests.configs import ext_cases
from tests.parity import assert_close, assert_cost_close, residue_cols
from towr2025_amd import TowrGpuProblem
from towr2025_amd import _capi as capi
from towr2025_amd.problem import TowrGpuError

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ext_cases()
D = C.POINTER(C.c_double)


def _x(o, seed, scale=0.03):
    x = o.initial_x()
    if seed:
        x = x + scale * np.random.default_rng(seed).standard_normal(o.n)
    return x


def _fd_grad(o, x, cols, h_rel=1e-5):
    out = np.zeros(len(cols))
    for k, j in enumerate(cols):
        h = h_rel * max(1.0, abs(x[j]))
        xp, xm = x.copy(), x.copy()
        xp[j] += h
        xm[j] -= h
        out[k] = (o.eval_f(xp) - o.eval_f(xm)) / (2 * h)
    return out


def _hard_copy(desc, ci):
    """The description with constraint ci as the only (hard) constraint and no costs."""
    d = capi.ProblemDesc.from_buffer_copy(desc)
    d.constraints[0] = desc.constraints[ci]
    d.constraints[0].role = capi.ROLE_HARD
    d.n_constraints = 1
    d.n_costs = 0
    return d


# ------------------------------------------------------------------ oracle pins ----------------
@pytest.mark.parametrize("name", ["procedural_lineq", "anymal_gait_lineq"])
def test_oracle_linear_equality(name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    rows = o.constraint_rows()
    cols = o.varset_cols()
    x = _x(o, 3)
    g = o.eval_g(x)
    r, c, v = o.eval_jac(x)
    for kind, ci, M in data:
        assert kind == capi.DATA_LINEAR_M
        r0, nr = rows[ci]
        c0, nc = cols[desc.constraints[ci].ip[0]]
        assert M.shape == (nr, nc)
        np.testing.assert_allclose(g[r0:r0 + nr], M @ x[c0:c0 + nc], rtol=1e-13, atol=1e-13)
        sel = (r >= r0) & (r < r0 + nr)
        nzr, nzc = np.nonzero(M)   # M.sparseView(): the nonzeros, row-major
        assert np.array_equal(r[sel] - r0, nzr) and np.array_equal(c[sel] - c0, nzc)
        assert np.array_equal(v[sel], M[nzr, nzc])


def test_oracle_soft_constraint_against_hard_copy():
    for name in ("procedural_soft", "anymal_gait_soft"):
        desc, data = CASES[name]
        o = Oracle(desc, data)
        x = _x(o, 4, 0.01)
        f_ref, grad_ref = 0.0, np.zeros(o.n)
        mats = {i: M for (k, i, M) in data if k == capi.DATA_LINEAR_M}
        for (kind, ti, bnd) in data:
            if kind != capi.DATA_SOFT_BOUNDS:
                continue
            ci = desc.costs[ti].ip[0]
            hd = _hard_copy(desc, ci)
            hdata = [(capi.DATA_LINEAR_M, 0, mats[ci])] if ci in mats else []
            h = Oracle(hd, hdata)
            g = h.eval_g(x)
            rr, cc, vv = h.eval_jac(x)
            nr = len(g)
            b = (bnd[nr:] + bnd[:nr]) / 2.0
            f_ref += 0.5 * np.dot(g - b, g - b)
            np.add.at(grad_ref, cc, vv * (g - b)[rr])
        # plus the NodeCost of procedural_soft
        f_node = 0.0
        if name == "procedural_soft":
            od = capi.ProblemDesc.from_buffer_copy(desc)
            od.costs[0] = desc.costs[2]
            od.n_costs = 1
            on = Oracle(od, data)
            f_node = on.eval_f(x)
            grad_ref += on.eval_grad_f(x)
        assert abs(o.eval_f(x) - (f_ref + f_node)) <= 1e-10 * abs(f_ref + f_node)
        np.testing.assert_allclose(o.eval_grad_f(x), grad_ref, rtol=1e-9, atol=1e-9 * np.abs(grad_ref).max())
        # the soft-only sets are not rows of g
        hard = sum(1 for i in range(desc.n_constraints) if desc.constraints[i].role == capi.ROLE_HARD)
        assert sum(1 for (r0, nr) in o.constraint_rows() if r0 >= 0) == hard


def test_oracle_soft_gradient_matches_fd():
    desc, data = CASES["procedural_soft"]
    o = Oracle(desc, data)
    x = _x(o, 5, 0.01)
    cols = list(range(0, o.n, 3))
    fd = _fd_grad(o, x, cols)
    g = o.eval_grad_f(x)[cols]
    assert np.max(np.abs(fd - g) / np.maximum(1.0, np.abs(g))) < 1e-4


@pytest.mark.parametrize("name", ["biped_base_height_cost", "anymal_stairs_base_height_cost"])
def test_oracle_base_height_cost_fd_and_partial_gradient(name):
    """Base-linear columns: FD-consistent. Other columns: the reference differentiates only the base
    height (base_height_cost.cc:70-86), so the feet's contribution through the stance average is absent
    even though the objective depends on them."""
    desc, data = CASES[name]
    o = Oracle(desc, data)
    x = _x(o, 6, 0.01)
    cols = o.varset_cols()
    kinds = [desc.varsets[i].kind for i in range(desc.n_varsets)]
    c0, nb = cols[kinds.index(capi.VAR_BASE_LIN)]
    # only the base-height term (NodeCosts removed) for the partial-gradient check
    d1 = capi.ProblemDesc.from_buffer_copy(desc)
    d1.n_costs = 1
    assert desc.costs[0].kind == capi.COST_BASE_HEIGHT
    o1 = Oracle(d1, data)
    g1 = o1.eval_grad_f(x)
    bl = list(range(c0, c0 + nb))
    fd = _fd_grad(o1, x, bl, h_rel=1e-6)
    assert np.max(np.abs(fd - g1[bl]) / np.maximum(1.0, np.abs(g1[bl]))) < 1e-4
    others = [j for j in range(o.n) if not (c0 <= j < c0 + nb)]
    assert np.all(g1[others] == 0.0)
    cm, nm = cols[kinds.index(capi.VAR_EE_MOTION)]
    assert np.max(np.abs(_fd_grad(o1, x, list(range(cm, cm + nm)), h_rel=1e-6))) > 1e-6


def test_oracle_base_height_flight_uses_terrain():
    """ANYmal's flying trot has instants without stance feet: the target there is the terrain height
    under the base (base_height_cost.cc:117-121). Moving the terrain changes f only through them."""
    desc, data = CASES["anymal_stairs_base_height_cost"]
    o = Oracle(desc, data)
    x = o.initial_x()
    d2 = capi.ProblemDesc.from_buffer_copy(desc)
    d2.terrain.p[2] += 0.05   # first step height: the base crosses the stairs during flight phases
    o2 = Oracle(d2, data)
    assert o.eval_f(x) != o2.eval_f(x)


# ------------------------------------------------------------------ host emulation -------------
@pytest.fixture(scope="module")
def emu():
    lib = os.path.join(HERE, "host_emu", "build", "libemu.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "host_emu")])
    L = C.CDLL(lib)
    L.emu_eval_ex.argtypes = [C.POINTER(capi.ProblemDesc), C.c_int, C.POINTER(capi.SideData), D, D, D, C.c_char_p, C.c_int]
    L.emu_cost.argtypes = [C.POINTER(capi.ProblemDesc), D, D, D, C.c_char_p, C.c_int]
    return L


@pytest.mark.parametrize("name", ["procedural_lineq", "anymal_gait_lineq"])
def test_emulated_linear_equality_matches_oracle(emu, name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    arr, keep = capi.side_data(data)
    for seed in (0, 1):
        x = _x(o, seed)
        r, c, v_ref = o.eval_jac(x)
        g, v = np.zeros(o.m), np.zeros(len(v_ref))
        err = C.create_string_buffer(256)
        assert emu.emu_eval_ex(C.byref(desc), len(data), arr, x.ctypes.data_as(D), g.ctypes.data_as(D),
                               v.ctypes.data_as(D), err, 256) == 0, err.value
        assert_close(o.eval_g(x), g, r, v_ref, v, o.m, f"{name} seed {seed}", cols_ref=c,
                     floor_cols=residue_cols(desc, o.n, data))


@pytest.mark.parametrize("name", ["biped_base_height_cost", "biped_gait_base_height_cost", "anymal_stairs_base_height_cost"])
def test_emulated_base_height_cost_matches_oracle(emu, name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    for seed in (0, 2):
        x = _x(o, seed, 0.02)
        f, g = C.c_double(), np.zeros(o.n)
        err = C.create_string_buffer(256)
        assert emu.emu_cost(C.byref(desc), x.ctypes.data_as(D), C.byref(f), g.ctypes.data_as(D), err, 256) == 0, err.value
        assert_cost_close(o.eval_f(x), f.value, o.eval_grad_f(x), g, f"{name} seed {seed}")


# ------------------------------------------------------------------ layout-only handles ---------
@pytest.mark.parametrize("name", sorted(CASES))
def test_sizes_and_pattern_match_oracle(name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    p = TowrGpuProblem(desc, device=-1, data=data)
    assert (p.n, p.m) == (o.n, o.m)
    r, c, _ = o.eval_jac(o.initial_x())
    pr, pc = p.jac_structure()
    assert np.array_equal(pr, r) and np.array_equal(pc, c)


def _create_rc(desc, data):
    try:
        TowrGpuProblem(desc, device=-1, data=data)
        return 0
    except TowrGpuError as e:
        return str(e)


def test_side_data_validation():
    desc, data = CASES["procedural_lineq"]
    assert _create_rc(desc, data) == 0
    assert "matrix" in _create_rc(desc, data[:1])                                 # second matrix missing
    bad = [(k, i, M[:, :-1]) for (k, i, M) in data]
    assert "matrix" in _create_rc(desc, bad)                                      # wrong shape
    d2 = capi.ProblemDesc.from_buffer_copy(desc)
    d2.constraints[desc.n_constraints - 1].ip[0] = 99
    assert "LinearEquality" in _create_rc(d2, data)
    sdesc, sdata = CASES["procedural_soft"]
    assert _create_rc(sdesc, sdata) == 0
    assert "SoftConstraint" in _create_rc(sdesc, sdata[:1])                       # bounds of term 1 missing
    assert "SoftConstraint" in _create_rc(sdesc, [(k, i, b[:-2]) for (k, i, b) in sdata])
    d3 = capi.ProblemDesc.from_buffer_copy(sdesc)
    d3.costs[0].ip[0] = 60
    assert "SoftConstraint" in _create_rc(d3, sdata)
    d4 = capi.ProblemDesc.from_buffer_copy(sdesc)
    d4.constraints[0].role = 7
    assert "role" in _create_rc(d4, sdata)
    bdesc, _ = CASES["biped_base_height_cost"]
    d5 = capi.ProblemDesc.from_buffer_copy(bdesc)
    d5.costs[0].dt = 0.0
    assert "dt" in _create_rc(d5, [])


# ------------------------------------------------------------------ GPU parity ------------------
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["procedural_lineq", "anymal_gait_lineq"])
def test_gpu_linear_equality(name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    p = TowrGpuProblem(desc, device=0, data=data)
    fc = residue_cols(desc, o.n, data)
    for seed in (0, 1, 2):
        x = _x(o, seed)
        r, c, v_ref = o.eval_jac(x)
        pr, pc = p.jac_structure()
        assert np.array_equal(pr, r) and np.array_equal(pc, c)
        g, v = p.eval_g_jac(x)
        stats = assert_close(o.eval_g(x), g, r, v_ref, v, o.m, f"{name} seed {seed}", cols_ref=c, floor_cols=fc)
        print(name, seed, stats)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["biped_base_height_cost", "biped_gait_base_height_cost", "anymal_stairs_base_height_cost",
                                  "procedural_soft", "anymal_gait_soft"])
def test_gpu_cost_terms(name):
    desc, data = CASES[name]
    o = Oracle(desc, data)
    p = TowrGpuProblem(desc, device=0, data=data)
    for seed in (0, 1, 2):
        x = _x(o, seed, 0.02)
        assert_cost_close(o.eval_f(x), p.eval_f(x), o.eval_grad_f(x), p.eval_grad_f(x), f"{name} seed {seed}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["biped_base_height_cost", "procedural_soft", "anymal_gait_soft"])
def test_gpu_cost_batch(name):
    """B problems through eval_cost_batch_device (the soft child runs on the caller's stream): a sample
    against the oracle, every problem equal to its own single-problem evaluation up to the gradient's
    atomic summation order, and f-only calls equal to f of the gradient calls."""
    import torch
    desc, data = CASES[name]
    o = Oracle(desc, data)
    p = TowrGpuProblem(desc, device=0, data=data)
    B = 37
    rng = np.random.default_rng(9)
    X = np.stack([o.initial_x() + 0.02 * rng.standard_normal(o.n) for _ in range(B)])
    Xd = torch.zeros((B, p.n + 3), dtype=torch.float64, device="cuda")
    Xd[:, :p.n] = torch.from_numpy(X)
    F = torch.full((B,), float("nan"), dtype=torch.float64, device="cuda")
    G = torch.full((B, p.n + 5), float("nan"), dtype=torch.float64, device="cuda")
    p.eval_cost_batch_device(Xd, F, G)
    F0 = torch.full((B,), float("nan"), dtype=torch.float64, device="cuda")
    p.eval_cost_batch_device(Xd, F0)
    torch.cuda.synchronize()
    Fh, Gh, F0h = F.cpu().numpy(), G.cpu().numpy(), F0.cpu().numpy()
    assert np.all(np.isnan(Gh[:, p.n:]))
    assert np.array_equal(F0h, Fh)
    for b in (0, 17, B - 1):
        assert_cost_close(o.eval_f(X[b]), Fh[b], o.eval_grad_f(X[b]), Gh[b, :p.n], f"{name} problem {b}")
    for b in range(B):
        assert_cost_close(p.eval_f(X[b]), Fh[b], p.eval_grad_f(X[b]), Gh[b, :p.n], f"{name} problem {b} vs B=1")
