"""C++ host side (towr2025_amd/host): the NlpFormulation mirror builds byte-identical problem
descriptions to the Python mirror, and the Engine / NlpCallbacks (IPOPT TNLP-shaped eval_f /
eval_grad_f / eval_g / eval_jac_g) driver reproduces the oracle's sizes, x0 and pattern (CPU, layout-only handle) and its
values on the GPU. The driver runs as a child process (tests/.. towr_host_check)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from towr2025_amd import _capi as capi
from towr2025_amd import formulation as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "towr2025_amd", "host")
EXE = os.path.join(HOST, "build", "towr_host_check")
def _biped_next():
    from tests.configs import _with_next_tier
    return _with_next_tier(F.biped_walk())


def _anymal_costs():
    from tests.configs import _with_costs
    return _with_costs(F.anymal_trot()).to_desc()


def _anymal_rotvec():
    f = F.anymal_trot()
    f.params_.angular_rep_ = 1
    return f.to_desc()


def _anymal_gait():
    return F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True).to_desc()


CFGS = {"anymal_rotvec": _anymal_rotvec, "anymal_gait": _anymal_gait, "anymal": lambda: F.anymal_trot().to_desc(), "biped": lambda: F.biped_walk().to_desc(),
        "hopper": lambda: F.monoped_hopper().to_desc(), "biped_next": _biped_next, "anymal_costs": _anymal_costs}


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(os.path.join(ROOT, "towr2025_amd", "lib", "libtowr_gpu.so")):
        pytest.skip("libtowr_gpu.so not built")
    subprocess.check_call(["make", "-s", "-C", HOST])
    return EXE


def _run(exe, cfg, out, device):
    subprocess.check_call([exe, cfg, str(out), str(device)], stdout=subprocess.DEVNULL)
    raw = open(out, "rb").read()
    ds = C.sizeof(capi.ProblemDesc)
    desc = raw[:ds]
    n, m = np.frombuffer(raw, np.int32, 2, ds)
    nnz = int(np.frombuffer(raw, np.int64, 1, ds + 8)[0])
    off = ds + 16
    x0 = np.frombuffer(raw, np.float64, n, off); off += 8 * n
    r = np.frombuffer(raw, np.int32, nnz, off); off += 4 * nnz
    c = np.frombuffer(raw, np.int32, nnz, off); off += 4 * nnz
    out = dict(desc=desc, n=int(n), m=int(m), nnz=nnz, x0=x0, iRow=r, jCol=c)
    if device >= 0:
        out["g"] = np.frombuffer(raw, np.float64, m, off); off += 8 * m
        out["values"] = np.frombuffer(raw, np.float64, nnz, off); off += 8 * nnz
        out["f"] = float(np.frombuffer(raw, np.float64, 1, off)[0]); off += 8
        out["grad"] = np.frombuffer(raw, np.float64, n, off)
    return out


@pytest.mark.parametrize("cfg", sorted(CFGS))
def test_cpp_layout_matches_python_and_oracle(exe, tmp_path, cfg):
    from oracle.oracle import Oracle
    res = _run(exe, cfg, tmp_path / "o.bin", -1)
    desc = CFGS[cfg]()
    assert res["desc"] == bytes(desc), "C++ and Python NlpFormulation mirrors build different descriptions"
    o = Oracle(desc)
    assert (res["n"], res["m"]) == (o.n, o.m)
    np.testing.assert_array_equal(res["x0"], o.initial_x())
    r, c, _ = o.eval_jac(o.initial_x())
    np.testing.assert_array_equal(res["iRow"], r)
    np.testing.assert_array_equal(res["jCol"], c)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", sorted(CFGS))
def test_cpp_callbacks_on_gpu_match_oracle(exe, tmp_path, cfg):
    from oracle.oracle import Oracle
    from tests.parity import assert_close, assert_cost_close, residue_cols
    res = _run(exe, cfg, tmp_path / "o.bin", 0)
    desc = CFGS[cfg]()
    o = Oracle(desc)
    x0 = o.initial_x()
    r, c, v = o.eval_jac(x0)
    # (phase-duration optimisation: the schedule columns' column-scaled floor, tests/parity.py)
    assert_close(o.eval_g(x0), res["g"], r, v, res["values"], o.m, f"C++ host {cfg}", cols_ref=c, floor_cols=residue_cols(desc, o.n))
    assert_cost_close(o.eval_f(x0), res["f"], o.eval_grad_f(x0), res["grad"], f"C++ host {cfg} costs")
    # SaveTrajectoryToCSV text from the C++ host (6 decimals) against the oracle's samples
    from towr2025_amd import trajectory as T
    text = open(str(tmp_path / "o.bin") + ".csv").read().splitlines()
    n_ee = CFGS[cfg]().robot.n_ee
    assert text[0] == ",".join(T.csv_header(n_ee))
    got = np.array([[float(v) for v in line.split(",")] for line in text[1:]])
    ref = o.sample_trajectory(x0, 0.01)
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=5e-7 + 1e-12 * np.abs(ref).max())


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["anymal", "anymal_gait"])
def test_cpp_callbacks_zero_copy_jacobian(exe, cfg):
    """NlpCallbacks::eval_jac_g writes the Jacobian straight into IPOPT's (registered) values array and eval_g
    evaluates g alone: bit-identical to the engine's own evaluation with IPOPT's array stable across calls (one
    registration), with the Jacobian asked for before g, with an array that moves between calls, and after
    finalize_solution (towr_host_check --zerocopy). Prints the per-iteration timings of the callbacks against the
    round-4 cached path (fused evaluation + nnz-value copy)."""
    out = subprocess.check_output([exe, cfg, "--zerocopy", "0", "100"], text=True)
    print(out.strip())
    assert out.startswith("zerocopy ok")
