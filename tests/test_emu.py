"""Values of the shared item math (towr2025_amd/csrc/engine_math.h) vs the oracle, through the
test-only host emulation of the kernel's item loop (tests/host_emu). Catches math and
candidate-order errors on CPU; the GPU parity tests (test_gpu_parity.py) then check the device."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle.oracle import Oracle
from tests.configs import config_descs
from tests.parity import assert_close, residue_cols
from tests.gap_frozen import frozen_reference, is_gap
from towr2025_amd import _capi as capi

HERE = os.path.dirname(os.path.abspath(__file__))
CONFIGS = config_descs()
D = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def emu():
    lib = os.path.join(HERE, "host_emu", "build", "libemu.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "host_emu")])
    L = C.CDLL(lib)
    L.emu_eval.argtypes = [C.POINTER(capi.ProblemDesc), D, D, D, C.c_char_p, C.c_int]
    return L


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_emulated_values_match_oracle(emu, name):
    desc = CONFIGS[name]
    o = Oracle(desc)
    x0 = o.initial_x()
    r0, c0, _ = o.eval_jac(x0)
    for seed in (0, 1, 2):
        x = x0 if seed == 0 else x0 + 0.05 * np.random.default_rng(seed).standard_normal(o.n)
        r, c, v = o.eval_jac(x)
        if len(r) != len(r0) or not (np.array_equal(r, r0) and np.array_equal(c, c0)):
            # only curved terrain moves the reference's pattern: compare on the frozen (x0) pattern
            assert is_gap(desc), f"{name} seed {seed}: pattern moved on a non-Gap terrain"
            v, _ = frozen_reference(o, r0, c0, x)
            r, c = r0, c0
        g, ve = np.zeros(o.m), np.zeros(len(v))
        err = C.create_string_buffer(256)
        assert emu.emu_eval(C.byref(desc), x.ctypes.data_as(D), g.ctypes.data_as(D), ve.ctypes.data_as(D), err, 256) == 0, err.value
        assert_close(o.eval_g(x), g, r, v, ve, o.m, f"{name} seed {seed}", cols_ref=c, floor_cols=residue_cols(desc, o.n))


@pytest.mark.parametrize("name", ["anymal_trot_2p4s", "biped_walk_2s"])
def test_small_kinds_stage_part_of_x(emu, name):
    """The small-kind blocks stage only the x spans their items read (Layout::misc_xspan, kernel_common.h
    stage_x_spans); test_emulated_values_match_oracle runs those items with every other column NaN. With fixed
    phase durations the bench's ANYmal problem stages well under all of x (the force nodes are never read)."""
    if name not in CONFIGS:
        pytest.skip(f"{name} not a parity config")
    desc = CONFIGS[name]
    out = (C.c_int64 * 3)()
    assert emu.emu_misc_xspan(C.byref(desc), out) == 0
    spans, units, total = out[0], out[1], out[2]
    assert 0 < spans and 0 < units < 0.8 * total, (spans, units, total)
