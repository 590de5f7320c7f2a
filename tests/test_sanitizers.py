"""AddressSanitizer + UndefinedBehaviorSanitizer runs of the CPU-side code (VERDICT r1 weak item 12,
SURVEY §5): the oracle (oracle/sancheck.c) and the engine's host code — the layout builder and the host
instantiation of engine_math.h through the emulation (tests/host_emu/sancheck.cc, built host-only) —
over every parity configuration. GPU sanitizers are not available on this pool; these are host-only."""
import os
import struct
import subprocess

import numpy as np
import pytest

from tests.configs import config_descs, cost_descs, ext_cases
from towr2025_amd import _capi as capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "build", "sancheck")
EMU = os.path.join(ROOT, "tests", "host_emu", "build", "sancheck")


def _cases():
    out = {k: (v, []) for k, v in config_descs().items()}
    out.update({k: (v, []) for k, v in cost_descs().items()})
    out.update(ext_cases())
    return out


CASES = _cases()


@pytest.fixture(scope="module")
def binaries():
    for d, exe in ((os.path.join(ROOT, "oracle"), ORACLE), (os.path.join(ROOT, "tests", "host_emu"), EMU)):
        subprocess.check_call(["make", "-s", "-C", d, "sanitize"])
        assert os.path.exists(exe)
    return ORACLE, EMU


def _write(path, desc, data):
    with open(path, "wb") as f:
        f.write(bytes(desc))
        f.write(struct.pack("<i", len(data)))
        for kind, index, arr in data:
            a = np.ascontiguousarray(arr, dtype=np.float64).ravel()
            f.write(struct.pack("<iiq", kind, index, a.size))
            f.write(a.tobytes())


@pytest.mark.parametrize("name", sorted(CASES))
def test_sanitized_host_code(binaries, tmp_path, name):
    desc, data = CASES[name]
    p = str(tmp_path / "problem.bin")
    _write(p, desc, data)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    for exe in binaries:
        r = subprocess.run([exe, p], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0 and r.stdout.startswith("ok"), f"{os.path.basename(exe)}: rc {r.returncode}\n{r.stderr[-3000:]}"
        assert "runtime error" not in r.stderr and "Sanitizer" not in r.stderr, r.stderr[-3000:]
