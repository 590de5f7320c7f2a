"""Self-test of the parity gate (tests/parity.py): check_values / assert_close / assert_cost_close must flag a NaN
or an infinity in g, in the Jacobian values and in the objective gradient, on either side, and still accept
results inside the tolerance. Rounds 1-3 wrote the check as `err > tol`, which a NaN never satisfies; an
infinity facing a finite value has an infinite tolerance (REL * inf), so `err <= tol` alone passes it."""
import numpy as np
import pytest

from tests.parity import REL, assert_close, assert_cost_close, check_values

BAD = [np.nan, np.inf, -np.inf]


def _case(rng):
    m, n_per_row = 6, 4
    rows = np.repeat(np.arange(m), n_per_row)
    v_ref = rng.standard_normal(len(rows)) * 10.0
    g_ref = rng.standard_normal(m)
    return g_ref, rows, v_ref, m


def test_gate_accepts_values_within_tolerance():
    g_ref, rows, v_ref, m = _case(np.random.default_rng(0))
    g = g_ref * (1 + 0.1 * REL)
    v = v_ref * (1 - 0.1 * REL)
    bad_g, bad_v, _ = check_values(g_ref, g, rows, v_ref, v, m)
    assert len(bad_g) == 0 and len(bad_v) == 0
    assert_close(g_ref, g, rows, v_ref, v, m, "within tolerance")
    assert_cost_close(3.0, 3.0 * (1 + 0.1 * REL), g_ref, g, "cost within tolerance")


def test_gate_rejects_values_outside_tolerance():
    g_ref, rows, v_ref, m = _case(np.random.default_rng(1))
    v = v_ref.copy()
    v[5] *= 1 + 100 * REL
    _, bad_v, _ = check_values(g_ref, g_ref.copy(), rows, v_ref, v, m)
    assert list(bad_v) == [5]


@pytest.mark.parametrize("bad", BAD)
@pytest.mark.parametrize("side", ["engine", "reference"])
def test_gate_rejects_non_finite_g_and_jacobian(bad, side):
    g_ref, rows, v_ref, m = _case(np.random.default_rng(2))
    g, v = g_ref.copy(), v_ref.copy()
    (g if side == "engine" else g_ref)[3] = bad
    (v if side == "engine" else v_ref)[7] = bad
    bad_g, bad_v, _ = check_values(g_ref, g, rows, v_ref, v, m)
    assert list(bad_g) == [3], f"g: {bad} on the {side} side not flagged"
    assert 7 in bad_v, f"J: {bad} on the {side} side not flagged"
    with pytest.raises(AssertionError):
        assert_close(g_ref, g, rows, v_ref, v, m, "non-finite")


@pytest.mark.parametrize("bad", BAD)
def test_gate_rejects_non_finite_objective_and_gradient(bad):
    rng = np.random.default_rng(3)
    grad_ref = rng.standard_normal(50)
    grad = grad_ref.copy()
    grad[11] = bad
    with pytest.raises(AssertionError, match="gradient"):
        assert_cost_close(2.5, 2.5, grad_ref, grad, "gradient")
    with pytest.raises(AssertionError, match="f ref"):
        assert_cost_close(2.5, bad, grad_ref, grad_ref.copy(), "objective")
    with pytest.raises(AssertionError):
        assert_cost_close(bad, 2.5, grad_ref, grad_ref.copy(), "objective, reference side")


def test_gate_identical_infinities_match():
    """An infinity on both sides (the same one) is a match: the gate compares results, it does not judge them."""
    g_ref, rows, v_ref, m = _case(np.random.default_rng(4))
    g_ref[0] = np.inf
    v_ref[0] = -np.inf
    bad_g, bad_v, _ = check_values(g_ref, g_ref.copy(), rows, v_ref, v_ref.copy(), m)
    assert len(bad_g) == 0 and len(bad_v) == 0
