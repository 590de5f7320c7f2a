"""Shared parity helpers: the tolerance of BASELINE.md / SURVEY §8(d), written once.

values:  |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, rowscale, colscale)
where rowscale / colscale = max |J| over the reference row / column. The floor covers entries that
are exact zeros in exact arithmetic and come out as rounding residue of much larger terms:
Hermite basis functions that vanish at a polynomial end (the reference rounds to exactly 0.0,
fused multiply-adds give ~4e-16), and, with phase-duration optimisation, d pos / d duration of a
PhaseSpline at an instant where the spline is analytically flat (a zero force in swing: its
velocity is the ~1e-11 residue of ~1e5-sized Hermite terms). Such residue differs with any change
of operation order, the reference's own build included; the column scale bounds its size.
g:       |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, |J row| scale)
Pattern: bit-exact (same (row, col) list in the same order).
"""
import numpy as np

REL = 1e-9
ABS = 1e-12


def check_values(g_ref, g, rows_ref, v_ref, v, m, cols_ref=None):
    rs = np.zeros(m)
    np.maximum.at(rs, rows_ref, np.abs(v_ref))
    floor = ABS * np.maximum(1.0, rs)
    floor_v = floor[rows_ref]
    if cols_ref is not None:
        cs = np.zeros(int(cols_ref.max()) + 1 if len(cols_ref) else 1)
        np.maximum.at(cs, cols_ref, np.abs(v_ref))
        floor_v = np.maximum(floor_v, ABS * cs[cols_ref])
    tol_v = REL * np.maximum(np.abs(v_ref), np.abs(v)) + floor_v
    bad_v = np.flatnonzero(np.abs(v_ref - v) > tol_v)
    tol_g = REL * np.maximum(np.abs(g_ref), np.abs(g)) + floor
    bad_g = np.flatnonzero(np.abs(g_ref - g) > tol_g)
    return bad_g, bad_v


def assert_close(g_ref, g, rows_ref, v_ref, v, m, what="", cols_ref=None):
    bad_g, bad_v = check_values(g_ref, g, rows_ref, v_ref, v, m, cols_ref)
    msg = []
    if len(bad_g):
        i = bad_g[0]
        msg.append(f"{len(bad_g)} g mismatches, first row {i}: ref {g_ref[i]!r} got {g[i]!r}")
    if len(bad_v):
        i = bad_v[0]
        j = bad_v[np.argmax(np.abs(v_ref[bad_v] - v[bad_v]))]
        msg.append(f"{len(bad_v)} J mismatches, first nz {i} (row {rows_ref[i]}): ref {v_ref[i]!r} got {v[i]!r}; "
                   f"largest at nz {j} (row {rows_ref[j]}): ref {v_ref[j]!r} got {v[j]!r}")
    assert not msg, what + ": " + "; ".join(msg)


def assert_cost_close(f_ref, f, g_ref, g, what=""):
    """Objective and dense gradient: the value tolerance above with the floor 1e-12 * max(1, |f|) for f
    and 1e-12 * max(1, max |grad|) for the gradient (its entries are sums over many samples whose
    order differs: the device accumulates them with atomics)."""
    assert abs(f - f_ref) <= REL * max(abs(f), abs(f_ref)) + ABS * max(1.0, abs(f_ref)), \
        f"{what}: f ref {f_ref!r} got {f!r}"
    scale = max(1.0, float(np.max(np.abs(g_ref))) if len(g_ref) else 1.0)
    tol = REL * np.maximum(np.abs(g_ref), np.abs(g)) + ABS * scale
    bad = np.flatnonzero(np.abs(g_ref - g) > tol)
    if len(bad):
        j = bad[np.argmax(np.abs(g_ref[bad] - g[bad]))]
        raise AssertionError(f"{what}: {len(bad)} gradient mismatches, largest at {j}: ref {g_ref[j]!r} got {g[j]!r}")
