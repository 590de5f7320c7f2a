"""Shared parity helpers: the tolerance of BASELINE.md / SURVEY §8(d), written once.

values:  |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, rowscale)
where rowscale = max |J| over the reference row. The unit floor covers rows whose reference
entries are all structural zeros (e.g. Hermite basis functions that vanish at a polynomial end,
where the reference happens to round to exactly 0.0 and fused multiply-adds give ~4e-16).
g:       |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, |J row| scale)
Pattern: bit-exact (same (row, col) list in the same order).
"""
import numpy as np

REL = 1e-9
ABS = 1e-12


def check_values(g_ref, g, rows_ref, v_ref, v, m):
    rs = np.zeros(m)
    np.maximum.at(rs, rows_ref, np.abs(v_ref))
    floor = ABS * np.maximum(1.0, rs)
    tol_v = REL * np.maximum(np.abs(v_ref), np.abs(v)) + floor[rows_ref]
    bad_v = np.flatnonzero(np.abs(v_ref - v) > tol_v)
    tol_g = REL * np.maximum(np.abs(g_ref), np.abs(g)) + floor
    bad_g = np.flatnonzero(np.abs(g_ref - g) > tol_g)
    return bad_g, bad_v


def assert_close(g_ref, g, rows_ref, v_ref, v, m, what=""):
    bad_g, bad_v = check_values(g_ref, g, rows_ref, v_ref, v, m)
    msg = []
    if len(bad_g):
        i = bad_g[0]
        msg.append(f"{len(bad_g)} g mismatches, first row {i}: ref {g_ref[i]!r} got {g[i]!r}")
    if len(bad_v):
        i = bad_v[0]
        msg.append(f"{len(bad_v)} J mismatches, first nz {i} (row {rows_ref[i]}): ref {v_ref[i]!r} got {v[i]!r}")
    assert not msg, what + ": " + "; ".join(msg)
