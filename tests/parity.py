"""Shared parity helpers: the tolerance of BASELINE.md / SURVEY §8(d), written once.

values:  |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, rowscale)
where rowscale = max |J| over the reference row (BASELINE.md's gate, on every entry).

Two whitelisted widenings, and only where they are needed (`residue_cols`): an entry in such a column
gets the floor 1e-12 * max(1, rowscale, colscale), colscale = max |J| over the reference column.
 1. PHASE-DURATION (schedule) columns of a phase-duration-optimisation problem. These entries are
    d pos / d duration of a PhaseSpline (phase_spline.cc:67-93, polynomial.cc:236-257); where the
    spline is analytically flat at an instant (a zero force in swing) the value is the ~1e-11 residue
    of ~1e5-sized Hermite terms, which differs with any change of operation order, the reference's own
    build included.
 2. Endeffector-motion columns of the ForceConstraintDiscretized / TorqueConstraintDiscretized rows on
    curved (Gap) terrain (the other rows of those columns keep the row gate). ForceConstraintDiscretized's motion block is
    scale * basis with scale = f . d(pyramid)/dp (force_constraint_discretized.cc:125-155); at a phase
    junction the force spline's value cancels to a rounding residue (~1e-14 N of ~1e2 N nodes), so the
    entry is a residue of ~1e3-sized terms. Its bits depend on the libm: the reference's std::pow is
    glibc's, which is not correctly rounded (pow(x, 3) differs from the correctly rounded cube in
    ~0.09 % of arguments, measured), while the engine's device powers are; a reference build on
    another libm gives another residue. Rows made only of such residues have no row scale to hide
    behind; the column's scale (the same block at instants away from the junction) bounds them.
The column scale bounds the residue's size. No other entry is widened.

g:       |a - b| <= 1e-9 * max(|a|, |b|) + 1e-12 * max(1, |J row| scale)
Pattern: bit-exact (same (row, col) list in the same order).
"""
import numpy as np

REL = 1e-9
ABS = 1e-12

VAR_EE_SCHEDULE = 6   # towr_varset_kind (include/towr_gpu.h), PhaseDurations sets


def schedule_cols(desc, n, data=None):
    """Boolean mask over the n columns: True for PhaseDurations (schedule) variable columns."""
    from oracle.oracle import Oracle   # column offsets: the oracle's layout (ifopt's AddVariableSet order)
    mask = np.zeros(n, dtype=bool)
    if not desc.optimize_timings:
        return mask
    o = Oracle(desc, data)
    for i, (c0, nc) in enumerate(o.varset_cols()):
        if desc.varsets[i].kind == VAR_EE_SCHEDULE:
            mask[c0:c0 + nc] = True
    return mask


VAR_EE_MOTION = 2     # endeffector-motion node sets
TERRAIN_GAP = 3       # towr_terrain_id: the only terrain with curvature
from towr2025_amd._capi import C_FORCE_DISCRETIZED, C_TORQUE_DISCRETIZED  # noqa: E402


class ResidueMask:
    """The entries that get the column-scaled floor: every entry of a schedule column, and on Gap terrain the
    entries of endeffector-motion columns in ForceConstraintDiscretized / TorqueConstraintDiscretized rows."""

    def __init__(self, sched_cols, motion_cols, motion_rows):
        self.sched_cols, self.motion_cols, self.motion_rows = sched_cols, motion_cols, motion_rows

    def any(self):
        return bool(self.sched_cols.any() or (self.motion_cols.any() and self.motion_rows.any()))

    def entries(self, rows, cols):
        if not self.motion_rows.any():
            return self.sched_cols[cols]
        return self.sched_cols[cols] | (self.motion_cols[cols] & self.motion_rows[rows])


def residue_cols(desc, n, data=None):
    """The ResidueMask of a description (see the module docstring): the schedule columns, and on Gap terrain
    the endeffector-motion columns of the discretized force / torque rows."""
    sched = schedule_cols(desc, n, data)
    motion = np.zeros(n, dtype=bool)
    rows = np.zeros(0, dtype=bool)
    if desc.terrain.id == TERRAIN_GAP:
        from oracle.oracle import Oracle
        o = Oracle(desc, data)
        for i, (c0, nc) in enumerate(o.varset_cols()):
            if desc.varsets[i].kind == VAR_EE_MOTION:
                motion[c0:c0 + nc] = True
        rows = np.zeros(o.m, dtype=bool)
        for i, (r0, nr) in enumerate(o.constraint_rows()):
            if desc.constraints[i].kind in (C_FORCE_DISCRETIZED, C_TORQUE_DISCRETIZED):
                rows[r0:r0 + nr] = True
    return ResidueMask(sched, motion, rows)


def _within(a, b, err, tol):
    """Entries inside the tolerance. A NaN on either side is a mismatch (err <= tol is False for it), and so is an
    infinity facing a finite value: its tolerance REL * inf is itself infinite, so err <= tol alone would pass it.
    Identical values (the same infinity included) always match."""
    return (a == b) | ((err <= tol) & np.isfinite(a) & np.isfinite(b))


def check_values(g_ref, g, rows_ref, v_ref, v, m, cols_ref=None, floor_cols=None):
    """Indices of g and J entries outside the tolerance, and a summary dict:
    max_rel = largest |a-b| / max(|a|,|b|) over entries above their floor; worst = largest
    |a-b| / tolerance; widened = entries whose tolerance the schedule-column floor raised."""
    rs = np.zeros(m)
    np.maximum.at(rs, rows_ref, np.abs(v_ref))
    floor = ABS * np.maximum(1.0, rs)
    floor_v = floor[rows_ref]
    widened = 0
    if cols_ref is not None and floor_cols is not None and floor_cols.any():
        on = floor_cols.entries(rows_ref, cols_ref) if isinstance(floor_cols, ResidueMask) else floor_cols[cols_ref]
        cs = np.zeros(int(cols_ref.max()) + 1 if len(cols_ref) else 0)
        np.maximum.at(cs, cols_ref, np.abs(v_ref))
        col_floor = np.where(on, ABS * cs[cols_ref], 0.0)
        widened = int(np.count_nonzero(col_floor > floor_v))
        floor_v = np.maximum(floor_v, col_floor)
    mag_v = np.maximum(np.abs(v_ref), np.abs(v))
    err_v = np.abs(v_ref - v)
    tol_v = REL * mag_v + floor_v
    bad_v = np.flatnonzero(~_within(v_ref, v, err_v, tol_v))
    mag_g = np.maximum(np.abs(g_ref), np.abs(g))
    err_g = np.abs(g_ref - g)
    tol_g = REL * mag_g + floor
    bad_g = np.flatnonzero(~_within(g_ref, g, err_g, tol_g))
    big_v = mag_v > floor_v
    big_g = mag_g > floor
    stats = {
        "max_rel": float(max(np.max(err_v[big_v] / mag_v[big_v], initial=0.0),
                             np.max(err_g[big_g] / mag_g[big_g], initial=0.0))),
        "worst": float(max(np.max(err_v / tol_v, initial=0.0), np.max(err_g / tol_g, initial=0.0))),
        "widened": widened,
    }
    return bad_g, bad_v, stats


def assert_close(g_ref, g, rows_ref, v_ref, v, m, what="", cols_ref=None, floor_cols=None):
    """BASELINE.md's gate; returns the summary of check_values (printed by the parity tests)."""
    bad_g, bad_v, stats = check_values(g_ref, g, rows_ref, v_ref, v, m, cols_ref, floor_cols)
    msg = []
    if len(bad_g):
        i = bad_g[0]
        msg.append(f"{len(bad_g)} g mismatches, first row {i}: ref {g_ref[i]!r} got {g[i]!r}")
    if len(bad_v):
        i = bad_v[0]
        j = bad_v[np.argmax(np.abs(v_ref[bad_v] - v[bad_v]))]
        cinfo = f" col {cols_ref[j]}" if cols_ref is not None else ""
        msg.append(f"{len(bad_v)} J mismatches, first nz {i} (row {rows_ref[i]}): ref {v_ref[i]!r} got {v[i]!r}; "
                   f"largest at nz {j} (row {rows_ref[j]}{cinfo}): ref {v_ref[j]!r} got {v[j]!r}")
    assert not msg, what + ": " + "; ".join(msg)
    return stats


def assert_cost_close(f_ref, f, g_ref, g, what=""):
    """Objective and dense gradient: the value tolerance above with the floor 1e-12 * max(1, |f|) for f
    and 1e-12 * max(1, max |grad|) for the gradient (its entries are sums over many samples whose
    order differs: the device accumulates them with atomics)."""
    assert bool(_within(np.float64(f_ref), np.float64(f), abs(f - f_ref), REL * max(abs(f), abs(f_ref)) + ABS * max(1.0, abs(f_ref)))), \
        f"{what}: f ref {f_ref!r} got {f!r}"
    fin = np.abs(g_ref)[np.isfinite(g_ref)]
    scale = max(1.0, float(np.max(fin)) if len(fin) else 1.0)
    tol = REL * np.maximum(np.abs(g_ref), np.abs(g)) + ABS * scale
    bad = np.flatnonzero(~_within(g_ref, g, np.abs(g_ref - g), tol))
    if len(bad):
        j = bad[np.argmax(np.abs(g_ref[bad] - g[bad]))]
        raise AssertionError(f"{what}: {len(bad)} gradient mismatches, largest at {j}: ref {g_ref[j]!r} got {g[j]!r}")
