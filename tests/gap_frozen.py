"""Helpers shared by the emulation and GPU parity tests (no GPU needed)."""
import numpy as np

from towr2025_amd import formulation as F


def is_gap(desc):
    return desc.terrain.id == F.HeightMap.GapID


def frozen_reference(o, r, c, x):
    """The reference Jacobian at x mapped onto the engine's pattern (frozen at x0). On Gap terrain the
    reference's pattern moves with x (skip-on-zero, force_constraint_discretized.cc:58): entries of the
    frozen pattern the reference skips at x are expected as 0.0; reference entries outside the frozen
    pattern are returned as a count (IPOPT's structure is fixed at x0, so they cannot be delivered)."""
    rr, cc, vv = o.eval_jac(x)
    key_ref = rr.astype(np.int64) * o.n + cc
    key = r.astype(np.int64) * o.n + c
    idx = np.minimum(np.searchsorted(key_ref, key), len(key_ref) - 1)
    found = key_ref[idx] == key
    v_exp = np.where(found, vv[idx], 0.0)
    outside = int(np.count_nonzero(~np.isin(key_ref, key)))
    return v_exp, outside
