"""Generates the committed golden fixtures tests/golden/*.npz (TEST INFRASTRUCTURE).

The reference's own tests hold no golden vectors (towr/test/dynamic_constraint_test.cc:40-43 and
dynamic_model_test.cc:36-49 are empty) and the reference cannot be built here (Eigen3, ifopt and
Ipopt are absent), so these fixtures are produced by the CPU oracle (oracle/towr_oracle.c, the C
restatement of the reference path, itself pinned by the sympy KATs and finite differences of
tests/test_oracle_kat.py / test_oracle_fd.py). They freeze the oracle's outputs so that any later
change of the oracle or of the engine is checked against fixed vectors:
monoped-procedural and ANYmal trot (BASELINE configs[2]) at x0 and two seeded perturbations.

usage: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

SEEDS = (0, 20261016, 20261017)    # 0 = x0 itself
SCALE = 0.05


def cases():
    from towr2025_amd import formulation as F
    return {"monoped_procedural": F.procedural_desc(), "anymal_trot_2p4s": F.anymal_trot().to_desc()}


def xs_for(x0):
    out = []
    for s in SEEDS:
        out.append(x0.copy() if s == 0 else x0 + SCALE * np.random.default_rng(s).standard_normal(x0.shape))
    return np.stack(out)


def main():
    from oracle.oracle import Oracle, build
    build()
    for name, desc in cases().items():
        o = Oracle(desc)
        x0 = o.initial_x()
        X = xs_for(x0)
        r, c, _ = o.eval_jac(x0)
        G = np.stack([o.eval_g(x) for x in X])
        V = np.stack([o.eval_jac(x)[2] for x in X])
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, x=X, g=G, iRow=r.astype(np.int32), jCol=c.astype(np.int32), values=V,
                            seeds=np.array(SEEDS), n=o.n, m=o.m)
        print(f"{path}: n={o.n} m={o.m} nnz={len(r)} ({os.path.getsize(path) / 1e3:.0f} kB)")


if __name__ == "__main__":
    main()
