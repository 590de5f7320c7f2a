"""TEST INFRASTRUCTURE ONLY — ctypes binding of the CPU oracle (oracle/build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, as the
checker / CPU baseline. The product package towr2025_amd never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from towr2025_amd import _capi as capi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")
LIB_NATIVE = os.path.join(_HERE, "build", "liboracle_native.so")
_libs = {}


def build(native=False):
    subprocess.check_call(["make", "-s", "-C", _HERE] + (["native"] if native else []))


def lib(native=False):
    """The oracle library; native=True: the -O3 -march=native build of this host (CPU baseline only)."""
    if native not in _libs:
        path = LIB_NATIVE if native else LIB
        if native or not os.path.exists(path):
            build(native)
        L = C.CDLL(path)
        D, I, Lg = C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_long)
        L.oracle_create.restype = C.c_void_p
        L.oracle_create.argtypes = [C.POINTER(capi.ProblemDesc), C.c_char_p, C.c_int]
        L.oracle_create_ex.restype = C.c_void_p
        L.oracle_create_ex.argtypes = [C.POINTER(capi.ProblemDesc), C.c_int, C.POINTER(capi.SideData), C.c_char_p, C.c_int]
        L.oracle_destroy.argtypes = [C.c_void_p]
        L.oracle_sizes.argtypes = [C.c_void_p, I, I]
        L.oracle_initial_x.argtypes = [C.c_void_p, D]
        L.oracle_eval_g.argtypes = [C.c_void_p, D, D]
        L.oracle_eval_jac.restype = C.c_long
        L.oracle_eval_jac.argtypes = [C.c_void_p, D, C.c_long, I, I, D]
        L.oracle_eval_jac_values.restype = C.c_long
        L.oracle_eval_jac_values.argtypes = [C.c_void_p, D, D]
        L.oracle_eval_f.argtypes = [C.c_void_p, D, D]
        L.oracle_eval_grad_f.argtypes = [C.c_void_p, D, D]
        L.oracle_sample_trajectory.argtypes = [C.c_void_p, D, C.c_double, D]
        L.oracle_constraint_rows.argtypes = [C.c_void_p, C.c_int, I, I]
        L.oracle_varset_cols.argtypes = [C.c_void_p, C.c_int, I, I]
        L.oracle_bench.restype = C.c_double
        L.oracle_bench.argtypes = [C.POINTER(capi.ProblemDesc), C.c_int, C.c_int, C.c_int, D, Lg]
        _libs[native] = L
    return _libs[native]


def _d(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _i(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


class Oracle:
    """ifopt::Problem-shaped view of the CPU restatement. `data`: side data as for towr_gpu_create_ex,
    a list of (towr_data_kind, index, float64 array)."""

    def __init__(self, desc: capi.ProblemDesc, data=None):
        self.desc = desc
        err = C.create_string_buffer(256)
        arr, self._keep = capi.side_data(data)
        self.h = lib().oracle_create_ex(C.byref(desc), len(data or []), arr, err, 256)
        if not self.h:
            raise ValueError("oracle_create failed: " + err.value.decode())
        n, m = C.c_int(), C.c_int()
        lib().oracle_sizes(self.h, C.byref(n), C.byref(m))
        self.n, self.m = n.value, m.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_destroy(self.h)
            self.h = None

    def initial_x(self):
        x = np.zeros(self.n)
        lib().oracle_initial_x(self.h, _d(x))
        return x

    def eval_g(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        g = np.zeros(self.m)
        lib().oracle_eval_g(self.h, _d(x), _d(g))
        return g

    def eval_f(self, x):
        """Problem::EvaluateCostFunction (IpoptAdapter::eval_f)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        f = np.zeros(1)
        lib().oracle_eval_f(self.h, _d(x), _d(f))
        return float(f[0])

    def eval_grad_f(self, x):
        """Problem::EvaluateCostFunctionGradient (IpoptAdapter::eval_grad_f), dense."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        g = np.zeros(self.n)
        lib().oracle_eval_grad_f(self.h, _d(x), _d(g))
        return g

    def sample_trajectory(self, x, dt):
        """SaveTrajectoryToCSV's sample rows (save_data.cpp:9-130): (n_samples, 19 + 25 E)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        ns = lib().oracle_sample_trajectory(self.h, _d(x), dt, None)
        out = np.zeros((ns, 19 + 25 * self.desc.robot.n_ee))
        lib().oracle_sample_trajectory(self.h, _d(x), dt, _d(out))
        return out

    def eval_jac(self, x):
        """(rows, cols, vals) of GetJacobianOfConstraints at x — pattern at x, sorted row-major."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        nnz = lib().oracle_eval_jac(self.h, _d(x), 0, None, None, None)
        r = np.zeros(nnz, dtype=np.int32)
        c = np.zeros(nnz, dtype=np.int32)
        v = np.zeros(nnz)
        lib().oracle_eval_jac(self.h, _d(x), nnz, _i(r), _i(c), _d(v))
        return r, c, v

    def constraint_rows(self):
        out = []
        for i in range(self.desc.n_constraints):
            a, b = C.c_int(), C.c_int()
            lib().oracle_constraint_rows(self.h, i, C.byref(a), C.byref(b))
            out.append((a.value, b.value))
        return out

    def varset_cols(self):
        out = []
        for i in range(self.desc.n_varsets):
            a, b = C.c_int(), C.c_int()
            lib().oracle_varset_cols(self.h, i, C.byref(a), C.byref(b))
            out.append((a.value, b.value))
        return out


def bench(desc, threads, calls_per_thread, X, native=False):
    X = np.ascontiguousarray(X, dtype=np.float64)
    done = C.c_long()
    secs = lib(native).oracle_bench(C.byref(desc), threads, calls_per_thread, X.shape[0], _d(X), C.byref(done))
    return secs, done.value
