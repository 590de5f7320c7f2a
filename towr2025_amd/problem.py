"""ifopt::Problem-shaped host API over the HIP engine's C-ABI (include/towr_gpu.h).

Mirrors what IPOPT reaches through ifopt's IpoptAdapter for the hot path:
  GetNumberOfOptimizationVariables / GetNumberOfConstraints / nonzeros  -> sizes()
  GetVariableValues (starting point)                                    -> initial_x()
  EvalConstraints(x)                         (IpoptAdapter::eval_g)     -> eval_g(x)
  GetJacobianOfConstraints structure         (eval_jac_g, values=NULL)  -> jac_structure()
  EvalNonzerosOfJacobian(x)                  (eval_jac_g, values!=NULL) -> eval_jac_values(x)
  EvaluateCostFunction / ...Gradient         (eval_f / eval_grad_f)     -> eval_f(x) / eval_grad_f(x)
  SaveTrajectoryToCSV's samples              (save_data.cpp:9-130)      -> sample_trajectory(x, dt)
plus the batched, device-resident entry points used by bench.py.

Every evaluation runs on the GPU through libtowr_gpu.so; there is no CPU path. A missing or
unloadable extension raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi as capi


class TowrGpuError(RuntimeError):
    pass


def _check_tensor(t, what, min_cols, device=None):
    """A device batch operand: float64, on a HIP device (the handle's), rows contiguous (stride(1) == 1),
    at least min_cols columns. The C-ABI sees only a pointer and a leading dimension, so a float32 or
    strided tensor would otherwise be read or written out of bounds."""
    import torch
    if t.dtype != torch.float64:
        raise TowrGpuError(f"{what}: dtype {t.dtype}, expected torch.float64")
    if t.device.type != "cuda":
        raise TowrGpuError(f"{what}: tensor on {t.device}, expected a HIP device tensor")
    if device is not None and t.device.index != device:
        raise TowrGpuError(f"{what}: tensor on {t.device}, the handle is on device {device}")
    if t.dim() == 2:
        if t.shape[1] > 1 and t.stride(1) != 1:
            raise TowrGpuError(f"{what}: stride(1) = {t.stride(1)}, expected 1 (row-major rows)")
        if t.shape[1] < min_cols:
            raise TowrGpuError(f"{what}: {t.shape[1]} columns, needs >= {min_cols}")
        if t.shape[0] > 1 and t.stride(0) < min_cols:
            raise TowrGpuError(f"{what}: leading dimension {t.stride(0)} < {min_cols}")
    elif t.dim() != 1:
        raise TowrGpuError(f"{what}: expected a 1-D or 2-D tensor")


class TowrGpuProblem:
    """`data`: side data of towr_gpu_create_ex, [(towr_data_kind, index, float64 array)]: the matrix M of
    each LinearEqualityConstraint (capi.DATA_LINEAR_M, constraint index, rows x n_set row-major) and the
    wrapped set's bounds of each SoftConstraint term (capi.DATA_SOFT_BOUNDS, cost index, [lower, upper])."""

    def __init__(self, desc: capi.ProblemDesc, device: int = 0, data=None):
        self._lib = capi.load_library()
        self.desc = desc
        self.device = device
        h = C.c_void_p()
        arr, keep = capi.side_data(data)
        rc = self._lib.towr_gpu_create_ex(C.byref(desc), len(data or []), arr, device, C.byref(h))
        if rc != capi.TOWR_OK:
            raise TowrGpuError(f"towr_gpu_create failed ({rc}): {self._lib.towr_gpu_last_error(None).decode()}")
        self._h = h
        self._pinned = {}
        n, m, nnz = C.c_int32(), C.c_int32(), C.c_int64()
        self._check(self._lib.towr_gpu_sizes(h, C.byref(n), C.byref(m), C.byref(nnz)))
        self.n, self.m, self.nnz = n.value, m.value, nnz.value

    def _check(self, rc):
        if rc != capi.TOWR_OK:
            raise TowrGpuError(f"towr_gpu error {rc}: {self._lib.towr_gpu_last_error(self._h).decode()}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.towr_gpu_destroy(self._h)   # unregisters the registered host arrays
            self._h = None
            self._pinned = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------------- structure ----------
    def sizes(self):
        return self.n, self.m, self.nnz

    def initial_x(self) -> np.ndarray:
        x = np.zeros(self.n)
        self._check(self._lib.towr_gpu_initial_x(self._h, capi.dptr(x)))
        return x

    def initial_x_for(self, init: capi.InitDesc, terrain: capi.Terrain) -> np.ndarray:
        """x0 of another start/goal/terrain instance on this layout (batch harness)."""
        x = np.zeros(self.n)
        self._check(self._lib.towr_gpu_initial_x_for(self._h, C.byref(init), C.byref(terrain), capi.dptr(x)))
        return x

    def varset_info(self):
        out = []
        for i in range(self.desc.n_varsets):
            k, e, c0, n = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
            self._check(self._lib.towr_gpu_varset_info(self._h, i, C.byref(k), C.byref(e), C.byref(c0), C.byref(n)))
            out.append((k.value, e.value, c0.value, n.value))
        return out

    def jac_structure(self):
        r = np.zeros(self.nnz, dtype=np.int32)
        c = np.zeros(self.nnz, dtype=np.int32)
        self._check(self._lib.towr_gpu_jac_structure(self._h, capi.iptr(r), capi.iptr(c)))
        return r, c

    def jac_csr(self):
        rp = np.zeros(self.m + 1, dtype=np.int64)
        c = np.zeros(self.nnz, dtype=np.int32)
        self._check(self._lib.towr_gpu_jac_csr(self._h, capi.lptr(rp), capi.iptr(c)))
        return rp, c

    # -------------------------------------------------------------------- evaluation ---------
    def eval_g(self, x) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        g = np.zeros(self.m)
        self._check(self._lib.towr_gpu_eval_g(self._h, capi.dptr(x), capi.dptr(g)))
        return g

    def eval_jac_values(self, x) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        v = np.zeros(self.nnz)
        self._check(self._lib.towr_gpu_eval_jac_values(self._h, capi.dptr(x), capi.dptr(v)))
        return v

    def eval_g_jac(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        g, v = np.zeros(self.m), np.zeros(self.nnz)
        self._check(self._lib.towr_gpu_eval_g_jac(self._h, capi.dptr(x), capi.dptr(g), capi.dptr(v)))
        return g, v

    def eval_g_keep_jac(self, x) -> np.ndarray:
        """g at x, the Jacobian kept on the device for eval_jac_values_kept (IPOPT's eval_g at a new x)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        g = np.zeros(self.m)
        self._check(self._lib.towr_gpu_eval_g_keep_jac(self._h, capi.dptr(x), capi.dptr(g)))
        return g

    def eval_jac_values_kept(self, x) -> np.ndarray:
        """The Jacobian values at x: the kept ones when x is bit-identical to eval_g_keep_jac's, else evaluated."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        v = np.zeros(self.nnz)
        self._check(self._lib.towr_gpu_eval_jac_values_kept(self._h, capi.dptr(x), capi.dptr(v)))
        return v

    def eval_g_jac_into(self, x, g, v):
        """eval_g + eval_jac_g into caller arrays (contiguous float64): with x, g, v registered
        (register_host) the transfers run in place, as an IPOPT driver reusing its buffers would."""
        for a, k in ((x, self.n), (g, self.m), (v, self.nnz)):
            if a.dtype != np.float64 or not a.flags.c_contiguous or a.size < k:
                raise TowrGpuError("eval_g_jac_into: contiguous float64 arrays of n / m / nnz entries expected")
        self._check(self._lib.towr_gpu_eval_g_jac(self._h, capi.dptr(x), capi.dptr(g), capi.dptr(v)))

    def register_host(self, a):
        """Page-lock a contiguous numpy array for in-place host transfers (towr_gpu_register_host)."""
        if not a.flags.c_contiguous:
            raise TowrGpuError("register_host: contiguous array expected")
        self._check(self._lib.towr_gpu_register_host(self._h, C.c_void_p(a.ctypes.data), a.nbytes))
        self._pinned[a.ctypes.data] = a   # keep it alive while registered

    def unregister_host(self, a):
        self._check(self._lib.towr_gpu_unregister_host(self._h, C.c_void_p(a.ctypes.data)))
        self._pinned.pop(a.ctypes.data, None)

    def eval_f(self, x) -> float:
        """Objective (IpoptAdapter::eval_f): the sum of every cost term."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        f = C.c_double()
        self._check(self._lib.towr_gpu_eval_f(self._h, capi.dptr(x), C.byref(f)))
        return f.value

    def eval_grad_f(self, x) -> np.ndarray:
        """Dense objective gradient (IpoptAdapter::eval_grad_f)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        grad = np.zeros(self.n)
        self._check(self._lib.towr_gpu_eval_grad_f(self._h, capi.dptr(x), capi.dptr(grad)))
        return grad

    def eval_cost_batch_device(self, X, F, GRAD=None, stream=None):
        """Device batch objective on torch HIP tensors: X (B, ldx) -> F (B,), GRAD (B, ldgrad) or None."""
        import torch
        B = X.shape[0]
        _check_tensor(X, "X", self.n, self.device)
        _check_tensor(F, "F", 1, self.device)
        if F.dim() != 1 or F.shape[0] < B or (B > 1 and F.stride(0) != 1):
            raise TowrGpuError("F: expected a contiguous 1-D tensor of >= B entries")
        if GRAD is not None:
            _check_tensor(GRAD, "GRAD", self.n, self.device)
            if GRAD.shape[0] < B:
                raise TowrGpuError("GRAD: fewer rows than X")
        if stream is None:
            stream = torch.cuda.current_stream(X.device)
        self._check(self._lib.towr_gpu_eval_cost_batch_device(
            self._h, B, C.c_void_p(X.data_ptr()), X.stride(0), C.c_void_p(F.data_ptr()),
            C.c_void_p(GRAD.data_ptr() if GRAD is not None else 0), GRAD.stride(0) if GRAD is not None else 0,
            C.c_void_p(stream.cuda_stream)))

    def trajectory_size(self, dt: float):
        """(n_samples, n_cols) of the trajectory export at sample period dt."""
        ns, nc = C.c_int32(), C.c_int32()
        self._check(self._lib.towr_gpu_trajectory_size(self._h, dt, C.byref(ns), C.byref(nc)))
        return ns.value, nc.value

    def sample_trajectory(self, x, dt: float = 0.001) -> np.ndarray:
        """SaveTrajectoryToCSV's samples (save_data.cpp:9-130) on the device: (n_samples, 19 + 25 n_ee)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        ns, nc = self.trajectory_size(dt)
        out = np.zeros((ns, nc))
        self._check(self._lib.towr_gpu_sample_trajectory(self._h, capi.dptr(x), dt, capi.dptr(out)))
        return out

    def sample_trajectory_batch_device(self, X, dt, OUT, stream=None):
        """Device batch on torch HIP tensors: X (B, ldx) -> OUT (B, ldo >= n_samples * n_cols)."""
        import torch
        _check_tensor(X, "X", self.n, self.device)
        ns, nc = self.trajectory_size(dt)
        _check_tensor(OUT, "OUT", ns * nc, self.device)
        if OUT.shape[0] < X.shape[0]:
            raise TowrGpuError("OUT: fewer rows than X")
        if stream is None:
            stream = torch.cuda.current_stream(X.device)
        self._check(self._lib.towr_gpu_sample_trajectory_batch_device(
            self._h, X.shape[0], C.c_void_p(X.data_ptr()), X.stride(0), dt, C.c_void_p(OUT.data_ptr()), OUT.stride(0),
            C.c_void_p(stream.cuda_stream)))

    def set_batch_terrain(self, terrains):
        arr = (capi.Terrain * len(terrains))(*terrains)
        self._check(self._lib.towr_gpu_set_batch_terrain(self._h, len(terrains), arr))

    def eval_batch(self, X, G=None, V=None):
        """Host batch: X (B, n) -> G (B, m), V (B, nnz) (new arrays, or the given contiguous ones)."""
        X = np.ascontiguousarray(X, dtype=np.float64)
        B = X.shape[0]
        if G is None:
            G = np.zeros((B, self.m))
        if V is None:
            V = np.zeros((B, self.nnz))
        for a, k, name in ((G, self.m, "G"), (V, self.nnz, "V")):
            if a.dtype != np.float64 or not a.flags.c_contiguous or a.shape != (B, k):
                raise TowrGpuError(f"eval_batch: {name} must be a contiguous float64 array of shape ({B}, {k})")
        self._check(self._lib.towr_gpu_eval_batch(self._h, B, capi.dptr(X), capi.dptr(G), capi.dptr(V)))
        return G, V

    def eval_batch_device(self, X, G, V, want_g=True, want_jac=True, stream=None):
        """Device batch on torch CUDA (HIP) tensors: X (B, ldx), G (B, ldg), V (B, ldv) float64.
        `stream`: a torch.cuda.Stream (default: torch's current stream)."""
        import torch
        B = X.shape[0]
        self._check_batch(X, G, V, want_g, want_jac)
        if stream is None:
            stream = torch.cuda.current_stream(X.device)
        def ptr(t):   # an output that is not wanted may be None (NULL: the C-ABI never touches it)
            return (C.c_void_p(None), 0) if t is None else (C.c_void_p(t.data_ptr()), t.stride(0))
        (gp, ldg), (vp, ldv) = ptr(G), ptr(V)
        self._check(self._lib.towr_gpu_eval_batch_device(
            self._h, B, C.c_void_p(X.data_ptr()), X.stride(0), gp, ldg, vp, ldv,
            int(want_g), int(want_jac), C.c_void_p(stream.cuda_stream)))

    def _check_batch(self, X, G, V, want_g=True, want_jac=True):
        B = X.shape[0]
        _check_tensor(X, "X", self.n, self.device)
        for t, name, cols, want in ((G, "G", self.m, want_g), (V, "V", self.nnz, want_jac)):
            if want or t is not None:
                _check_tensor(t, name, cols, self.device)
                if t.shape[0] < B:
                    raise TowrGpuError(f"{name}: fewer rows than X")

    def step_launches(self):
        """Kernel indices (see kernels()) that one evaluation launches: fusion groups, then the unfused classes."""
        buf = (C.c_int32 * 16)()
        n = self._lib.towr_gpu_step_launches(self._h, buf, 16)
        if n < 0:
            self._check(n)
        return list(buf[:n])

    def kernels(self):
        """[(index, name, n_tiles, algorithmic bytes per problem)] of the launch classes' kernels and the
        fusion groups (index >= 5) this handle uses."""
        out = []
        for k in range(self._lib.towr_gpu_num_kernels()):
            name, nt, by = C.c_char_p(), C.c_int32(), C.c_int64()
            self._check(self._lib.towr_gpu_kernel_info(self._h, k, C.byref(name), C.byref(nt), C.byref(by)))
            if nt.value:
                out.append((k, name.value.decode(), nt.value, by.value))
        return out

    def pattern_outside(self, x) -> int:
        """Reference Jacobian entries at x outside the frozen (x0) pattern: non-zero only on curved terrain,
        where ForceConstraintDiscretized / TorqueConstraintDiscretized blocks appear with x (towr_gpu.h)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        c = C.c_int64()
        self._check(self._lib.towr_gpu_pattern_outside(self._h, x.ctypes.data_as(capi._DP), C.byref(c)))
        return int(c.value)

    def pattern_outside_batch(self, X, counts, stream=None):
        """pattern_outside of every problem of a device batch X (per-problem batch terrains as eval_batch_device)
        into the host int32 array `counts`; synchronous (X is copied to the host and checked there)."""
        import torch
        _check_tensor(X, "X", self.n, self.device)
        if not (isinstance(counts, np.ndarray) and counts.dtype == np.int32 and counts.flags.c_contiguous and counts.size >= X.shape[0]):
            raise TowrGpuError("counts: contiguous int32 numpy array with one entry per problem expected")
        s = stream.cuda_stream if stream is not None else torch.cuda.current_stream(X.device).cuda_stream
        self._check(self._lib.towr_gpu_pattern_outside_batch_device(self._h, X.shape[0], C.c_void_p(X.data_ptr()), X.stride(0),
                                                                     counts.ctypes.data_as(capi._IP), C.c_void_p(s)))

    def kernel_path(self, kernel: int) -> int:
        """Implementation of launch class `kernel` (0..4): 0 tile kernel, 1 record + stream kernels, -1 unused."""
        rc = self._lib.towr_gpu_kernel_path(self._h, kernel)
        if rc < -1:
            self._check(rc)
        return rc

    def eval_batch_device_kernel(self, kernel, X, G, V, stream):
        """Launch one kernel only: a launch class or a fusion group (roofline accounting)."""
        self._check_batch(X, G, V)
        self._check(self._lib.towr_gpu_eval_batch_device_kernel(
            self._h, kernel, X.shape[0], C.c_void_p(X.data_ptr()), X.stride(0),
            C.c_void_p(G.data_ptr()), G.stride(0), C.c_void_p(V.data_ptr()), V.stride(0),
            C.c_void_p(stream.cuda_stream)))

    def set_tiles_per_block(self, t: int):
        self._check(self._lib.towr_gpu_set_tiles_per_block(self._h, t))

    def algorithmic_bytes_per_call(self) -> int:
        return int(self._lib.towr_gpu_algorithmic_bytes_per_call(self._h))
