"""ctypes mirror of include/towr_gpu.h (the C-ABI boundary) and the loader of libtowr_gpu.so.

The structs here must stay byte-identical to the C header; tests/test_capi.py checks sizes and
that every symbol declared in the header is exported by the built library.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 4
MAX_EE = 4
MAX_PHASES = 48
MAX_VARSETS = 2 + 5 * MAX_EE
MAX_CONSTRAINTS = 64

TOWR_OK = 0
TOWR_ERR_INVALID = -1
TOWR_ERR_UNSUPPORTED = -2
TOWR_ERR_HIP = -3
TOWR_ERR_NO_DEVICE = -4

# towr_terrain_id  (towr/include/towr/terrain/height_map.h:79-86 + hopper_example.cc FiveStepStairs)
TERRAIN_FLAT, TERRAIN_BLOCK, TERRAIN_STAIRS, TERRAIN_GAP, TERRAIN_SLOPE, TERRAIN_CHIMNEY, \
    TERRAIN_CHIMNEY_LR, TERRAIN_STEPS = range(8)

# towr_varset_kind (towr/include/towr/variables/variable_names.h:43-75)
VAR_BASE_LIN, VAR_BASE_ANG, VAR_EE_MOTION, VAR_EE_ANG, VAR_EE_FORCE, VAR_EE_TORQUE, \
    VAR_EE_SCHEDULE = range(7)

# towr_constraint_kind
C_DYNAMIC, C_RANGE_OF_MOTION, C_FORCE, C_FORCE_DISCRETIZED, C_TERRAIN, C_BASE_MOTION, \
    C_SPLINE_ACC, C_BASE_HEIGHT, C_SWING, C_TOTAL_DURATION, C_TORQUE_DISCRETIZED, C_TORQUE, C_TERRAIN_HARD, \
    C_EE_LINEAR, C_LINEAR_EQ = range(15)
ROLE_HARD, ROLE_SOFT = 0, 1   # towr_constraint_role

INIT_FORMULATION, INIT_PROCEDURAL = 0, 1


class Terrain(C.Structure):
    _fields_ = [("id", C.c_int32), ("reserved", C.c_int32),
                ("friction_coeff", C.c_double), ("p", C.c_double * 8)]


class Robot(C.Structure):
    _fields_ = [("mass", C.c_double), ("gravity", C.c_double), ("inertia", C.c_double * 6),
                ("n_ee", C.c_int32), ("reserved", C.c_int32),
                ("nominal_stance", (C.c_double * 3) * MAX_EE),
                ("max_dev", (C.c_double * 3) * MAX_EE),
                ("min_dev", (C.c_double * 3) * MAX_EE)]


class VarSetDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ee", C.c_int32)]


class ConstraintDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ee", C.c_int32), ("T", C.c_double), ("dt", C.c_double),
                ("p", C.c_double * 6), ("ip", C.c_int32 * 9), ("role", C.c_int32)]


class InitDesc(C.Structure):
    _fields_ = [("mode", C.c_int32), ("reserved", C.c_int32),
                ("base_lin_p0", C.c_double * 3), ("base_lin_v0", C.c_double * 3),
                ("base_ang_p0", C.c_double * 3), ("base_ang_v0", C.c_double * 3),
                ("base_lin_p1", C.c_double * 3), ("base_lin_v1", C.c_double * 3),
                ("base_ang_p1", C.c_double * 3), ("base_ang_v1", C.c_double * 3),
                ("ee_p0", (C.c_double * 3) * MAX_EE), ("ee_p1", (C.c_double * 3) * MAX_EE)]


# towr_cost_kind
COST_NODE, COST_ENERGY, COST_ANG_MOMENTUM, COST_EE_BASE_POS, COST_BASE_HEIGHT, COST_SOFT = range(6)
# towr_data_kind (side data of towr_gpu_create_ex)
DATA_LINEAR_M, DATA_SOFT_BOUNDS = 0, 1
MAX_COSTS = 128


class CostDesc(C.Structure):
    _fields_ = [("kind", C.c_int32), ("ee", C.c_int32), ("weight", C.c_double), ("dt", C.c_double),
                ("p", C.c_double * 4), ("ip", C.c_int32 * 4)]


class ProblemDesc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("angular_rep", C.c_int32),
                ("robot", Robot), ("terrain", Terrain),
                ("total_time", C.c_double), ("duration_base_polynomial", C.c_double),
                ("ee_polynomials_per_swing_phase", C.c_int32),
                ("force_polynomials_per_stance_phase", C.c_int32),
                ("torque_polynomials_per_stance_phase", C.c_int32),
                ("optimize_timings", C.c_int32),
                ("bound_phase_duration", C.c_double * 2),
                ("n_phases", C.c_int32 * MAX_EE), ("contact_at_start", C.c_int32 * MAX_EE),
                ("phase_durations", (C.c_double * MAX_PHASES) * MAX_EE),
                ("n_varsets", C.c_int32), ("n_constraints", C.c_int32),
                ("varsets", VarSetDesc * MAX_VARSETS),
                ("constraints", ConstraintDesc * MAX_CONSTRAINTS),
                ("init", InitDesc),
                ("n_costs", C.c_int32), ("reserved_costs", C.c_int32),
                ("costs", CostDesc * MAX_COSTS)]


class SideData(C.Structure):
    _fields_ = [("kind", C.c_int32), ("index", C.c_int32), ("count", C.c_int64),
                ("data", C.POINTER(C.c_double))]


# symbol table of include/towr_gpu.h: name -> (restype, argtypes)
_HANDLE = C.c_void_p
_DP = C.POINTER(C.c_double)
_IP = C.POINTER(C.c_int32)
_LP = C.POINTER(C.c_int64)
SYMBOLS = {
    "towr_gpu_create": (C.c_int, [C.POINTER(ProblemDesc), C.c_int, C.POINTER(_HANDLE)]),
    "towr_gpu_create_ex": (C.c_int, [C.POINTER(ProblemDesc), C.c_int32, C.POINTER(SideData), C.c_int,
                                      C.POINTER(_HANDLE)]),
    "towr_gpu_destroy": (C.c_int, [_HANDLE]),
    "towr_gpu_last_error": (C.c_char_p, [_HANDLE]),
    "towr_gpu_abi_version": (C.c_int, []),
    "towr_gpu_sizes": (C.c_int, [_HANDLE, _IP, _IP, _LP]),
    "towr_gpu_jac_structure": (C.c_int, [_HANDLE, _IP, _IP]),
    "towr_gpu_jac_csr": (C.c_int, [_HANDLE, _LP, _IP]),
    "towr_gpu_initial_x": (C.c_int, [_HANDLE, _DP]),
    "towr_gpu_initial_x_for": (C.c_int, [_HANDLE, C.POINTER(InitDesc), C.POINTER(Terrain), _DP]),
    "towr_gpu_varset_info": (C.c_int, [_HANDLE, C.c_int32, _IP, _IP, _IP, _IP]),
    "towr_gpu_eval_g": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_jac_values": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_g_jac": (C.c_int, [_HANDLE, _DP, _DP, _DP]),
    "towr_gpu_eval_g_keep_jac": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_jac_values_kept": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_f": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_grad_f": (C.c_int, [_HANDLE, _DP, _DP]),
    "towr_gpu_eval_cost_batch_device": (C.c_int, [_HANDLE, C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                                   C.c_void_p, C.c_int64, C.c_void_p]),
    "towr_gpu_trajectory_size": (C.c_int, [_HANDLE, C.c_double, _IP, _IP]),
    "towr_gpu_sample_trajectory": (C.c_int, [_HANDLE, _DP, C.c_double, _DP]),
    "towr_gpu_sample_trajectory_batch_device": (C.c_int, [_HANDLE, C.c_int32, C.c_void_p, C.c_int64, C.c_double,
                                                          C.c_void_p, C.c_int64, C.c_void_p]),
    "towr_gpu_set_batch_terrain": (C.c_int, [_HANDLE, C.c_int32, C.POINTER(Terrain)]),
    "towr_gpu_eval_batch_device": (C.c_int, [_HANDLE, C.c_int32, C.c_void_p, C.c_int64,
                                              C.c_void_p, C.c_int64, C.c_void_p, C.c_int64,
                                              C.c_int32, C.c_int32, C.c_void_p]),
    "towr_gpu_eval_batch": (C.c_int, [_HANDLE, C.c_int32, _DP, _DP, _DP]),
    "towr_gpu_kernel_info": (C.c_int, [_HANDLE, C.c_int32, C.POINTER(C.c_char_p), _IP, _LP]),
    "towr_gpu_eval_batch_device_kernel": (C.c_int, [_HANDLE, C.c_int32, C.c_int32, C.c_void_p, C.c_int64,
                                                     C.c_void_p, C.c_int64, C.c_void_p, C.c_int64, C.c_void_p]),
    "towr_gpu_num_kernels": (C.c_int, []),
    "towr_gpu_step_launches": (C.c_int, [_HANDLE, _IP, C.c_int32]),
    "towr_gpu_kernel_path": (C.c_int, [_HANDLE, C.c_int32]),
    "towr_gpu_pattern_outside": (C.c_int, [_HANDLE, _DP, _LP]),
    "towr_gpu_pattern_outside_batch_device": (C.c_int, [_HANDLE, C.c_int32, C.c_void_p, C.c_int64, _IP, C.c_void_p]),
    "towr_gpu_register_host": (C.c_int, [_HANDLE, C.c_void_p, C.c_int64]),
    "towr_gpu_unregister_host": (C.c_int, [_HANDLE, C.c_void_p]),
    "towr_gpu_set_tiles_per_block": (C.c_int, [_HANDLE, C.c_int32]),
    "towr_gpu_algorithmic_bytes_per_call": (C.c_int64, [_HANDLE]),
}

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TOWR_GPU_LIB") or os.path.join(_HERE, "lib", "libtowr_gpu.so")   # override: A/B builds
_lib = None


def load_library(path: str = LIB_PATH):
    """Load the in-tree HIP extension. Fails loudly: there is no CPU fallback for the product."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"towr2025_amd: HIP extension not built ({path} missing). Run __graft_entry__.build().")
    # One HIP runtime per process: torch bundles libamdhip64.so.7 (same SONAME as /opt/rocm's);
    # whichever loads first serves everyone, so when torch is present let its runtime load first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def side_data(entries):
    """[(kind, index, array)] -> (SideData array or None, the float64 arrays it points into)."""
    import numpy as np
    if not entries:
        return None, []
    keep = [np.ascontiguousarray(a, dtype=np.float64).ravel() for (_, _, a) in entries]
    arr = (SideData * len(entries))()
    for i, ((kind, index, _), a) in enumerate(zip(entries, keep)):
        arr[i].kind, arr[i].index, arr[i].count = kind, index, a.size
        arr[i].data = a.ctypes.data_as(_DP)
    return arr, keep


def dptr(a):
    """numpy float64 array -> double*"""
    return a.ctypes.data_as(_DP)


def iptr(a):
    return a.ctypes.data_as(_IP)


def lptr(a):
    return a.ctypes.data_as(_LP)
