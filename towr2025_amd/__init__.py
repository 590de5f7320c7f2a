"""towr2025_amd — MI355X (gfx950) engine for towr's eval_g / eval_jac_g hot path.

  towr2025_amd.formulation   reference-shaped setup API (Parameters, RobotModel, HeightMap,
                             GaitGenerator, NlpFormulation) -> include/towr_gpu.h ProblemDesc
  towr2025_amd.problem       TowrGpuProblem: ifopt::Problem-shaped evaluation over the C-ABI
  towr2025_amd._capi         ctypes mirror of include/towr_gpu.h, loader of lib/libtowr_gpu.so
"""
from . import _capi, formulation  # noqa: F401
from .problem import TowrGpuError, TowrGpuProblem  # noqa: F401

__all__ = ["TowrGpuProblem", "TowrGpuError", "formulation"]
