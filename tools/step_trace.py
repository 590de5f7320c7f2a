"""A fixed number of phase-duration-optimisation batch steps (bench.py gait legs) for a kernel trace:
rocprofv3 --kernel-trace --stats -- python tools/step_trace.py [--torque] [--steps 30]. A measurement tool."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--torque", action="store_true")
    ap.add_argument("--rotvec", action="store_true", help="fixed-gait ANYmal with the RotVec base (B = 4096)")
    ap.add_argument("--lib", default=None)
    args = ap.parse_args()
    import torch
    from towr2025_amd import _capi as capi
    if args.lib:
        capi.load_library(os.path.join(ROOT, args.lib))
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    import bench
    gait = not args.rotvec
    f = F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID) if args.torque else None, optimize_timings=gait)
    if args.torque:
        f.params_.constraints_.append(F.Parameters.Torque)
    if args.rotvec:
        f.params_.angular_rep_ = 1
    p = TowrGpuProblem(f.to_desc(), device=0)
    B = args.batch
    Xh, ter = bench.make_batch(p, B, 0, optimize_timings=gait)
    p.set_batch_terrain(ter)
    dev = torch.device("cuda", 0)
    X = torch.from_numpy(np.ascontiguousarray(Xh[0])).to(dev)
    G = torch.empty((B, (p.m + 15) // 16 * 16), dtype=torch.float64, device=dev)
    V = torch.empty((B, (p.nnz + 15) // 16 * 16), dtype=torch.float64, device=dev)
    for _ in range(args.steps):
        p.eval_batch_device(X, G, V)
    torch.cuda.synchronize()
    print("steps done", args.steps)


if __name__ == "__main__":
    main()
