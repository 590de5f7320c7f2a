"""Per-kernel times of the phase-duration-optimisation batch (bench.py's gait_optimization workload)
for one build of the engine: the product library or an experiment build under tools/build. A
measurement tool, not part of the product.
usage: python tools/gait_ab.py [--lib tools/build/libtowr_gpu_nozero.so] [--batch 1024] [--reps 20]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rotvec", action="store_true")
    ap.add_argument("--no-gait", action="store_true", help="the headline formulation (fixed phase durations)")
    ap.add_argument("--only", default=None, help="comma-separated part names: time only these, no whole step")
    ap.add_argument("--torque", action="store_true", help="ANYmal on stairs + Parameters::Torque (bench.py gait_torque)")
    ap.add_argument("--step-only", action="store_true", help="only the whole step (no per-kernel times)")
    ap.add_argument("--settle-ms", type=float, default=300.0, help="untimed steps before timing (clock ramp)")
    args = ap.parse_args()
    import torch
    from towr2025_amd import _capi as capi
    if args.lib:
        capi.load_library(os.path.join(ROOT, args.lib))
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    import bench
    f = F.anymal_trot(optimize_timings=not args.no_gait,
                      terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID) if args.torque else None)
    if args.torque:
        f.params_.constraints_.append(F.Parameters.Torque)
    if args.rotvec:
        f.params_.angular_rep_ = 1
    p = TowrGpuProblem(f.to_desc(), device=0)
    B = args.batch
    Xh, ter = bench.make_batch(p, B, 0, optimize_timings=not args.no_gait)
    p.set_batch_terrain(ter)
    dev = torch.device("cuda", 0)
    X = torch.from_numpy(np.ascontiguousarray(Xh[0])).to(dev)
    G = torch.empty((B, (p.m + 15) // 16 * 16), dtype=torch.float64, device=dev)
    V = torch.empty((B, (p.nnz + 15) // 16 * 16), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    only = args.only.split(",") if args.only else None
    for _ in range(0 if only else 30):
        p.eval_batch_device(X, G, V)
    import time
    t0 = time.perf_counter()   # untimed steps until the clocks have ramped (bench.py --settle-ms)
    while time.perf_counter() - t0 < args.settle_ms * 1e-3:
        for _ in range(10):
            p.eval_batch_device(X, G, V)
        torch.cuda.synchronize()
    out = {}
    for k, name, nt, by in ([] if args.step_only else p.kernels()):
        if only and name not in only:
            continue
        for _ in range(3):
            p.eval_batch_device_kernel(k, X, G, V, st)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(args.reps):
            p.eval_batch_device_kernel(k, X, G, V, st)
        z.record(st)
        torch.cuda.synchronize()
        ms = a.elapsed_time(z) / args.reps
        out[name] = ms
        print(f"{args.lib or 'product':40s} {name:20s} {ms:8.4f} ms  {B * by / (ms * 1e-3) / 1e9:7.0f} GB/s", flush=True)
    if only:
        return
    a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(args.reps):
        p.eval_batch_device(X, G, V)
    z.record(st)
    torch.cuda.synchronize()
    print(f"{args.lib or 'product':40s} {'step':20s} {a.elapsed_time(z) / args.reps:8.4f} ms", flush=True)


if __name__ == "__main__":
    main()
