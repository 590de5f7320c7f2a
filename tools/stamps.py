"""In-kernel phase timestamps of the experiment build (make -C towr2025_amd/csrc variant VNAME=stamps
VFLAGS=-DTOWR_STAMPS): one gait step (bench.py's gait_optimization workload) with every launch's TG_STAMP slots
(kernel_common.h) collected, then per launch: blocks, span, and the median / p90 of each phase per block.
usage: python tools/stamps.py [--lib tools/build/libtowr_gpu_stamps.so] [--batch 1024] [--torque | --fixed] [--only KERNEL]
A measurement tool, not part of the product."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REGION, NREG = 1 << 21, 12
TICK_US = 0.01   # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="tools/build/libtowr_gpu_stamps.so")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--torque", action="store_true")
    ap.add_argument("--fixed", action="store_true", help="the headline formulation (fixed phase durations, B = 4096 default)")
    ap.add_argument("--only", type=int, default=-1, help="launch class index (towr_gpu_eval_batch_device_kernel)")
    ap.add_argument("--steps", type=int, default=20, help="untimed steps before the stamped one")
    args = ap.parse_args()
    import torch
    from towr2025_amd import _capi as capi
    capi.load_library(os.path.join(ROOT, args.lib))
    lib = capi.lib() if hasattr(capi, "lib") else capi._lib
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    import bench
    f = F.anymal_trot(optimize_timings=not args.fixed, terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID) if args.torque else None)
    if args.torque:
        f.params_.constraints_.append(F.Parameters.Torque)
    p = TowrGpuProblem(f.to_desc(), device=0)
    B = args.batch if not (args.fixed and args.batch == 1024) else 4096
    Xh, ter = bench.make_batch(p, B, 0, optimize_timings=not args.fixed)
    p.set_batch_terrain(ter)
    dev = torch.device("cuda", 0)
    X = torch.from_numpy(np.ascontiguousarray(Xh[0])).to(dev)
    G = torch.empty((B, (p.m + 15) // 16 * 16), dtype=torch.float64, device=dev)
    V = torch.empty((B, (p.nnz + 15) // 16 * 16), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    run = (lambda: p.eval_batch_device_kernel(args.only, X, G, V, st)) if args.only >= 0 else (lambda: p.eval_batch_device(X, G, V))
    for _ in range(args.steps):
        run()
    buf = torch.zeros(REGION * NREG, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    lib.towr_gpu_debug_stamps.argtypes = [C.c_void_p]
    lib.towr_gpu_debug_stamp_kernel.argtypes = [C.c_int]
    lib.towr_gpu_debug_stamp_kernel.restype = C.c_char_p
    lib.towr_gpu_debug_stamps(C.c_void_p(buf.data_ptr()))
    run()
    torch.cuda.synchronize()
    names = []
    for i in range(NREG):
        n = lib.towr_gpu_debug_stamp_kernel(i)
        if n is None:
            break
        names.append(n.decode().replace("void tg::(anonymous namespace)::", "").split("(")[0])
    lib.towr_gpu_debug_stamps(None)
    S = buf.cpu().numpy().reshape(NREG, -1, 8, 8)   # region, block, wave, phase
    starts = [int(S[i][S[i] > 0].min()) for i in range(len(names)) if (S[i] > 0).any()]
    if not starts:
        print("no stamps recorded (launches: %s)" % names)
        return
    t0 = min(starts)
    for i, nm in enumerate(names):
        R = S[i]
        used = (R[:, :, :] > 0).any(axis=(1, 2))
        R = R[used].astype(np.float64)
        if len(R) == 0:
            print(f"{nm}: no stamps")
            continue
        R[R == 0] = np.nan
        rel = (R - t0) * TICK_US
        start = np.nanmin(rel[:, :, 0], axis=1)
        last = np.nanmax(rel.reshape(len(R), -1), axis=1)
        print(f"{nm}: {len(R)} blocks, first start {np.nanmin(start):.1f} us, last end {np.nanmax(last):.1f} us, "
              f"block life median {np.nanmedian(last - start):.1f} p90 {np.nanpercentile(last - start, 90):.1f} us")
        ks = [k for k in range(8) if not np.isnan(rel[:, :, k]).all()]
        # phases between consecutive stamps in time order (the slowest wave's stamps, median over blocks)
        ks.sort(key=lambda k: np.nanmedian(np.nanmax(rel[:, :, k], axis=1)))
        for k0, k1 in zip(ks, ks[1:]):
            a = np.nanmax(rel[:, :, k0], axis=1)
            b = np.nanmax(rel[:, :, k1], axis=1)
            d = b - a
            print(f"    phase {k0}->{k1}: median {np.nanmedian(d):7.2f} us  p90 {np.nanpercentile(d, 90):7.2f} us")
        # start histogram: how many blocks start in each 20 us window
        h, e = np.histogram(start, bins=np.arange(0, np.nanmax(last) + 20, 20))
        print("    starts per 20 us: " + " ".join(str(x) for x in h))


if __name__ == "__main__":
    main()
