"""Per-block phase timing of each launch class (stage x / evaluate / copy-out), from the
-DTOWR_PHASE_TIMING build of the engine (tools/build/libtowr_gpu_timing.so, `make -C
towr2025_amd/csrc timing`). Runs the bench workload (ANYmal trot, B problems) once per class and
prints mean phase durations in microseconds, the block lifetime and the mean number of resident
blocks. A measurement tool, not part of the product.
usage: python tools/phase_timing.py [--batch 4096] [--gait] [--rotvec]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--gait", action="store_true")
    ap.add_argument("--rotvec", action="store_true")
    ap.add_argument("--lib", default="libtowr_gpu_timing.so", help="library under tools/build")
    args = ap.parse_args()
    import torch
    from towr2025_amd import _capi as capi
    lib = capi.load_library(os.path.join(ROOT, "tools", "build", args.lib))
    lib.towr_gpu_debug_set_timing_buffer.argtypes = [C.c_void_p]
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    import bench
    f = F.anymal_trot(optimize_timings=args.gait)
    if args.rotvec:
        f.params_.angular_rep_ = 1
    prob = TowrGpuProblem(f.to_desc(), device=0)
    B = args.batch
    Xh, terrains = bench.make_batch(prob, B, 0) if not args.gait else (None, None)
    if Xh is None:
        x0 = prob.initial_x()
        Xh = np.stack([x0 + 0.01 * np.random.default_rng(b).standard_normal(prob.n) for b in range(B)])[None]
    else:
        prob.set_batch_terrain(terrains)
    dev = torch.device("cuda", 0)
    X = torch.from_numpy(np.ascontiguousarray(Xh[0])).to(dev)
    G = torch.empty((B, prob.m), dtype=torch.float64, device=dev)
    V = torch.empty((B, prob.nnz), dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    print(f"B={B} n={prob.n} m={prob.m} nnz={prob.nnz}  (us; mean over blocks)")
    lib.towr_gpu_debug_occupancy.argtypes = [C.c_void_p, C.c_int32]
    for lc in range(5):
        r = lib.towr_gpu_debug_occupancy(prob._h, lc)
        if r >= 0:
            print(f"  class {lc}: runtime max blocks/CU {r // 1000}, LDS {r % 1000} KiB")
    print(f"{'class':20s} {'blocks':>7s} {'stage':>7s} {'eval w0':>8s} {'w1':>6s} {'w2':>6s} {'w3':>6s} {'bar':>6s} "
          f"{'copy':>6s} {'life':>6s} {'span':>7s} {'resident':>8s}")
    for k, name, nt, _by in prob.kernels():
        if nt == 0:
            continue
        grid = ((B * nt + 7) // 8) * 8
        buf = torch.zeros(grid * 16, dtype=torch.int64, device=dev)
        lib.towr_gpu_debug_set_timing_buffer(None)
        for _ in range(3):
            prob.eval_batch_device_kernel(k, X, G, V, st)
        lib.towr_gpu_debug_set_timing_buffer(C.c_void_p(buf.data_ptr()))
        prob.eval_batch_device_kernel(k, X, G, V, st)
        torch.cuda.synchronize()
        lib.towr_gpu_debug_set_timing_buffer(None)
        t = buf.view(grid, 16).cpu().numpy().astype(np.float64)
        t = t[t[:, 9] > 0]
        real_life = (t[:, 9] - t[:, 0]) * 0.01              # s_memrealtime: 100 MHz -> us
        mem_life = t[:, 8] - t[:, 1]
        us_per_tick = np.sum(real_life) / np.sum(mem_life)
        stage = (t[:, 2] - t[:, 1]) * us_per_tick
        ev = [(t[:, 3 + w] - t[:, 2]) * us_per_tick for w in range(4)]
        ev = [e[t[:, 3 + w] > 0] for w, e in enumerate(ev)]
        bar = (t[:, 7] - np.max(t[:, 3:7], axis=1)) * us_per_tick
        copy = (t[:, 8] - t[:, 7]) * us_per_tick
        span = (t[:, 9].max() - t[:, 0].min()) * 0.01
        resident = real_life.sum() / span
        evs = [f"{(e.mean() if len(e) else 0.0):6.2f}" for e in ev]
        print(f"{name:20s} {len(t):7d} {stage.mean():7.2f} {evs[0]:>8s} {evs[1]} {evs[2]} {evs[3]} {bar.mean():6.2f} {copy.mean():6.2f} "
              f"{real_life.mean():6.2f} {span:7.1f} {resident:8.1f}")
        probes = [(s, t[:, s]) for s in range(10, 16) if (t[:, s] > 0).any()]
        if probes:   # engine_math.h TG_STAMP probes (wave 2), us after the staging barrier
            print("    probes (wave 2, us after staging): " +
                  "  ".join(f"[{s}] {((v[v > 0] - t[v > 0, 2]) * us_per_tick).mean():.2f}" for s, v in probes))


if __name__ == "__main__":
    main()
