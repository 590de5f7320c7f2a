"""B = 1 latency breakdown (GPU box): towr_gpu_eval_g_jac with registered g / values, timed per call;
then the same call's pieces in isolation on torch device buffers: the kernel alone (eval_batch_device,
B = 1, synchronised), an 8.7 kB H2D, the g + values D2H into pinned memory.
Usage: python tools/single_probe.py [gait] [--lib tools/build/libtowr_gpu_x.so]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from towr2025_amd import TowrGpuProblem, formulation as F  # noqa: E402


def med(f, reps=300):
    for _ in range(20):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e6)


gait = "gait" in sys.argv[1:]
if "--lib" in sys.argv:   # an experiment / baseline build under tools/build
    from towr2025_amd import _capi
    _capi.load_library(sys.argv[sys.argv.index("--lib") + 1])
p = TowrGpuProblem(F.anymal_trot(optimize_timings=gait).to_desc())
x = p.initial_x()
g, v = np.zeros(p.m), np.zeros(p.nnz)
p.register_host(g)
p.register_host(v)
out = {"call_registered_us": med(lambda: p.eval_g_jac_into(x, g, v))}
g2, v2 = np.zeros(p.m), np.zeros(p.nnz)
out["call_staged_us"] = med(lambda: p.eval_g_jac_into(x, g2, v2))
dev = torch.device("cuda:0")
s = torch.cuda.Stream(dev)
Xd = torch.from_numpy(x.reshape(1, -1).copy()).to(dev).contiguous()
Gd = torch.zeros((1, p.m), dtype=torch.float64, device=dev)
Vd = torch.zeros((1, p.nnz), dtype=torch.float64, device=dev)


def kern():
    p.eval_batch_device(Xd, Gd, Vd, stream=s)
    s.synchronize()


out["batch_device_B1_kernel_us"] = med(kern)
xp = torch.from_numpy(x).pin_memory()
gp = torch.zeros(p.m, dtype=torch.float64).pin_memory()
vp = torch.zeros(p.nnz, dtype=torch.float64).pin_memory()


def h2d():
    with torch.cuda.stream(s):
        Xd[0].copy_(xp, non_blocking=True)
    s.synchronize()


def d2h():
    with torch.cuda.stream(s):
        gp.copy_(Gd[0], non_blocking=True)
        vp.copy_(Vd[0], non_blocking=True)
    s.synchronize()


def empty():
    s.synchronize()


out["h2d_x_us"] = med(h2d)
out["d2h_g_values_us"] = med(d2h)
out["sync_only_us"] = med(empty)
for k, name, nt, by in p.kernels():   # each launch class alone at B = 1, device outputs
    out[f"class_{name}_B1_us"] = med(lambda: (p.eval_batch_device_kernel(k, Xd, Gd, Vd, s), s.synchronize()), reps=200)
print(out)
