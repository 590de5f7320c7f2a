"""Objective-kernel breakdown on the GPU box (tool, not product): eval_f alone vs eval_f + eval_grad_f,
and each cost kind alone, on the bench batch (B = 4096 randomised ANYmal trot problems)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from towr2025_amd import TowrGpuProblem  # noqa: E402
from towr2025_amd import formulation as F  # noqa: E402

P = F.Parameters
B = int(os.environ.get("B", "4096"))
dev = torch.device("cuda", 0)
base = TowrGpuProblem(F.anymal_trot().to_desc(), device=0)
Xh, terrains = bench.make_batch(base, B, first_id=0)
X = torch.from_numpy(Xh).to(dev)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
variants = {
    "all": dict(),
    "forces": dict(costs=[(P.ForcesCostID, 1e-3)], ee_base_pos=False),
    "eemotion": dict(costs=[(P.EEMotionCostID, 0.5)], ee_base_pos=False),
    "energy": dict(costs=[(P.EnergyCostID, 1e-4)], ee_base_pos=False),
    "angmom": dict(costs=[(P.AngMomCostID, 0.1)], ee_base_pos=False),
    "eebasepos": dict(costs=[], ee_base_pos=True),
}
for name, kw in variants.items():
    p = TowrGpuProblem(F.with_costs(F.anymal_trot(), **kw).to_desc(), device=0)
    p.set_batch_terrain(terrains)
    Fo = torch.empty(B, dtype=torch.float64, device=dev)
    Go = torch.empty((B, (p.n + 15) // 16 * 16), dtype=torch.float64, device=dev)
    for grad in (False, True):
        for i in range(3):
            p.eval_cost_batch_device(X[i % 4], Fo, Go if grad else None, stream)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(30):
            p.eval_cost_batch_device(X[i % 4], Fo, Go if grad else None, stream)
        z.record(stream)
        torch.cuda.synchronize()
        print(f"{name:10s} grad={int(grad)}  {a.elapsed_time(z) / 30:.4f} ms", flush=True)
