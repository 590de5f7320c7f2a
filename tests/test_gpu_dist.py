"""The sharded multi-process path on the GPU: 2 ranks (gloo process group, both on the box's one
GPU) each evaluate their shard of the bench batch with the device kernels, bench.py's way (rank r
owns problems [r*B, (r+1)*B), no data-path collective); the shards, gathered here for the check
only, equal the single-process device evaluation of the whole batch bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
B = 96


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _device_eval(first, count):
    import torch
    import bench
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    prob = TowrGpuProblem(F.anymal_trot().to_desc(), device=0)
    X, terrains = bench.make_batch(prob, count, first_id=first)
    prob.set_batch_terrain(terrains)
    dev = torch.device("cuda:0")
    G = torch.zeros((count, prob.m), dtype=torch.float64, device=dev)
    V = torch.zeros((count, prob.nnz), dtype=torch.float64, device=dev)
    prob.eval_batch_device(torch.from_numpy(np.ascontiguousarray(X[1])).to(dev), G, V)
    torch.cuda.synchronize()
    out = torch.cat([G, V], dim=1).cpu()
    prob.close()
    return out


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = _device_eval(bench.shard_first_id(rank, B), B)
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    wall, _ = bench.max_over_ranks(float(rank + 1), 0.0, True)
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), torch.cat(parts).numpy())
        np.save(os.path.join(outdir, "wall.npy"), np.array([wall]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_device_shards_match_single_process(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    whole = _device_eval(0, world * B).numpy()
    np.testing.assert_array_equal(np.load(tmp_path / "gathered.npy"), whole)
    assert np.load(tmp_path / "wall.npy")[0] == 2.0   # max over ranks
