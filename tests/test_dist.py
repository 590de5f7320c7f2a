"""Multi-process (N>1) path of bench.py on CPU with the gloo backend, world_size 2.

The batch of independent problems is the only parallel axis: rank r owns problems
[r*B, (r+1)*B) with no data-path collective; the only collectives are the timing barrier and the
max-over-ranks reduction. Checked here: the shards partition exactly the single-process batch
(same seeded instances, same x sets, same terrains), and the timing reduction takes the max."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

B = 3


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import bench
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    dist.init_process_group("gloo", rank=rank, world_size=world)
    prob = TowrGpuProblem(F.anymal_trot().to_desc(), device=-1)   # layout only: no GPU here
    first = bench.shard_first_id(rank, B)
    X, terrains = bench.make_batch(prob, B, first_id=first)
    np.save(os.path.join(outdir, f"x{rank}.npy"), X)
    np.save(os.path.join(outdir, f"t{rank}.npy"), np.array([[t.id, *list(t.p)] for t in terrains]))
    wall, kern = bench.max_over_ranks(float(rank + 1), 10.0 * (rank + 1), world > 1)
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.array([wall, kern]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_partition_the_batch(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    import bench
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    prob = TowrGpuProblem(F.anymal_trot().to_desc(), device=-1)
    X, terrains = bench.make_batch(prob, world * B, first_id=0)
    Xs = np.concatenate([np.load(tmp_path / f"x{r}.npy") for r in range(world)], axis=1)
    np.testing.assert_array_equal(Xs, X)
    T = np.concatenate([np.load(tmp_path / f"t{r}.npy") for r in range(world)])
    np.testing.assert_array_equal(T, np.array([[t.id, *list(t.p)] for t in terrains]))
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"r{r}.npy"), [2.0, 20.0])


def _emu_lib():
    import ctypes as C
    import subprocess
    from towr2025_amd import _capi as capi
    here = os.path.dirname(os.path.abspath(__file__))
    lib = os.path.join(here, "host_emu", "build", "libemu.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-C", os.path.join(here, "host_emu")])
    L = C.CDLL(lib)
    D = C.POINTER(C.c_double)
    L.emu_eval.argtypes = [C.POINTER(capi.ProblemDesc), D, D, D, C.c_char_p, C.c_int]
    return L


def _eval_shard(first, count, x_set=1):
    """g and J values of problems [first, first + count) of the bench batch through the engine's item
    math on the host (tests/host_emu): each problem on its own terrain."""
    import ctypes as C
    import bench
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    emu = _emu_lib()
    prob = TowrGpuProblem(F.anymal_trot().to_desc(), device=-1)
    X, terrains = bench.make_batch(prob, count, first_id=first)
    D = C.POINTER(C.c_double)
    G, V = np.zeros((count, prob.m)), np.zeros((count, prob.nnz))
    for b in range(count):
        d = F.anymal_trot().to_desc()
        d.terrain = terrains[b]
        x = np.ascontiguousarray(X[x_set, b])
        err = C.create_string_buffer(256)
        assert emu.emu_eval(C.byref(d), x.ctypes.data_as(D), G[b].ctypes.data_as(D), V[b].ctypes.data_as(D), err, 256) == 0, err.value
    return G, V


def _eval_worker(rank, world, port, outdir):
    """One rank of the sharded evaluation: its problems only, no data-path collective; the results
    are gathered here for the check alone (gloo all_gather), the timing reduction as in bench.py."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G, V = _eval_shard(bench.shard_first_id(rank, B), B)
    gathered = [torch.zeros(B, G.shape[1] + V.shape[1], dtype=torch.float64) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(np.concatenate([G, V], axis=1)))
    if rank == 0:
        np.save(os.path.join(outdir, "gathered.npy"), torch.cat(gathered).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_evaluate_the_batch(tmp_path):
    """Each of 2 gloo ranks evaluates its shard (the engine's item math, host emulation); the gathered
    shards equal the single-process evaluation of the whole batch bit for bit."""
    _emu_lib()   # build once, before the ranks start
    world = 2
    mp.spawn(_eval_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    G, V = _eval_shard(0, world * B)
    got = np.load(tmp_path / "gathered.npy")
    np.testing.assert_array_equal(got, np.concatenate([G, V], axis=1))
