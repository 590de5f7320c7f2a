"""bench.py — eval_g + eval_jac_g throughput of the MI355X engine on the ANYmal trot (2.4 s) batch.

Contract (see the task's bench section): `python bench.py --gpus N --steps K --warmup W`; for N>1
launched by torch.distributed.run, one rank per GPU. A "step" is one evaluation of g and every
Jacobian nonzero for the rank's batch of B independent ANYmal problems (the engine's launches: the
RangeOfMotion + ForceConstraintDiscretized fusion group, Dynamic, the small kinds) (BASELINE configs[2],
randomised start/goal/terrain as configs[4] describes). Inputs are resident in HBM before the timed
region; K steps are bracketed by barrier + synchronize, the max over ranks is taken, rank 0 prints
one JSON line. Weak scaling: B problems per GPU, no collective on the data path.

roofline: the dominant launch's algorithmic bytes (B x its CSR values + g rows written + distinct x
entries read, towr_gpu_kernel_info) over its average duration, measured with HIP events on the launch
stream; the whole step's 8 (n + m + nnz) bytes per problem over the step time beside it.
cpu_baseline: the CPU oracle (oracle/, a faithful C restatement of the reference path; kind
"port"), rank 0 at N=1 only, on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 20261015
N_X = 4          # pre-generated x sets cycled over (every step reads a different x)


def make_batch(prob, B, first_id, optimize_timings=False):
    """Randomised instances: start xy ~ U(-0.5,0.5), yaw ~ U(-0.3,0.3);
    goal = start + (U(1.5,2.5), U(-0.3,0.3)); terrain Flat(h~U(0,0.3)) or Stairs(start~U(0.8,1.4),
    heights~U(0.1,0.25)); x = x0 + sigma * N(0,1) per variable-set kind. With optimize_timings (the
    phase-duration variables of BASELINE configs[3]) the durations get +-3 % multiplicative noise."""
    from towr2025_amd import formulation as F
    from towr2025_amd import _capi as capi
    sig_kind = {capi.VAR_BASE_LIN: 0.05, capi.VAR_BASE_ANG: 0.1, capi.VAR_EE_MOTION: 0.05,
                capi.VAR_EE_ANG: 0.1, capi.VAR_EE_FORCE: 20.0, capi.VAR_EE_TORQUE: 1.0}
    sigma = np.zeros(prob.n)
    sched = np.zeros(prob.n, dtype=bool)
    for kind, _ee, c0, n in prob.varset_info():
        if kind == capi.VAR_EE_SCHEDULE:
            sched[c0:c0 + n] = True
        else:
            sigma[c0:c0 + n] = sig_kind[kind]
    X = np.zeros((N_X, B, prob.n))
    terrains = []
    for b in range(B):
        rng = np.random.default_rng(SEED + first_id + b)
        sx, sy = rng.uniform(-0.5, 0.5, 2)
        syaw = rng.uniform(-0.3, 0.3)
        gx, gy = sx + rng.uniform(1.5, 2.5), sy + rng.uniform(-0.3, 0.3)
        if rng.uniform() < 0.5:
            ter = F.HeightMap.Flat(rng.uniform(0.0, 0.3))
        else:
            ter = F.HeightMap(F.HeightMap.StairsID, (rng.uniform(0.8, 1.4), 0.4, rng.uniform(0.1, 0.25),
                                                     rng.uniform(0.1, 0.25), 1.0))
        f = F.anymal_trot(goal=(gx, gy, 0.0), terrain=ter, start_xy=(sx, sy), start_yaw=syaw, goal_yaw=syaw,
                          optimize_timings=optimize_timings)
        d = f.to_desc()
        x0 = prob.initial_x_for(d.init, d.terrain)
        for k in range(N_X):
            X[k, b] = x0 + sigma * rng.standard_normal(prob.n)
            X[k, b, sched] = x0[sched] * (1.0 + 0.03 * rng.standard_normal(int(sched.sum())))
        terrains.append(d.terrain)
    return X, terrains


def shard_first_id(rank, B):
    """Rank r owns problems [r*B, (r+1)*B) of the global batch (weak scaling, no collective)."""
    return rank * B


def max_over_ranks(wall, kern_ms, distributed):
    """Timing reduction: the slowest rank defines the job time (gloo, host tensors: the data path has no
    collective, so RCCL is never initialised)."""
    if not distributed:
        return wall, kern_ms
    import torch
    import torch.distributed as dist
    t = torch.tensor([wall, kern_ms], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])


def host_cpus():
    """The measuring host's CPUs: lscpu sockets x cores per socket x threads per core, the CPUs this
    process may run on (affinity), and the cgroup CPU quota (the GPU box grants each job a share)."""
    info = {"sockets": None, "cores_per_socket": None, "threads_per_core": None, "model": None}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        keys = {"Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "Model name": "model"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                v = v.strip()
                info[keys[k.strip()]] = int(v) if v.isdigit() else v
    except Exception:
        pass
    info["affinity"] = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    info["cgroup_quota_cpus"] = quota
    if isinstance(info["sockets"], int) and isinstance(info["cores_per_socket"], int):
        info["physical_cores"] = info["sockets"] * info["cores_per_socket"]
    else:
        info["physical_cores"] = None
    return info


def cpu_baseline(desc, X, seconds):
    """The oracle (built -O3 -march=native on this host) timed on this host's cores, one
    independent problem per thread. Threads = every physical core this job may use: the affinity
    set, capped by the cgroup CPU quota (more threads than the quota only time-slice) and by the
    physical core count (no SMT siblings)."""
    from oracle import oracle as O
    cpus = host_cpus()
    threads = cpus["affinity"]
    for cap in (cpus["cgroup_quota_cpus"], cpus["physical_cores"]):
        if cap:
            threads = min(threads, cap)
    threads = max(1, threads)
    O.bench(desc, 1, 3, X, native=True)                    # builds liboracle_native.so, warms caches
    t1, _ = O.bench(desc, 1, 20, X, native=True)           # 1-thread per-call time
    per_call = t1 / 20
    calls = max(4, int(seconds / per_call))
    secs, done = O.bench(desc, threads, calls, X, native=True)
    rate = done / secs
    phys = cpus["physical_cores"]
    return {"value": rate, "unit": "calls/s", "cores": threads, "kind": "port",
            "one_thread": 1.0 / per_call, "host": cpus,
            "all_physical_cores_extrapolated": (rate / threads * phys) if phys else None,
            "sample": f"{done} calls ({calls}/thread x {threads} threads) of the CPU oracle (oracle/towr_oracle.c, "
                      f"gcc -O3 -march=native on this host) on ANYmal trot x-vectors, {secs:.1f} s wall; "
                      f"1 thread {1.0 / per_call:.1f} calls/s; threads = min(affinity {cpus['affinity']}, "
                      f"cgroup quota {cpus['cgroup_quota_cpus']}, physical cores {phys})"}


def single_call(prob, X, reps=300, register=True):
    """B = 1 latency: towr_gpu_eval_g_jac through host pointers (what IpoptAdapter::eval_g + eval_jac_g
    drive per iteration, hopper_example.cc:175-180): H2D of x, one launch, D2H of g and the values.
    register: the g / values arrays are page-locked once (towr_gpu_register_host), as the C++
    NlpCallbacks cache is, so the D2H lands in place; x comes from an unregistered array each call."""
    x = [np.ascontiguousarray(X[k]) for k in range(len(X))]
    g, v = np.zeros(prob.m), np.zeros(prob.nnz)
    if register:
        prob.register_host(g)
        prob.register_host(v)
    for k in range(20):
        prob.eval_g_jac_into(x[k % len(x)], g, v)
    ts = []
    for k in range(reps):
        t0 = time.perf_counter()
        prob.eval_g_jac_into(x[k % len(x)], g, v)
        ts.append(time.perf_counter() - t0)
    if register:
        prob.unregister_host(g)
        prob.unregister_host(v)
    ts = np.array(ts) * 1e6
    return {"us_median": float(np.median(ts)), "us_p10": float(np.percentile(ts, 10)),
            "us_p90": float(np.percentile(ts, 90)), "calls": reps, "registered_outputs": register}


def single_leg(desc, name, note, device, reps=300, cpu=True, sigma=0.02):
    """B = 1 latency of one BASELINE configuration (single_call, registered outputs) beside the oracle's
    one-thread time per eval_g + eval_jac_g on the same x vectors."""
    from towr2025_amd import TowrGpuProblem
    p = TowrGpuProblem(desc, device=device)
    x0 = p.initial_x()
    rng = np.random.default_rng(SEED)
    X = np.stack([x0 + sigma * np.abs(x0).clip(0.1, 1.0) * rng.standard_normal(p.n) for _ in range(N_X)])
    out = single_call(p, X, reps=reps)
    out.update({"config": name, "n": p.n, "m": p.m, "nnz": p.nnz, "note": note})
    if cpu:
        from oracle import oracle as O
        O.bench(desc, 1, 2, X, native=True)
        secs, done = O.bench(desc, 1, 10, X, native=True)
        out["cpu_one_thread_us"] = secs / done * 1e6
        out["speedup_vs_cpu_one_thread"] = out["cpu_one_thread_us"] / out["us_median"]
    p.close()
    return out


def pattern_watch(Xd, B, device, reps=3):
    """towr_gpu_pattern_outside_batch_device on B ANYmal problems with randomised Gap terrains (the curved
    terrain whose reference pattern moves with x): a synchronous host pass — X copied to the host, the
    watched instants evaluated on up to 16 host threads with the reference's operations (include/towr_gpu.h)."""
    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    p = TowrGpuProblem(F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.GapID)).to_desc(), device=device)
    rng = np.random.default_rng(SEED)
    p.set_batch_terrain([F.HeightMap(F.HeightMap.GapID, (rng.uniform(0.9, 1.1), rng.uniform(0.45, 0.55),
                                                         rng.uniform(1.2, 1.6))).to_c() for _ in range(B)])
    counts = np.zeros(B, dtype=np.int32)
    p.pattern_outside_batch(Xd, counts)
    t0 = time.perf_counter()
    for _ in range(reps):
        p.pattern_outside_batch(Xd, counts)
    ms = (time.perf_counter() - t0) / reps * 1e3
    p.close()
    return {"ms_per_batch": ms, "problems": B, "value": B / (ms * 1e-3), "unit": "problems/s",
            "entries_outside_total": int(counts.sum()),
            "note": "host pass (D2H of X, up to 16 host threads), ANYmal on randomised Gap terrains, the headline's x"}


def host_batch(prob, Xh, reps=3):
    """PCIe-inclusive rate of towr_gpu_eval_batch (host X, G, V; the caller's G / V reused across
    calls): through the pinned staging, and with G / V registered (in-place DMA)."""
    B = Xh.shape[1]
    G, V = np.zeros((B, prob.m)), np.zeros((B, prob.nnz))
    out = {}
    for reg in (False, True):
        if reg:
            prob.register_host(G)
            prob.register_host(V)
        prob.eval_batch(Xh[0], G, V)
        t0 = time.perf_counter()
        for i in range(reps):
            prob.eval_batch(Xh[i % len(Xh)], G, V)
        th = (time.perf_counter() - t0) / reps
        out["registered" if reg else "staged"] = {"value": B / th, "ms_per_batch": th * 1e3,
                                                   "GB/s_d2h": B * 8 * (prob.m + prob.nnz) / th / 1e9}
    prob.unregister_host(G)
    prob.unregister_host(V)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 5 warmup steps leave the clocks ramping inside the timed region (0.287 ms per step vs 0.255 ms
    # after 50 warmup steps, same box): the defaults warm up for ~13 ms of work first
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="after the W warmup steps, keep running untimed steps until this much wall time has "
                         "passed since warmup began (GPU clocks ramp up over the first ~100 ms)")
    ap.add_argument("--batch", type=int, default=4096, help="problems per GPU (weak scaling)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--no-gait", action="store_true", help="skip the phase-duration optimisation figure")
    ap.add_argument("--tiles-per-block", type=int, default=0)
    ap.add_argument("--legs", default=None, help="A/B runs: comma-separated side legs to measure (objective, "
                                                 "gait_optimization, gait_torque, rotvec, pattern_watch); default all")
    args = ap.parse_args()
    legs = set(args.legs.split(",")) if args.legs else None

    def want(leg):
        return legs is None or leg in legs

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torch.distributed.run (RANK set) the process group is used at every world size, so the
    # launcher path the multi-GPU runs take is the one a 1-GPU run under the launcher exercises
    distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    if distributed:   # timing barrier + max-over-ranks only: gloo (the problem shards never communicate)
        dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from towr2025_amd import TowrGpuProblem
    from towr2025_amd import formulation as F
    desc = F.anymal_trot().to_desc()
    prob = TowrGpuProblem(desc, device=local)
    if args.tiles_per_block:
        prob.set_tiles_per_block(args.tiles_per_block)
    B = args.batch
    Xh, terrains = make_batch(prob, B, first_id=shard_first_id(rank, B))
    prob.set_batch_terrain(terrains)
    ldv = (prob.nnz + 15) // 16 * 16
    ldg = (prob.m + 15) // 16 * 16
    X = torch.from_numpy(Xh).to(dev)
    G = torch.empty((B, ldg), dtype=torch.float64, device=dev)
    V = torch.empty((B, ldv), dtype=torch.float64, device=dev)
    stream = torch.cuda.Stream(dev)          # kernels and timing events share this stream
    torch.cuda.set_stream(stream)

    def step(i):
        prob.eval_batch_device(X[i % N_X], G, V, stream=stream)

    tw = time.perf_counter()
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    settle = 0
    while (time.perf_counter() - tw) * 1e3 < args.settle_ms:
        for i in range(8):
            step(i)
        settle += 8
        torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for i in range(args.steps):
        step(i)
    e1.record(stream)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / args.steps
    wall, kern_ms = max_over_ranks(wall, kern_ms, distributed)

    calls = B * world * args.steps
    value = calls / wall
    bytes_call = prob.algorithmic_bytes_per_call()
    step_gbs = B * bytes_call / (kern_ms * 1e-3) / 1e9
    peak = 8000.0
    # per-kernel durations (each launch class alone, and each fusion group), HIP events on the launch
    # stream; the roofline's kernel is the longest of the launches one step actually makes
    kernels = {}
    reps = max(5, args.steps // 2)
    # the side legs (objective, phase-duration optimisation, RotVec): untimed warm-up calls, then at least
    # 20 timed ones (a leg follows other work, and its first calls settle caches and clocks)
    leg_warm, leg_reps = 20, max(20, args.steps // 2)
    step_ks = set(prob.step_launches())
    step_names = []
    for k, name, nt, by in prob.kernels():
        if k in step_ks:
            step_names.append(name)
        for i in range(2):
            prob.eval_batch_device_kernel(k, X[i % N_X], G, V, stream)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(reps):
            prob.eval_batch_device_kernel(k, X[i % N_X], G, V, stream)
        z.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(z) / reps
        kernels[name] = {"ms": ms, "bytes_per_launch": B * by, "GB/s": B * by / (ms * 1e-3) / 1e9, "tiles_per_problem": nt}
    dom = max(step_names, key=lambda n: kernels[n]["ms"])
    achieved = kernels[dom]["GB/s"]
    out = {
        "metric": "full eval_g+eval_jac_g calls/sec, ANYmal trot 2.4s horizon; 1/2/4/8-GPU batch",
        "value": value, "unit": "calls/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "warmup_settle": {"extra_untimed_steps": settle, "settle_ms": args.settle_ms},
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: randomised ANYmal trot instances (start/goal/terrain), x = x0 + seeded noise",
        "config": {"workload": "ANYmal trot 2.4s (quadruped C1), NlpFormulation defaults, batch of independent problems",
                   "problems_per_gpu": B, "n": prob.n, "m": prob.m, "nnz": prob.nnz,
                   "calls_per_step": B * world, "terrains": "Flat(h~U(0,0.3)) | Stairs(randomised)",
                   "parallelism": f"dp{world} (problem shards, no collective)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
                     "frac": achieved / peak, "traffic": None,
                     "kernel": dom, "kernel_ms": kernels[dom]["ms"], "bytes_per_launch": kernels[dom]["bytes_per_launch"],
                     "step": {"ms": kern_ms, "bytes": B * bytes_call, "GB/s": step_gbs, "frac": step_gbs / peak,
                              "launches": step_names},
                     "kernels": kernels},
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as fh:
                rec = json.load(fh)
            k = rec.get("kernels", {}).get(dom)
            if k and k.get("problems_per_launch", rec.get("problems_per_launch")) == B:
                out["roofline"]["traffic"] = k["hbm_bytes_per_launch"]
                out["roofline"]["traffic_source"] = rec.get("source")
        except Exception:
            pass
    if rank == 0 and want("objective"):
        # the objective callbacks on the same batch: every cost kind of
        # NlpFormulation::GetCosts on this formulation; one eval_f + eval_grad_f per problem
        cdesc = F.with_costs(F.anymal_trot()).to_desc()
        cprob = TowrGpuProblem(cdesc, device=local)
        cprob.set_batch_terrain(terrains)
        Fo = torch.empty(B, dtype=torch.float64, device=dev)
        Go = torch.empty((B, (prob.n + 15) // 16 * 16), dtype=torch.float64, device=dev)
        for i in range(leg_warm):
            cprob.eval_cost_batch_device(X[i % N_X], Fo, Go, stream)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(leg_reps):
            cprob.eval_cost_batch_device(X[i % N_X], Fo, Go, stream)
        z.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(z) / leg_reps
        cbytes = 8 * (2 * prob.n + 1)
        out["objective"] = {"value": B / (ms * 1e-3), "unit": "eval_f+eval_grad_f calls/s", "ms_per_batch": ms,
                            "cost_terms": cdesc.n_costs, "bytes_per_call": cbytes,
                            "GB/s": B * cbytes / (ms * 1e-3) / 1e9,
                            "note": "ANYmal trot + Forces/EEMotion/Energy/AngularMomentum/EEBasePos costs, same batch"}
        cprob.close()
    def batch_leg(lprob, Xl, Bl, ter):
        """ms per eval_batch_device of Bl problems (leg_warm untimed calls, then leg_reps timed ones, HIP
        events on the launch stream), cycling over the x sets Xl (device tensors)."""
        lprob.set_batch_terrain(ter)
        Gl = torch.empty((Bl, (lprob.m + 15) // 16 * 16), dtype=torch.float64, device=dev)
        Vl = torch.empty((Bl, (lprob.nnz + 15) // 16 * 16), dtype=torch.float64, device=dev)
        for i in range(leg_warm):
            lprob.eval_batch_device(Xl[i % len(Xl)], Gl, Vl, stream=stream)
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for i in range(leg_reps):
            lprob.eval_batch_device(Xl[i % len(Xl)], Gl, Vl, stream=stream)
        z.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(z) / leg_reps
        lb = lprob.algorithmic_bytes_per_call()
        return {"value": Bl / (ms * 1e-3), "unit": "calls/s", "ms_per_batch": ms, "problems": Bl,
                "n": lprob.n, "m": lprob.m, "nnz": lprob.nnz, "GB/s": Bl * lb / (ms * 1e-3) / 1e9}

    if rank == 0 and not args.no_gait:
        # BASELINE configs[3]'s formulation (phase-duration optimisation: PhaseSplines with x-dependent
        # durations, schedule Jacobian columns) on a batch of the same randomised instances
        Bg = min(B, 1024)
        for key, f, note in (
                ("gait_optimization", F.anymal_trot(optimize_timings=True),
                 "BASELINE configs[3] formulation (ANYmal, phase-duration optimisation), randomised Flat/Stairs "
                 "instances, durations +-3 %"),
                ("gait_torque", F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True),
                 "the same + Parameters::Torque (TorqueConstraintDiscretized per foot, dt 0.02, on the record + "
                 "compose path), the formulation class of the fork's hopper driver (hopper_example.cc:145-150)")):
            if not want(key):
                continue
            if key == "gait_torque":
                f.params_.constraints_.append(F.Parameters.Torque)
            gprob = TowrGpuProblem(f.to_desc(), device=local)
            Xg, gter = make_batch(gprob, Bg, first_id=shard_first_id(rank, Bg), optimize_timings=True)
            out[key] = batch_leg(gprob, [torch.from_numpy(Xg[k]).to(dev) for k in range(2)], Bg, gter)
            out[key]["note"] = note
            gprob.close()
    if rank == 0 and not args.no_gait and want("rotvec"):
        # RotVecConverter base orientation (Parameters::RotationVector) on the same
        # randomised instances: the headline formulation with the rotation-vector base parameterisation
        fr = F.anymal_trot()
        fr.params_.angular_rep_ = 1
        rprob = TowrGpuProblem(fr.to_desc(), device=local)
        out["rotvec"] = batch_leg(rprob, [X[k] for k in range(N_X)], B, terrains)
        out["rotvec"]["note"] = ("ANYmal trot with the RotVecConverter base orientation (angular_rep = 1), the "
                                 "headline's randomised instances and x")
        rprob.close()
    if rank == 0 and not args.no_gait and want("pattern_watch"):
        # the frozen-pattern check (towr_gpu_pattern_outside_batch_device, a host pass) on a Gap batch
        out["pattern_watch"] = pattern_watch(X[0], B, local)
    if rank == 0 and not args.no_host:
        # PCIe-inclusive rate through the host-buffer entry point (towr_gpu_eval_batch: H2D of X,
        # chunked launches, D2H of G and V overlapping the next chunk) — reported beside, never as `value`
        hb = host_batch(prob, Xh)
        out["host_batch"] = {"value": hb["staged"]["value"], "unit": "calls/s", "ms_per_batch": hb["staged"]["ms_per_batch"],
                             "registered": hb["registered"], "staged": hb["staged"],
                             "note": "host X/G/V buffers, PCIe transfers included (per GPU); value = through the pinned "
                                     "staging, 'registered' = G/V page-locked by towr_gpu_register_host"}
    if rank == 0 and not args.no_host:
        out["single_call"] = single_call(prob, Xh[:, 0])
        out["single_call"]["staged_outputs_us_median"] = single_call(prob, Xh[:, 0], reps=100, register=False)["us_median"]
        out["single_call"]["note"] = ("B = 1 through host pointers (towr_gpu_eval_g_jac): H2D x, one launch, D2H g + "
                                      "values into registered arrays; per problem, the latency IPOPT sees per "
                                      "eval_g + eval_jac_g pair")
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(desc, Xh[0, :8], args.cpu_seconds)
        if "single_call" in out:
            out["single_call"]["cpu_one_thread_us"] = 1e6 / out["cpu_baseline"]["one_thread"]
    if rank == 0 and not args.no_host:
        # B = 1 latency of the other single-problem configurations: BASELINE configs[1] (biped walk 2 s)
        # and configs[3] (ANYmal on stairs with phase-duration optimisation, the fork's hopper driver's
        # formulation class, hopper_example.cc:145-180), each beside the oracle's one-thread time
        cpu = world == 1 and not args.no_cpu
        out["single_call_biped"] = single_leg(F.biped_walk().to_desc(), "BASELINE configs[1]: biped walk 2 s",
                                              "B = 1 through host pointers, registered outputs", local, cpu=cpu)
        out["single_call_gait"] = single_leg(
            F.anymal_trot(terrain=F.HeightMap.MakeTerrain(F.HeightMap.StairsID), optimize_timings=True).to_desc(),
            "BASELINE configs[3]: ANYmal on stairs, phase-duration optimisation",
            "B = 1 through host pointers, registered outputs", local, cpu=cpu)
        out["single_call_hopper_gait"] = single_leg(
            F.hopper_example_desc(), "the fork's hopper driver (hopper_example.cc:95-171): monoped, FiveStepStairs, "
            "Torque, phase-duration optimisation", "B = 1 through host pointers, registered outputs", local, cpu=cpu)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
