"""A/B of engine builds / environment switches on one GPU box: alternating runs of bench.py itself (the driver's
program: its x sets, leg order and reps), 3 rounds. The default arguments are the driver's flags.
A measurement tool, not part of the product.
usage: python tools/ab.py TAG "name:VAR=v,VAR2=v2" "name2:TOWR_GPU_LIB=tools/build/libtowr_gpu_x.so" ...
       [--args "--steps 20 --warmup 5 --no-cpu --no-host --legs objective,gait_optimization"] [--rounds 3]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEGS = ("objective", "gait_optimization", "gait_torque", "rotvec")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("cfgs", nargs="+")
    ap.add_argument("--args", default="--steps 20 --warmup 5 --no-cpu --no-host "
                                      "--legs objective,gait_optimization,gait_torque,rotvec")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    res = {}
    for r in range(a.rounds):
        for cfg in a.cfgs:
            name, _, kv = cfg.partition(":")
            env = dict(os.environ)
            for item in filter(None, kv.split(",")):
                k, _, v = item.partition("=")
                env[k] = os.path.join(ROOT, v) if k == "TOWR_GPU_LIB" else v
            log = os.path.join(ROOT, "gpurun_out", f"{a.tag}_{name}_{r}.log")
            with open(log, "w") as f:
                rc = subprocess.call(["timeout", "-k", "10", "240", sys.executable, "bench.py"] + a.args.split(),
                                     cwd=ROOT, env=env, stdout=f, stderr=subprocess.STDOUT)
            if rc != 0:
                print(f"{name} round {r}: rc {rc}", flush=True)
                sys.exit(rc)
            line = [l for l in open(log) if l.startswith("{")][-1]
            j = json.loads(line)
            ks = j["roofline"]["kernels"]
            legs = {k: j[k]["ms_per_batch"] for k in LEGS if k in j}
            res.setdefault(name, []).append((j["ms_per_step"], {k: v["ms"] for k, v in ks.items()}, legs))
            print(f"{name:12s} r{r} step {j['ms_per_step']:.4f} ms  " +
                  "  ".join(f"{k} {v['ms']:.4f}" for k, v in ks.items()) +
                  "".join(f"  {k} {v:.4f}" for k, v in legs.items()), flush=True)
    for name, v in res.items():
        steps = sorted(s for s, _, _ in v)
        line = f"== {name}: step {steps[0]:.4f}-{steps[-1]:.4f} ms"
        for k in LEGS:
            xs = sorted(l[k] for _, _, l in v if k in l)
            if xs:
                line += f" | {k} {xs[0]:.4f}-{xs[-1]:.4f}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
