"""A/B of engine builds / environment switches on one GPU box: alternating bench runs, 3 rounds.
A measurement tool, not part of the product.
usage: python tools/ab.py TAG "name:VAR=v,VAR2=v2" "name2:TOWR_GPU_LIB=tools/build/libtowr_gpu_x.so" ...
       [--args "--steps 200 --warmup 20 --no-cpu --no-host --no-gait"] [--rounds 3]"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("cfgs", nargs="+")
    ap.add_argument("--args", default="--steps 200 --warmup 20 --no-cpu --no-host --no-gait")
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
            res.setdefault(name, []).append((j["ms_per_step"], {k: v["ms"] for k, v in ks.items()},
                                             j.get("gait_optimization", {}).get("ms_per_batch")))
            print(f"{name:12s} r{r} step {j['ms_per_step']:.4f} ms  " +
                  "  ".join(f"{k} {v['ms']:.4f}" for k, v in ks.items()) +
                  (f"  gait {res[name][-1][2]:.4f}" if res[name][-1][2] else ""), flush=True)
    for name, v in res.items():
        steps = sorted(s for s, _, _ in v)
        print(f"== {name}: step min {steps[0]:.4f} median {steps[len(steps) // 2]:.4f} ms")


if __name__ == "__main__":
    main()
