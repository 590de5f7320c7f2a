"""Per-kernel durations and the last steps' timeline from a rocprofv3 kernel trace (the rocpd SQLite database
rocprofv3 writes by default, or a kernel_trace.csv): python tools/trace_summ.py gpurun_out/DIR [launches_per_step]
A measurement tool."""
import csv
import glob
import sqlite3
import sys
from collections import defaultdict


def short(n):
    return n.replace("void tg::(anonymous namespace)::", "").replace("tg::(anonymous namespace)::", "").split("(")[0]


def load(d):
    dbs = sorted(glob.glob(f"{d}/**/*.db", recursive=True))
    if dbs:
        cur = sqlite3.connect(dbs[-1]).cursor()
        return [(short(n), int(s), int(e), int(v), int(g), int(w), int(l)) for n, s, e, v, g, w, l in
                cur.execute("select name, start, end, vgpr_count, grid_x, workgroup_x, lds_size from kernels order by start")]
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    return [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"]), 0, 0, 0, 0) for r in rows]


def main():
    rows = load(sys.argv[1])
    dur = defaultdict(list)
    info = {}
    for n, s, e, v, g, w, l in rows:
        dur[n].append(e - s)
        info[n] = (v, g // max(w, 1), w, l)
    for n, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        ds = sorted(ds)
        v, nb, w, l = info[n]
        print(f"{n[:72]:72s} n {len(ds):4d} median {ds[len(ds) // 2] / 1e3:8.1f} us  min {ds[0] / 1e3:8.1f}  vgpr {v:3d} blocks {nb:6d}x{w:3d} lds {l}")
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tail = rows[-3 * k:]
    t0 = tail[0][1]
    print("timeline of the last launches (us from the first):")
    for n, s, e, *_ in tail:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f}  {n[:80]}")


if __name__ == "__main__":
    main()
