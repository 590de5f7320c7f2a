"""Per-launch durations and the step timeline from a rocprofv3 kernel_trace.csv (the last N steps):
python tools/trace_summ.py gpurun_out/DIR [launches_per_step]. A measurement tool."""
import csv
import glob
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    f = sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        n = n.split("(")[0].replace("void tg::(anonymous namespace)::", "").replace("tg::(anonymous namespace)::", "")
        dur[n].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for n, v in sorted(dur.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
        ds = sorted(e - s for s, e in v)
        print(f"{n:70s} calls {len(v):4d} median {ds[len(ds) // 2] / 1e3:9.1f} us  min {ds[0] / 1e3:9.1f}")
    # the last 5 steps' timeline, relative to the first launch of the window
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tail = rows[-5 * k:]
    t0 = int(tail[0]["Start_Timestamp"])
    for r in tail:
        n = r["Kernel_Name"].split("(")[0].replace("void tg::(anonymous namespace)::", "").replace("tg::(anonymous namespace)::", "")
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {(int(r['End_Timestamp']) - t0) / 1e3:9.1f}  {n}")


if __name__ == "__main__":
    main()
