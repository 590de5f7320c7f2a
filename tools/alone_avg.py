"""Average duration of a kernel's dispatches that overlapped no other dispatch (a rocprofv3 kernel_trace.csv):
with Dynamic and the small kinds beside the fused launch, the bench's per-kernel loop (each launch class alone,
HIP events) is what the roofline quotes, and these are its dispatches. A measurement tool.
usage: python tools/alone_avg.py gpurun_out/DIR/run_kernel_trace.csv KERNEL_SUBSTRING [grid_blocks]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
grid = int(sys.argv[3]) if len(sys.argv) > 3 else None
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows]
alone, shared = [], []
for i, (s, e, r) in enumerate(iv):
    if key not in r["Kernel_Name"]:
        continue
    if grid is not None and int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1) != grid:
        continue
    ov = any(s2 < e and e2 > s for j, (s2, e2, _) in enumerate(iv[max(0, i - 8):i + 8]) if iv[max(0, i - 8) + j] is not iv[i])
    (shared if ov else alone).append((e - s) / 1e3)
for name, d in (("alone", alone), ("overlapped", shared)):
    if d:
        print(f"{name:10s} n {len(d):4d} avg {sum(d) / len(d):8.1f} us  min {min(d):8.1f}")
