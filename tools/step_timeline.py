"""Timeline of one step of a rocprofv3 kernel trace around the N-th-from-last launch of a kernel:
python tools/step_timeline.py gpurun_out/DIR/run_kernel_trace.csv KERNEL_SUBSTRING [nth_from_last] [before] [after]
A measurement tool."""
import csv
import sys


def short(n):
    return n.replace("void tg::(anonymous namespace)::", "").replace("tg::(anonymous namespace)::", "").split("(")[0]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2]
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 3
before = int(sys.argv[4]) if len(sys.argv) > 4 else 3
after = int(sys.argv[5]) if len(sys.argv) > 5 else 12
idx = [i for i, r in enumerate(rows) if key in r["Kernel_Name"]]
i = idx[-nth]
t0 = int(rows[i - before]["Start_Timestamp"])
for r in rows[i - before:i + after]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    nb = int(r["Grid_Size_X"]) // max(int(r["Workgroup_Size_X"]), 1)
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  q{r['Queue_Id']} {nb:6d}x{r['Workgroup_Size_X']:4s} {short(r['Kernel_Name'])}")
