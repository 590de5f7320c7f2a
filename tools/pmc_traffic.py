"""Per-launch HBM traffic of every tile kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE passes
(tools/gpu.sh pmc), written to profiles/pmc_traffic.json for bench.py's roofline.traffic. Every entry carries its
own problems per launch: the bench's headline and objective launches run B = 4096 problems, its phase-duration
legs (the gait_* entries) 1024.

FETCH_SIZE and WRITE_SIZE are in KiB. Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section), on
gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced reads — the kernels' only
HBM reads are the 16 B/lane x staging loads — so FETCH_SIZE is doubled; WRITE_SIZE is exact for
the 16 B/lane stores of the tile copy-out and is used as is.
usage: python tools/pmc_traffic.py gpurun_out/TAG_FETCH_SIZE gpurun_out/TAG_WRITE_SIZE out.json [B [B_gait]]"""
import csv
import json
import sys
from collections import defaultdict

NAMES = {0: "dynamic", 1: "range_of_motion", 2: "force_discretized", 10: "torque_discretized"}


def per_kernel(d, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if r["Counter_Name"] != counter:
            continue
        if "towr_misc_kernel" in k:
            acc["gait_small_kinds" if "towr_misc_kernel<true>" in k else "small_kinds"].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_step_kernel<" in k:   # <gait, rotvec, block>: the default 192-lane group is RangeOfMotion + FDISC
            targs = [a.strip() for a in k.split("towr_step_kernel<")[1].split(">")[0].split(",")]
            pre = ("gait_" if targs[0] == "true" else "") + ("rotvec_" if targs[1] == "true" else "")
            acc[pre + ("range_of_motion+force_discretized" if targs[2] == "192" else "fused_256")].append(
                float(r["Counter_Value"]) * 1024.0)
        elif "towr_tile_kernel<" in k:   # <type, block, gait, rotvec>: gait and RotVec launches reported apart
            targs = [a.strip() for a in k.split("towr_tile_kernel<")[1].split(">")[0].split(",")]
            t = int(targs[0])
            name = ("gait_" if targs[2] == "true" else "") + ("rotvec_" if targs[3] == "true" else "") + NAMES[t]
            acc[name].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_gait_frec_kernel" in k:   # phase-duration path: the FDISC (1) / TQDISC (4) / both (5) record launch
            roles = int(k.split("towr_gait_frec_kernel<")[1].split(">")[0]) if "towr_gait_frec_kernel<" in k else 1
            acc["gait_records_" + {1: "fdisc", 4: "tqdisc", 5: "fdisc+tqdisc"}[roles]].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_gait_rec_kernel" in k:   # the RangeOfMotion / Dynamic record launch (<rotvec, roles>)
            acc["gait_records"].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_gait_compose_kernel<" in k:   # <block, roles>: 1 FDISC, 2 RangeOfMotion, 4 Dynamic, 8 small kinds
            roles = int(k.split("towr_gait_compose_kernel<")[1].split(">")[0].split(",")[1])
            names = [n for bit, n in ((1, "fdisc"), (16, "tqdisc"), (2, "range_of_motion"), (4, "dynamic"), (8, "small_kinds")) if roles & bit]
            acc["gait_compose_" + "+".join(names)].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_rv_coef_kernel" in k:   # the RotVec base-angular coefficient pre-pass
            acc["rotvec_coef"].append(float(r["Counter_Value"]) * 1024.0)
        elif "towr_cost_kernel<" in k:   # <acc, gait, rotvec>: 0 f only, 1 slot gradient, 2 limb gradient
            targs = [a.strip() for a in k.split("towr_cost_kernel<")[1].split(">")[0].split(",")]
            acc["objective" + {"0": "_f_only", "1": "", "2": "_limbs"}[targs[0]] + ("_gait" if targs[1] == "true" else "")].append(
                float(r["Counter_Value"]) * 1024.0)
        elif "towr_dyn_g1_kernel" in k:
            acc["dyn_g1"].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    Bg = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
    f, w = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    rec = {"source": f"rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), {fdir} {wdir}; "
                     "FETCH_SIZE x2 (gfx950 16 B/lane read correction), WRITE_SIZE as is; per launch of "
                     "problems_per_launch problems (each entry's own)",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fb, wb = 2.0 * f.get(k, 0.0), w.get(k, 0.0)
        rec["kernels"][k] = {"problems_per_launch": Bg if k.startswith("gait_") else B,
                             "fetch_bytes_raw": f.get(k), "fetch_bytes": fb, "write_bytes": wb,
                             "hbm_bytes_per_launch": fb + wb}
    with open(out, "w") as fh:
        json.dump(rec, fh, indent=1)
    for k, v in rec["kernels"].items():
        print(f"{k:40s} B {v['problems_per_launch']:5d} fetch {v['fetch_bytes'] / 1e6:9.2f} MB  write {v['write_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
