"""Average PMC counters per kernel (by kernel name) over the tile-kernel dispatches of a rocprofv3
--pmc run: python tools/pmc_summ.py gpurun_out/TAG_sq [gpurun_out/TAG_fetch ...]"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
meta = {}
for d in sys.argv[1:]:
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if "towr" not in k:
            continue
        key = k.split("towr_tile_kernel<")[-1].split(">")[0] if "towr_tile_kernel" in k else ("misc" if "misc" in k else k.replace("void tg::(anonymous namespace)::", "").split("(")[0])
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[key] = (r["Grid_Size"], r["Workgroup_Size"], r["LDS_Block_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"])
for key, cs in acc.items():
    avg = {c: sum(v) / len(v) for c, v in cs.items()}
    g, wg, lds, vg, ag, sg = meta[key]
    print(f"{key}: grid {g} wg {wg} lds {lds} vgpr {vg} agpr {ag} sgpr {sg}")
    w = avg.get("SQ_WAVES")
    for c in sorted(avg):
        extra = f"  per-wave {avg[c] / w:.1f}" if w and c.startswith("SQ_") and c != "SQ_WAVES" else ""
        print(f"    {c:22s} {avg[c]:.4g}{extra}")
