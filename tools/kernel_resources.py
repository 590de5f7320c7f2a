"""Per-kernel resources of the engine's gfx950 code objects, and the occupancy of each launch.

Registers, spills, scratch and static LDS come from the AMDGPU metadata note of the code objects that
towr2025_amd/csrc/Makefile builds (build/*.o: the .hip_fatbin section, unbundled for gfx950, read with
llvm-readelf --notes) — no GPU needed. The dynamic LDS of a launch is a host-side choice the code object does
not record: with --launch-log, the "towr-launch <symbol> block <threads> lds <bytes> grid <blocks>" lines that
the library writes to stderr under TOWR_GPU_LAUNCH_LOG (towr_gpu.hip launch_kernel) give it, and the second table
lists each launch's blocks per CU and waves per SIMD (MI355X: 512 VGPR+AGPR per lane and SIMD, allocated in
granules of 8, at most 8 waves per SIMD and 32 per CU, 160 KiB of LDS per CU; a block of W waves occupies
ceil(W / 4) wave slots of every SIMD, /opt/skills/guides/MI355X_MICROARCH.md "Register files").

usage: python tools/kernel_resources.py [--launch-log LOG ...] > profiles/kernel_resources.txt
A measurement tool, not part of the product."""
import argparse
import glob
import os
import re
import subprocess
import tempfile

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
LDS_CU = 160 * 1024


def code_object_kernels(obj, tmp):
    """The metadata of every kernel in the gfx950 code object of one host object file (empty: no device code)."""
    base = os.path.join(tmp, os.path.basename(obj))
    fat, co = base + ".fat", base + ".co"
    if subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj],
                      capture_output=True).returncode != 0:
        return []
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True, text=True).stdout
    m = re.search(r"^\s*---\s*$(.*?)^\s*\.\.\.\s*$", notes, re.S | re.M)
    return yaml.safe_load(m.group(1))["amdhsa.kernels"] if m else []


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return [short(n) for n in out.splitlines()]


def short(n):
    n = n.replace("tg::(anonymous namespace)::", "").replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*\)$", "", n).replace("tg::", "")


def waves_per_simd(vgpr, agpr):
    alloc = (vgpr + agpr + 7) // 8 * 8
    return alloc, min(8, 512 // max(alloc, 8))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", default=os.path.join(ROOT, "towr2025_amd", "csrc", "build"))
    ap.add_argument("--launch-log", nargs="*", default=[])
    args = ap.parse_args()
    kern = {}
    with tempfile.TemporaryDirectory() as tmp:
        for obj in sorted(glob.glob(os.path.join(args.build, "*.o"))):
            for k in code_object_kernels(obj, tmp):
                kern[k[".name"]] = (os.path.basename(obj), k)
    names = sorted(kern)
    pretty = dict(zip(names, demangle(names)))
    print("# Kernel resources: gfx950 code-object metadata (tools/kernel_resources.py; build: towr2025_amd/csrc/Makefile)")
    print("# alloc = VGPR+AGPR rounded to the granule of 8; w/SIMD = waves per SIMD the registers allow; scratch = bytes per lane")
    print(f"{'kernel':58s} {'object':14s} {'VGPR':>4s} {'AGPR':>4s} {'alloc':>5s} {'w/SIMD':>6s} {'SGPR':>4s} "
          f"{'vspill':>6s} {'sspill':>6s} {'scratch':>7s} {'sLDS':>5s} {'maxWG':>5s}")
    for n in names:
        obj, k = kern[n]
        alloc, w = waves_per_simd(k[".vgpr_count"], k.get(".agpr_count", 0))
        print(f"{pretty[n][:58]:58s} {obj[:14]:14s} {k['.vgpr_count']:4d} {k.get('.agpr_count', 0):4d} {alloc:5d} {w:6d} "
              f"{k['.sgpr_count']:4d} {k.get('.vgpr_spill_count', 0):6d} {k.get('.sgpr_spill_count', 0):6d} "
              f"{k['.private_segment_fixed_size']:7d} {k['.group_segment_fixed_size']:5d} {k['.max_flat_workgroup_size']:5d}")
    launches = []
    for log in args.launch_log:
        for line in open(log, errors="replace"):
            m = re.match(r"towr-launch (\S+) block (\d+) lds (\d+) grid (\d+)", line.strip())
            if m:
                launches.append((m.group(1), int(m.group(2)), int(m.group(3)), int(m.group(4))))
    if not launches:
        return
    print()
    print("# Launches (TOWR_GPU_LAUNCH_LOG lines of " + ", ".join(os.path.relpath(p, ROOT) for p in args.launch_log) + ")")
    print("# blocks/CU = min(by registers: floor(w/SIMD / ceil(W/4)), by LDS: floor(160 KiB / (static + dynamic LDS)), by waves: floor(32 / W)),")
    print("# W = waves per block; waves/SIMD = blocks/CU * W / 4")
    print(f"{'kernel':58s} {'block':>5s} {'dynLDS':>7s} {'grid':>7s} {'by reg':>6s} {'by LDS':>6s} {'blk/CU':>6s} {'w/SIMD':>6s}")
    seen = set()
    for sym, block, lds, grid in launches:
        if (sym, block, lds) in seen:
            continue
        seen.add((sym, block, lds))
        k = kern.get(sym, (None, None))[1]
        nm = pretty.get(sym) or short(demangle([sym])[0])
        if k is None:
            print(f"{nm[:58]:58s} {block:5d} {lds:7d} {grid:7d}   (no metadata)")
            continue
        W = (block + 63) // 64
        _, w = waves_per_simd(k[".vgpr_count"], k.get(".agpr_count", 0))
        by_reg = w // ((W + 3) // 4)
        tot = lds + k[".group_segment_fixed_size"]
        by_lds = LDS_CU // tot if tot else 99
        bpc = min(by_reg, by_lds, 32 // W)
        print(f"{nm[:58]:58s} {block:5d} {lds:7d} {grid:7d} {by_reg:6d} {by_lds:6d} {bpc:6d} {bpc * W / 4:6.2f}")


if __name__ == "__main__":
    main()
