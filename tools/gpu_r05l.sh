#!/bin/bash
# GPU box: sub-phase stamps of the FDISC record lanes (FDISC alone, the gait step)
TAG=${1:-r05l}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamps.py --only 2 > gpurun_out/${TAG}_st_f.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py --only 2 --torque > gpurun_out/${TAG}_st_ft.log 2>&1 || exit 1
for f in f ft; do echo "== $f"; grep -v amdgpu.ids gpurun_out/${TAG}_st_$f.log | sed 's/_ZN2tg12_GLOBAL__N_1[0-9]*//; s/EvNS_7KParams.*E:/:/' | cut -c1-200; done
