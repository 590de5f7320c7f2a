#!/bin/bash
# GPU box: batch vs B = 1 after the contraction fix; phase stamps of the fused FDISC kernel (FDISC alone and the whole
# gait step) and of the records + compose path for comparison
TAG=${1:-r05j}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== product"; timeout -k 10 200 python tools/diag_batch_b1.py 2>&1 | grep -v amdgpu.ids | head -12 || exit 1
timeout -k 10 200 python tools/stamps.py --only 2 > gpurun_out/${TAG}_st_ff.log 2>&1 || exit 1
TOWR_GPU_FDISC_FUSED=0 timeout -k 10 200 python tools/stamps.py --only 2 > gpurun_out/${TAG}_st_rc.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_st_step.log 2>&1 || exit 1
for f in ff rc step; do echo "== $f"; grep -v amdgpu.ids gpurun_out/${TAG}_st_$f.log | sed 's/_ZN2tg12_GLOBAL__N_1[0-9]*//; s/EvNS_7KParams.*E:/:/' | cut -c1-200; done
