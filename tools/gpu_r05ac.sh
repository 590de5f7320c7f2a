#!/bin/bash
# GPU box: the FDISC compose's store pattern without its arithmetic (TOWR_FS_PURE), with plain stores (TOWR_FS_PLAIN):
# the FDISC class alone and the gait step, one box
TAG=${1:-r05ac}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for V in "" fspure fspure4 fsplain; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    timeout -k 10 200 python tools/gait_ab.py --reps 60 $L 2>&1 | grep -E "force_disc|step" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
