#!/bin/bash
# GPU box: RotVec (and Euler) headline step with the RangeOfMotion tile value cap lowered (TOWR_TILE_VCAP_ROM: smaller
# tiles, less LDS per block) against the default, one box
TAG=${1:-r05aa}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TOWR_GPU_LAUNCH_LOG=1 TOWR_TILE_VCAP_ROM=4608 timeout -k 10 100 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 20 --step-only 2>&1 | grep -E "towr-launch" >> gpurun_out/${TAG}_launch.log
TOWR_GPU_LAUNCH_LOG=1 timeout -k 10 100 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 20 --step-only 2>&1 | grep -E "towr-launch" >> gpurun_out/${TAG}_launch.log
cat gpurun_out/${TAG}_launch.log
for i in 1 2 3; do
  for C in 0 5120 4608 3840; do
    r=$(TOWR_TILE_VCAP_ROM=$C timeout -k 10 200 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 200 2>&1 | grep -E "range_of|step" | tr '\n' ' ') || exit 1
    e=$(TOWR_TILE_VCAP_ROM=$C timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 200 --step-only 2>&1 | grep step) || exit 1
    echo "cap $C rotvec [$r] euler [$e]" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
