#!/bin/bash
# GPU box: gait / torque / RotVec parity; record-lane stamps (FDISC alone, the step); same-box A/B of the gait step
# (plain, + Torque) against the saved base build (round 4's code)
TAG=${1:-r05m}; BASE=${2:-tools/build/libtowr_gpu_base.so}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque or rotvec" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_pytest.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stamps.py --only 2 > gpurun_out/${TAG}_st_f.log 2>&1 || exit 1
timeout -k 10 200 python tools/stamps.py > gpurun_out/${TAG}_st_step.log 2>&1 || exit 1
for f in f step; do echo "== $f"; grep -v amdgpu.ids gpurun_out/${TAG}_st_$f.log | sed 's/_ZN2tg12_GLOBAL__N_1[0-9]*//; s/EvNS_7KParams.*E:/:/' | cut -c1-200; done
for i in 1 2 3; do
  for L in "" "--lib $BASE"; do
    for T in "" --torque; do
      echo "gait ${L:-product} $T $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T $L 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${TAG}_ab.log
