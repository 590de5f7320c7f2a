#!/bin/bash
# GPU box: gait / torque / RotVec parity (incl. the fused FDISC kernel, opt-in); same-box A/B of the gait step with the
# side streams at the greatest (default) or normal priority, against round 3's build; + Torque
TAG=${1:-r05k}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "gait or torque or rotvec" > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_pytest.log | tail -8
for i in 1 2 3; do
  for V in high normal r03; do
    for T in "" --torque; do
      L=""; P=high
      [ $V = r03 ] && L="--lib tools/build/libtowr_gpu_r03.so"
      [ $V = normal ] && P=normal
      echo "gait $V $T $(TOWR_GPU_SIDE_PRIO=$P timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T $L 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${TAG}_ab.log
