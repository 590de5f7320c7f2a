#!/bin/bash
# GPU box: parity of the gait / torque / RotVec paths; same-box A/Bs of the gait step (plain, + Torque): product
# (fused FDISC), TOWR_GPU_FDISC_FUSED=0, and a saved build (tools/build/libtowr_gpu_base.so); RotVec overlap on / off
TAG=${1:-r05h}; BASE=${2:-tools/build/libtowr_gpu_base.so}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque or rotvec" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in prod nofused base; do
    for T in "" --torque; do
      if [ $V = base ]; then L="--lib $BASE"; else L=""; fi
      if [ $V = nofused ]; then F=0; else F=1; fi
      echo "gait $V $T $(TOWR_GPU_FDISC_FUSED=$F timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T $L 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
  for O in 1 0; do
    echo "rotvec overlap=$O $(TOWR_GPU_ROTVEC_OVERLAP=$O timeout -k 10 200 python tools/gait_ab.py --reps 100 --step-only --rotvec --no-gait --batch 4096 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
timeout -k 10 300 python -u -m pytest tests/test_cpp_host.py -m gpu -x -q -s -k zero_copy --timeout 120 --timeout-method thread 2>&1 | grep -E "zerocopy|passed|failed"
