#!/bin/bash
# GPU box: where the batch differs from B = 1 (product, TOWR_GPU_FDISC_FUSED=0, the saved base build); then the A/Bs
# (product / no fused FDISC / base; gait, + Torque; RotVec overlap); then the gait / torque / RotVec parity tests
TAG=${1:-r05i}; BASE=${2:-tools/build/libtowr_gpu_base.so}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== product"; timeout -k 10 200 python tools/diag_batch_b1.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== no fused"; TOWR_GPU_FDISC_FUSED=0 timeout -k 10 200 python tools/diag_batch_b1.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== base"; timeout -k 10 200 python tools/diag_batch_b1.py --lib $BASE 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
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
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "gait or torque or rotvec" > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/${TAG}_pytest.log | tail -12
