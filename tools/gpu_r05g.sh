#!/bin/bash
# GPU box: parity of the gait and RotVec paths; same-box A/Bs: the gait step (plain, + Torque) and B = 1 gait against a
# saved build (tools/build/libtowr_gpu_base.so); the RotVec step with Dynamic + small kinds beside RangeOfMotion / FDISC
# (default) vs serial (TOWR_GPU_ROTVEC_OVERLAP=0); the C++ zero-copy callbacks with their timings
TAG=${1:-r05g}; BASE=${2:-tools/build/libtowr_gpu_base.so}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque or rotvec" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_cpp_host.py -m gpu -x -q -s -k zero_copy --timeout 120 --timeout-method thread 2>&1 | grep -E "zerocopy|passed|failed"
for i in 1 2 3; do
  for LIB in "" $BASE; do
    for T in "" --torque; do
      echo "gait ${LIB:-product} $T $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T ${LIB:+--lib $LIB} 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
  for O in 1 0; do
    echo "rotvec overlap=$O $(TOWR_GPU_ROTVEC_OVERLAP=$O timeout -k 10 200 python tools/gait_ab.py --reps 100 --step-only --rotvec --no-gait --batch 4096 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
  done
done
cat gpurun_out/${TAG}_ab.log
for LIB in "" $BASE; do
  echo "single gait ${LIB:-product}"; timeout -k 10 200 python tools/single_probe.py gait ${LIB:+--lib $LIB} 2>&1 | grep -v amdgpu.ids || exit 1
done
