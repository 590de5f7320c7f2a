#!/bin/bash
# GPU box: gait parity; same-box A/B of the gait step (plain, + Torque) and of B = 1 gait against a saved build
# (tools/build/libtowr_gpu_base.so); the C++ zero-copy callbacks with their timings
TAG=${1:-r05f}; BASE=${2:-tools/build/libtowr_gpu_base.so}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gait or torque" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_cpp_host.py -m gpu -x -q -s -k zero_copy --timeout 120 --timeout-method thread 2>&1 | grep -E "zerocopy|passed|failed"
for i in 1 2 3; do
  for LIB in "" $BASE; do
    for T in "" --torque; do
      echo "$LIB $T $(timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only $T ${LIB:+--lib $LIB} 2>&1 | grep step)" >> gpurun_out/${TAG}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${TAG}_ab.log
for LIB in "" $BASE; do
  echo "single gait ${LIB:-product}"; timeout -k 10 200 python tools/single_probe.py gait ${LIB:+--lib $LIB} 2>&1 | grep -v amdgpu.ids || exit 1
done
