#!/bin/bash
# GPU box: composer block sizes (TOWR_COMPOSE_BLOCK 512 -> 1024 for the FDISC / TQDISC composer, TOWR_COMPOSE_BLOCK_RD 256 ->
# 512 for RangeOfMotion / Dynamic): gait and gait + Torque steps, one box; the parity test of the chains first
TAG=${1:-r05ad}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in cb256 rd128; do
  TOWR_GPU_LIB=tools/build/libtowr_gpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
      --timeout-method thread -k "two_chains or gait_torque" > gpurun_out/${TAG}_pytest_$V.log 2>&1
  rc=$?; echo "pytest $V rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_$V.log
  [ $rc -eq 0 ] || exit $rc
done
for i in 1 2 3; do
  for V in "" cb256 rd128; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step) || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step) || exit 1
    echo "${V:-product} gait [$g] torque [$t]" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
