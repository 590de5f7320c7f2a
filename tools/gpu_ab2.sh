#!/bin/bash
# GPU-box A/B of experiment builds: the -m gpu suite on the product build, then per-kernel gait times
# (tools/gait_ab.py) for the product and each listed gait variant, then headline bench A/B (tools/ab.py)
# of the product against each listed headline variant. Stops at the first failure.
# Usage: tools/gpu_ab2.sh TAG "gait_lib1 VAR=value ..." "name:TOWR_GPU_LIB=lib ..."
TAG=${1:-ab2}
GAIT_LIBS=$2
HEAD_CFGS=$3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in product $GAIT_LIBS; do
    # an entry is a library path (experiment build) or VAR=value (environment for the product build)
    A=(); E=()
    case "$lib" in product) ;; *=*) E=("$lib"); echo "== env $lib" >> gpurun_out/${TAG}_gait.log ;; *) A=(--lib "$lib") ;; esac
    env "${E[@]}" timeout -k 10 120 python tools/gait_ab.py "${A[@]}" >> gpurun_out/${TAG}_gait.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "gait_ab $lib rc=$rc"; tail -5 gpurun_out/${TAG}_gait.log; exit $rc; }
  done
done
grep -E "step|==" gpurun_out/${TAG}_gait.log | tail -40
if [ -n "$HEAD_CFGS" ]; then
  # shellcheck disable=SC2086
  timeout -k 10 700 python tools/ab.py ${TAG}h "prod:" $HEAD_CFGS --args "--steps 200 --warmup 20 --no-cpu --no-host --no-gait" --rounds 3 > gpurun_out/${TAG}_ab.log 2>&1
  rc=$?; echo "ab rc=$rc"; tail -6 gpurun_out/${TAG}_ab.log
  exit $rc
fi
