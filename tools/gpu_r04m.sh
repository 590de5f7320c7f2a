#!/bin/bash
# GPU-box measurement session of round 4: the -m gpu suite and smoke, a same-box A/B of the gait chain layout, the
# bench with the driver's flags, its rocprofv3 kernel stats and the FETCH_SIZE / WRITE_SIZE passes.
# Usage: tools/gpu_r04m.sh TAG ["lib1 ..."]
TAG=${1:-r04m}; LIBS=$2
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_smoke.log
for i in 1 2; do
  for LIB in "" $LIBS; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
    timeout -k 10 200 python tools/gait_ab.py --reps 40 --torque ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log | grep step
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
tools/gpu_pmc.sh ${TAG}pmc 5 "fetch write" || exit $?
echo done
