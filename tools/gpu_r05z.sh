#!/bin/bash
# GPU box, round-5 close: the -m gpu suite, the bench with the launch log (kernel_resources.py input), the
# gait / Torque / RotVec steps of the product against round 4's code (tools/build/libtowr_gpu_base.so),
# rocprofv3 kernel-trace --stats of the bench, and the FETCH_SIZE / WRITE_SIZE passes. Stops at the first failure.
TAG=${1:-r05z}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
TOWR_GPU_LAUNCH_LOG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log \
    2> gpurun_out/${TAG}_launch.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" base; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step) || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step) || exit 1
    r=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --rotvec $L 2>&1 | grep step) || exit 1
    echo "${V:-product} gait [$g] torque [$t] rotvec [$r]" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
tools/gpu_pmc.sh ${TAG}_pmc 5 "fetch write"
