#!/bin/bash
# GPU box, round-5 close (final build): the -m gpu suite, the zero-copy callback timings, the bench with the launch log,
# gait / Torque / RotVec A/B against round 4's build, rocprofv3 kernel-trace --stats of the bench, FETCH_SIZE / WRITE_SIZE
TAG=${1:-r05zz}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_cpp_host.py -m gpu -q -s --timeout 120 --timeout-method thread -k zero_copy \
    > gpurun_out/${TAG}_zerocopy.log 2>&1 || exit 1
grep zerocopy gpurun_out/${TAG}_zerocopy.log
TOWR_GPU_LAUNCH_LOG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log \
    2> gpurun_out/${TAG}_launch.log
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  for V in "" base; do
    L=""; [ -n "$V" ] && L="--lib tools/build/libtowr_gpu_$V.so"
    g=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    t=$(timeout -k 10 200 python tools/gait_ab.py --reps 60 --step-only --torque $L 2>&1 | grep step | awk '{print $3}') || exit 1
    r=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --rotvec --batch 4096 --reps 200 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    h=$(timeout -k 10 200 python tools/gait_ab.py --no-gait --batch 4096 --reps 300 --step-only $L 2>&1 | grep step | awk '{print $3}') || exit 1
    echo "${V:-product} gait $g torque $t rotvec $r headline $h" >> gpurun_out/${TAG}_ab.log
  done
done
cat gpurun_out/${TAG}_ab.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host > gpurun_out/${TAG}_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
tools/gpu_pmc.sh ${TAG}_pmc 5 "fetch write"
