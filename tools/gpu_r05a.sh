#!/bin/bash
# GPU box, round 5 first call: the GPU suite; the bench with the launch log (kernel_resources.py); same-box A/B of the
# gait step against round 3's build (tools/build/libtowr_gpu_r03.so); kernel traces of the gait steps.
TAG=${1:-r05a}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
TOWR_GPU_LAUNCH_LOG=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_launch.log || exit $?
python tools/summ.py gpurun_out/${TAG}_bench.json
for i in 1 2; do
  for LIB in "" tools/build/libtowr_gpu_r03.so; do
    timeout -k 10 200 python tools/gait_ab.py --reps 40 --step-only ${LIB:+--lib $LIB} >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log
for LIB in "" tools/build/libtowr_gpu_r03.so; do
  name=$([ -z "$LIB" ] && echo prod || echo r03)
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr_$name -o run -- python tools/step_trace.py ${LIB:+--lib $LIB} > gpurun_out/${TAG}_tr_$name.log 2>&1 || exit $?
done
echo done
