set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TOWR_GPU_LIB=$PWD/tools/build/libtowr_gpu_mw3.so TOWR_GPU_FUSE=rfm timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fusion or bench_workload or batch_device" > gpurun_out/r02d_mw3_pytest.log 2>&1
tail -2 gpurun_out/r02d_mw3_pytest.log
timeout -k 10 900 python tools/ab.py r02d_ab "base:" "mw3:TOWR_GPU_LIB=tools/build/libtowr_gpu_mw3.so" "mw3rfm:TOWR_GPU_LIB=tools/build/libtowr_gpu_mw3.so,TOWR_GPU_FUSE=rfm" "rfm:TOWR_GPU_FUSE=rfm"
timeout -k 10 120 python tools/gait_ab.py > gpurun_out/r02d_gait.log 2>&1
cat gpurun_out/r02d_gait.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r02d_gsq -o run -- python3 tools/gait_ab.py --reps 3 > gpurun_out/r02d_gsq.log 2>&1
echo done
