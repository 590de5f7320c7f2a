#!/bin/bash
# The GPU-box script (measurement tooling, not product): every step under its own time limit, chained so that
# the first failure, fault, abort or time-out ends the run. Results land in gpurun_out/TAG_*; copy what is to
# be kept into profiles/.
#
# usage: tools/gpu.sh TAG STEP [STEP ...]
#   tests            the -m gpu suite                                      -> TAG_pytest.log
#   zerocopy         the IPOPT-callback timings (towr_host_check)          -> TAG_zerocopy.log
#   bench            bench.py with the driver's flags + the launch log     -> TAG_bench.log / .json, TAG_launch.log
#   ab:LIB[:N]       N (3) alternating driver-flag bench runs, product vs tools/build/libtowr_gpu_LIB.so
#                    (tools/ab.py: bench.py itself, the driver's x sets / legs / reps)      -> TAG_ab.log
#   prof             rocprofv3 --kernel-trace --stats of the bench         -> TAG_kernel_stats.csv, TAG_alone.txt
#   pmc              FETCH_SIZE and WRITE_SIZE passes (separate runs) of the bench and of the gait legs, summarised
#                    per launch with each entry's own problems per launch    -> TAG_pmc_traffic.json
#   sq               one SQ-counter pass of the bench                      -> TAG_sq.txt
#   stamps[:ARGS]    in-kernel phase stamps (experiment build -DTOWR_STAMPS; ARGS for tools/stamps.py)
#   cost             the objective kernel per cost kind (tools/cost_timing.py) -> TAG_cost.log
TAG=${1:?tag}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
O=gpurun_out/${TAG}
BENCH="--steps 20 --warmup 5"
step() {   # name, seconds, command...: run it, report, stop the script on failure
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@"
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}
for S in "$@"; do
  case $S in
    tests)
      step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > ${O}_pytest.log 2>&1
      tail -2 ${O}_pytest.log ;;
    zerocopy)
      step zerocopy 200 python -u -m pytest tests/test_cpp_host.py -m gpu -q -s --timeout 120 --timeout-method thread \
          -k zero_copy > ${O}_zerocopy.log 2>&1
      grep -i "zerocopy\|pair" ${O}_zerocopy.log ;;
    bench)
      TOWR_GPU_LAUNCH_LOG=1 step bench 400 python bench.py $BENCH > ${O}_bench.log 2> ${O}_launch.log
      grep '^{' ${O}_bench.log > ${O}_bench.json
      python3 -c "import json,sys; j=json.load(open('${O}_bench.json')); print('headline', round(j['ms_per_step'],4), 'ms', \
round(j['value']/1e6,3), 'M/s frac', round(j['roofline']['frac'],3), *[(k, round(j[k]['ms_per_batch'],4)) for k in \
('objective','gait_optimization','gait_torque','rotvec') if k in j])" ;;
    ab:*)
      IFS=: read -r _ LIB N <<< "$S"
      step ab 1500 python tools/ab.py ${TAG} "product:" "${LIB}:TOWR_GPU_LIB=tools/build/libtowr_gpu_${LIB}.so" \
          --rounds ${N:-3} > ${O}_ab.log 2>&1
      grep "==" ${O}_ab.log ;;
    prof)
      step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run -- \
          python3 bench.py $BENCH --no-cpu --no-host > ${O}_prof.log 2>&1
      find ${O}_prof -name "*kernel_stats.csv" -exec cp {} ${O}_kernel_stats.csv \;
      T=$(find ${O}_prof -name "*kernel_trace.csv" | head -1)
      [ -n "$T" ] && for K in towr_step_kernel towr_tile_kernel towr_misc_kernel towr_cost_kernel; do
        echo "== $K"; python3 tools/alone_avg.py "$T" $K; done > ${O}_alone.txt && cat ${O}_alone.txt ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        step pmc_$C 200 rocprofv3 --kernel-trace --pmc $C --output-format csv -d ${O}_$C -o run -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --legs gait_optimization,gait_torque,objective \
            > ${O}_$C.log 2>&1
      done
      step pmc_summary 60 python3 tools/pmc_traffic.py ${O}_FETCH_SIZE ${O}_WRITE_SIZE ${O}_pmc_traffic.json ;;
    sq)
      step sq 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d ${O}_sq -o run -- \
          python3 bench.py --steps 5 --warmup 2 --no-cpu --no-host --legs objective > ${O}_sq.log 2>&1
      step sq_summary 60 python3 tools/pmc_summ.py ${O}_sq > ${O}_sq.txt ;;
    stamps*)
      IFS=: read -r _ ARGS <<< "$S"
      step stamps 300 python3 tools/stamps.py $ARGS > ${O}_stamps.log 2>&1
      tail -40 ${O}_stamps.log ;;
    cost)
      step cost 200 python3 tools/cost_timing.py > ${O}_cost.log 2>&1
      grep -v amdgpu ${O}_cost.log ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
exit 0
