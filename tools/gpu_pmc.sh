#!/bin/bash
# GPU-box PMC passes (kernel-trace only, never combined with sys/runtime traces):
#   pass 1: SQ instruction/wait counters; pass 2: FETCH_SIZE; pass 3: WRITE_SIZE.
# Usage: tools/gpu_pmc.sh TAG [steps]
TAG=${1:-pmc}
STEPS=${2:-5}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/${TAG}_$name -o run -- \
      python3 bench.py --steps $STEPS --warmup 2 --no-cpu > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -2 gpurun_out/${TAG}_$name.log
  return $rc
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
