#!/bin/bash
# GPU-box PMC passes (kernel-trace only, never combined with sys/runtime traces), one counter group
# per pass: sq = SQ instruction/wait counters, fetch = FETCH_SIZE, write = WRITE_SIZE.
# Usage: tools/gpu_pmc.sh TAG [steps] [passes]
TAG=${1:-pmc}
STEPS=${2:-5}
PASSES=${3:-"sq fetch write"}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for p in $PASSES; do
  case $p in
    sq) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" ;;
    sq2) C="SQ_WAVES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" ;;
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE" ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d gpurun_out/${TAG}_$p -o run -- \
      ${PMC_CMD:-python3 bench.py --steps $STEPS --warmup 2 --no-cpu --no-host} > gpurun_out/${TAG}_$p.log 2>&1
  rc=$?; echo "$p rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
