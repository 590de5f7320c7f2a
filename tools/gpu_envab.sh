#!/bin/bash
# GPU-box: same-box A/B of environment configurations of the product library (tools/gait_ab.py whole steps).
# Usage: tools/gpu_envab.sh TAG "GAIT_AB_ARGS" "CONF1 CONF2 ..."   (a CONF is VAR=V[,VAR=V...]; NONE=1 = defaults)
TAG=$1; ARGS=$2; CONFS=$3
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  for C in $CONFS; do
    echo "== $C" >> gpurun_out/${TAG}_ab.log
    env ${C//,/ } timeout -k 10 200 python tools/gait_ab.py --step-only $ARGS >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
  done
done
grep -E "^==|step" gpurun_out/${TAG}_ab.log | paste - - | awk '{print $2, $(NF-1)}' | sort | awk '{a[$1]=a[$1]" "$2} END {for (k in a) print k, a[k]}'
