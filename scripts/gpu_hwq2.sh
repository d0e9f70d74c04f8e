#!/bin/bash
# multi-sequence rate: B sequences over cap hardware queues, one sequence per queue at a time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "8 4 4" "16 4 4" "8 5 4" "4 16 0" "8 8 8"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 240 python3 scripts/multi_pmc.py $1 64line $3 > gpurun_out/hwq2_$1_$2_$3.json 2> gpurun_out/hwq2_$1_$2_$3.err || { echo "B=$1 hwq=$2 cap=$3 failed"; tail -5 gpurun_out/hwq2_$1_$2_$3.err; exit 1; }
  echo "hwq=$2 $(cat gpurun_out/hwq2_$1_$2_$3.json)"
done
