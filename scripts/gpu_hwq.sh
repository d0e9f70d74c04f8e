#!/bin/bash
# multi-sequence rate against the process's hardware-queue count (one process of B sequences)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "4 4" "8 4" "16 4" "8 8" "4 16" "8 16"; do
  set -- $cfg
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 240 python3 scripts/multi_pmc.py $1 64line 0 > gpurun_out/hwq_$1_$2.json 2> gpurun_out/hwq_$1_$2.err || { echo "B=$1 hwq=$2 failed"; tail -5 gpurun_out/hwq_$1_$2.err; exit 1; }
  echo "hwq=$2 $(cat gpurun_out/hwq_$1_$2.json)"
done
