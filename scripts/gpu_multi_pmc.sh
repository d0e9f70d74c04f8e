#!/bin/bash
# the multi-sequence regression past B = 4: L2 hit rate and kernel durations at B = 4 and B = 8
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
for B in 4 8; do
  timeout -k 10 240 python3 scripts/multi_pmc.py $B > gpurun_out/mpmc_rate_B$B.json 2> gpurun_out/mpmc_rate_B$B.err || { echo "rate B=$B failed"; tail -5 gpurun_out/mpmc_rate_B$B.err; exit 1; }
  cat gpurun_out/mpmc_rate_B$B.json
  timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/mpmc_B$B -o run -- python3 scripts/multi_pmc.py $B > gpurun_out/mpmc_B$B.log 2>&1 || { echo "pmc B=$B failed"; tail -10 gpurun_out/mpmc_B$B.log; exit 1; }
done
python3 scripts/multi_pmc_summary.py gpurun_out/mpmc_B4 gpurun_out/mpmc_B8 > gpurun_out/mpmc_summary.json && head -60 gpurun_out/mpmc_summary.json
