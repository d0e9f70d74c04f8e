#!/bin/bash
# the multi-sequence counters (B = 4 vs B = 8), then the default bench's PMC
# traffic passes and kernel stats (gpu_pmc.sh); each step under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04f}
if [ -z "$SKIP_MULTI" ]; then
  bash scripts/gpu_multi_pmc.sh > gpurun_out/mpmc_$TAG.out 2>&1 || { tail -20 gpurun_out/mpmc_$TAG.out; exit 1; }
  tail -30 gpurun_out/mpmc_$TAG.out
fi
TAG=$TAG bash scripts/gpu_pmc.sh > gpurun_out/pmc_$TAG.out 2>&1 || { tail -20 gpurun_out/pmc_$TAG.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/pmc_traffic.json
