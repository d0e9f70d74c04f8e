#!/bin/bash
# tests + propagation probe + same-box A/B + trace (gpu_r04d.sh), the
# multi-sequence rates with and without the active-sequence cap, then the PMC
# traffic passes (event hand-offs: a counter pass serialises the kernels, so a
# polling hand-off kernel would wait for a kernel queued behind it)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash scripts/gpu_r04d.sh || exit 1
export GPU_MAX_HW_QUEUES=16
for cfg in "4 64line 0" "8 64line 0" "8 64line 4" "6 64line 4"; do
  set -- $cfg
  timeout -k 10 240 python3 scripts/multi_pmc.py $1 $2 $3 > gpurun_out/mrate_$1_$3.json 2> gpurun_out/mrate_$1_$3.err || { echo "rate $cfg failed"; tail -5 gpurun_out/mrate_$1_$3.err; exit 1; }
  cat gpurun_out/mrate_$1_$3.json
done
unset GPU_MAX_HW_QUEUES
VG_BENCH_DEBUG=14=0 TAG=${TAG}p bash scripts/gpu_pmc.sh > gpurun_out/pmc_${TAG}p.out 2>&1 || { tail -20 gpurun_out/pmc_${TAG}p.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_${TAG}p gpurun_out/pmc_${TAG}p/pmc_traffic.json | head -30
