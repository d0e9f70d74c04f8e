#!/bin/bash
# multi-sequence sweep: B values x GPU_MAX_HW_QUEUES settings (64-line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for hwq in ${HWQS:-16 8 32}; do
  VG_MULTI_HWQ=$hwq timeout -k 10 300 python -u bench.py --no-cpu --steps 4 --warmup 12 --stage-scans 0 --target-steps 0 --no-h2d --multi=${MULTI:-4,6,8,12} --multi-1m= > gpurun_out/msweep_$hwq.json 2> gpurun_out/msweep_$hwq.err || { echo "bench failed"; tail -20 gpurun_out/msweep_$hwq.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/msweep_$hwq.json').read().strip().splitlines()[-1]); print('hwq $hwq', d['value'], d['multi_sequence']['by_B'])"
done
