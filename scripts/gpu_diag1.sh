#!/bin/bash
# (1) kernel stats + stage breakdown of the 1M-ray single-sequence workload,
# (2) kernel traces of the multi-sequence leg at B=4 and B=8 (busy fraction,
# per-kernel shares). Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
( while sleep 30; do echo "diag running"; done ) & HB=$!
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1m -o run -- python3 -u bench.py --lidar 1M --no-cpu --steps 10 --stage-scans 4 --target-steps 0 --workers 1 --no-h2d --multi= --multi-1m= > gpurun_out/prof_1m.json 2> gpurun_out/prof_1m.err || { kill $HB; echo "1M prof failed"; tail -20 gpurun_out/prof_1m.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/prof_1m.json').read().strip().splitlines()[-1]); print(d['value'], d['config'], d['roofline']['stage_ms_per_scan'])"
for B in 4 8; do
  B=$B TAG=mt$B bash scripts/gpu_mtrace.sh > gpurun_out/mtrace_$B.txt 2>&1 || { kill $HB; echo "mtrace $B failed"; tail -20 gpurun_out/mtrace_$B.txt; exit 1; }
  head -40 gpurun_out/mtrace_$B.txt
done
kill $HB
