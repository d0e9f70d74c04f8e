#!/bin/bash
# multi-sequence sweep, then the kernel trace of the metric workload and its
# per-scan timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03g}
HWQS="${HWQS:-16 8}" bash scripts/gpu_msweep.sh || exit 1
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
