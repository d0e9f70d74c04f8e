#!/bin/bash
# round-4 GPU call: -m gpu tests, bench line, rocprofv3 stats + PMC passes (gpu_all.sh),
# then a kernel trace of the bench and its per-scan timeline. TAG names the outputs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r04}
TAG=$TAG bash scripts/gpu_all.sh || exit 1
[ -n "$NO_TRACE" ] && exit 0
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
