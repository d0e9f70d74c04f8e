#!/bin/bash
# probe of k_scan_prop (instrumented build), same-build A/B (AB_DEBUG), kernel trace of the default config
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r04d}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
  tail -1 gpurun_out/gputest_$TAG.log
fi
if [ -n "$PROBE" ]; then
  timeout -k 10 120 python3 scripts/$PROBE > gpurun_out/probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/probe_$TAG.txt; exit 1; }
  cat gpurun_out/probe_$TAG.txt | grep -v amdgpu.ids
fi
[ -n "$AB_DEBUG" ] && { timeout -k 10 900 bash scripts/ab_env.sh || exit 1; }
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
