#!/bin/bash
# one GPU call: kernel trace + per-scan timeline of the current build, then kernel stats of the bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r02f bash scripts/gpu_trace.sh > gpurun_out/trace.out 2>&1 || { tail -5 gpurun_out/trace.out; exit 1; }
f=$(find gpurun_out/trace_r02f -name '*kernel_trace.csv' | head -1)
python3 scripts/scan_timeline.py "$f" 4 > gpurun_out/scan_timeline_r02f.txt && tail -3 gpurun_out/scan_timeline_r02f.txt
TAG=r02f bash scripts/gpu_prof.sh > gpurun_out/prof.out 2>&1 || { tail -5 gpurun_out/prof.out; exit 1; }
tail -3 gpurun_out/prof.out
rm -f "$f"
