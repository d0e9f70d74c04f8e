#!/bin/bash
# stage-API parity (incl. the fusion A/B cases), a same-build A/B of one knob, then a kernel trace + scan timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05p}
timeout -k 10 600 python -u -m pytest tests/test_stage_api_gpu.py tests/test_ba_hessian_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_DEBUG="${AB_DEBUG:-36=0}" AB_ROUNDS=${AB_ROUNDS:-3} bash scripts/ab_env.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
