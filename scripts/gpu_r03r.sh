#!/bin/bash
# parity (BA, pipeline, stage API, multi-sequence, shard), A/B vs lib_alt, then the kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03r}
timeout -k 10 500 python -u -m pytest tests/test_ba_hessian_gpu.py tests/test_ba_solve_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py tests/test_shard_gpu.py tests/test_cold_start.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -30 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_ARGS="--multi= --multi-1m=" timeout -k 10 600 bash scripts/ab.sh || exit 1
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
