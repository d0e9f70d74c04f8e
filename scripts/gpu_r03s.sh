#!/bin/bash
# parity subset, A/B vs lib_alt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03s}
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -30 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_ARGS="--multi= --multi-1m=" timeout -k 10 600 bash scripts/ab.sh || exit 1
