#!/bin/bash
# IEKF parity tests, then a cross-build A/B (lib/ = working tree, lib_alt/ = scripts/build_alt.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05t}
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_ARGS="--no-tile1 --multi= --multi-1m=" bash scripts/ab.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
