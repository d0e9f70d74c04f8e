#!/bin/bash
# solve tests + parity tests, the solve's phase clocks, then a cross-build A/B (lib/ = working tree, lib_alt/ = HEAD)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05gg}
timeout -k 10 600 python -u -m pytest tests/test_ba_solve_gpu.py tests/test_ba_hessian_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_shard_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
timeout -k 10 200 python3 -u scripts/probe_ba.py > gpurun_out/probe_ba_$TAG.txt 2>&1 || { cat gpurun_out/probe_ba_$TAG.txt; exit 1; }
head -12 gpurun_out/probe_ba_$TAG.txt
AB_ARGS="--no-tile1 --multi= --multi-1m=" bash scripts/ab.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
