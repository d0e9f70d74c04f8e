#!/bin/bash
# the structural LM order + zero-tile skips: BA / pipeline parity, then a same-build A/B against Eigen's order
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05h}
timeout -k 10 600 python -u -m pytest tests/test_ba_solve_gpu.py tests/test_ba_hessian_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_DEBUG="${AB_DEBUG:-31=0}" AB_ROUNDS=${AB_ROUNDS:-3} bash scripts/ab_env.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
