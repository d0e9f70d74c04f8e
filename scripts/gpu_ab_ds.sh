#!/bin/bash
# one GPU call: pipeline parity tests on the A build, then the same-box A/B (A = lib, B = lib_alt)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
AB_ARGS="--multi=" bash scripts/ab.sh
