#!/bin/bash
# one GPU call: host-input / multi-context parity tests of the current build
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_multi_gpu.py tests/test_pipeline_gpu.py tests/test_deskew.py tests/test_node_core.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02g_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r02g_tests.log; exit 1; }
tail -2 gpurun_out/r02g_tests.log
