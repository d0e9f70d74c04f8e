#!/bin/bash
# pipeline parity tests on the current build, then a same-box A/B (lib vs lib_alt)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py tests/test_deskew.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
AB_ARGS="--multi=" bash scripts/ab.sh || exit 1
