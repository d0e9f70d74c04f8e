#!/bin/bash
# multi-sequence: parity test + B sweep (one stream per sequence)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/multi_test.log 2>&1 || { tail -20 gpurun_out/multi_test.log; exit 1; }
tail -2 gpurun_out/multi_test.log
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u scripts/multi_probe.py 64line 0,0 -- 1 2 4 8 16 4 2 8 > gpurun_out/multi1.jsonl 2> gpurun_out/multi1.err || { tail -5 gpurun_out/multi1.err; exit 1; }
cat gpurun_out/multi1.jsonl
