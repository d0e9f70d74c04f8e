#!/bin/bash
# one GPU call: parity tests that drive vg_step / vg_step_deskew with host buffers, then the bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_pipeline_gpu.py tests/test_deskew.py tests/test_node_core.py tests/test_cold_start.py tests/test_stage_api_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/hostin_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/hostin_tests.log; exit 1; }
tail -2 gpurun_out/hostin_tests.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_hostin.json 2> gpurun_out/bench_hostin.err || { echo "bench failed"; tail -30 gpurun_out/bench_hostin.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_hostin.json')); print(d['value'], d['ms_per_step'], d['host_input'])"
