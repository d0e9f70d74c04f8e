#!/bin/bash
# one GPU call: the no-drain host-input parity test, then the bench with the pinned copy on 1 and 4 threads
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -k "host_input or resident" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/hostin_ab_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/hostin_ab_tests.log; exit 1; }
tail -2 gpurun_out/hostin_ab_tests.log
for t in 1 4; do
  VG_COPY_THREADS=$t timeout -k 10 300 python -u bench.py > gpurun_out/bench_copy$t.json 2> gpurun_out/bench_copy$t.err || { echo "bench failed"; tail -30 gpurun_out/bench_copy$t.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_copy$t.json')); print('threads $t', d['value'], d['host_input']['value'], d['host_input']['ms_per_step'])"
done
