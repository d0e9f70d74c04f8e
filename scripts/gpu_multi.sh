#!/bin/bash
# multi-sequence legs only (twice) + the multi-sequence parity test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-multi}
timeout -k 10 300 python -u -m pytest tests/test_multi_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --stage-scans 0 --target-steps 0 --no-h2d --multi=${MULTI:-2,4,8,16} --multi-1m=${MULTI1M:-} ${BENCH_ARGS} > gpurun_out/multi_$TAG$i.json 2> gpurun_out/multi_$TAG$i.err || { echo "bench failed"; tail -20 gpurun_out/multi_$TAG$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/multi_$TAG$i.json').read().strip().splitlines()[-1]); print(d['value'], d['multi_sequence']['by_B'], (d.get('multi_sequence_1M') or {}).get('by_B'))"
done
