#!/bin/bash
# multi-sequence mode with one shared downsample stream (VG_MULTI_DS=1) against
# the downsample on each sequence's stream: parity tests first, then the
# multi-sequence legs (64-line and 1M) alternately
set -o pipefail
mkdir -p gpurun_out
VG_MULTI_DS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_multi_gpu.py > gpurun_out/t_mds.log 2>&1; tail -2 gpurun_out/t_mds.log
tail -1 gpurun_out/t_mds.log | grep -q " passed" || exit 1
A="--no-cpu --stage-scans 0 --target-steps 0 --no-h2d --no-tile1 --steps 10 --multi ${MD_B:-2,4,8} --multi-1m ${MD_1M:-2,4,8}"
for i in 1 2; do
  for v in 0 1; do
    VG_MULTI_DS=$v timeout -k 10 500 python bench.py $A > gpurun_out/mds_$v$i.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/mds_$v$i.json')); print('ds=$v', d['multi_sequence']['by_B'], d['multi_sequence_1M']['by_B'])"
  done
done
