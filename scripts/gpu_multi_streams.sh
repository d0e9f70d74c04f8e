#!/bin/bash
# multi-sequence streams sweep (VG_MULTI_STREAMS = G; unset: the library's
# default, four shared streams past four sequences), after the multi-sequence
# parity tests -> gpurun_out/ms_*.json, one line per run on stdout
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_multi_gpu.py > gpurun_out/t_ms.log 2>&1; tail -2 gpurun_out/t_ms.log
tail -1 gpurun_out/t_ms.log | grep -q " passed" || exit 1
A="--no-cpu --stage-scans 0 --target-steps 0 --no-h2d --no-tile1 --multi-1m= --multi ${MS_B:-4,8,16}"
for G in ${MS_G:-default 0 3 5 6}; do
  if [ $G = default ]; then unset VG_MULTI_STREAMS; else export VG_MULTI_STREAMS=$G; fi
  timeout -k 10 300 python bench.py $A > gpurun_out/ms_G$G.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ms_G$G.json')); print('G=$G', d['multi_sequence']['by_B'], d['multi_sequence'].get('streams_by_B'))"
done
