#!/bin/bash
# same-build A/B: A = default, B = VG_BENCH_DEBUG=$AB_DEBUG (test knobs on the metric leg), 3 alternating runs each
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export VG_BENCH_DEBUG=$AB_DEBUG; else unset VG_BENCH_DEBUG; fi
    timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi= --multi-1m= > gpurun_out/ab_$v$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$v$i.json')); print('$v', d['value'], d['ms_per_step'])"
  done
done
