#!/bin/bash
# same-build A/B: A = default, then each ';'-separated config of AB_DEBUG as VG_BENCH_DEBUG (test knobs on
# the metric leg), 3 alternating rounds
set -o pipefail
mkdir -p gpurun_out
IFS=';' read -ra CFGS <<< "$AB_DEBUG"
for i in $(seq 1 ${AB_ROUNDS:-3}); do
  for v in A "${CFGS[@]}"; do
    if [ "$v" = A ]; then unset VG_BENCH_DEBUG; tag=A; else export VG_BENCH_DEBUG=$v; tag=B_${v//[=,]/_}; fi
    timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --no-tile1 --multi= --multi-1m= ${AB_ARGS} > gpurun_out/ab_$tag$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$tag$i.json')); print('$tag', d['value'], d['ms_per_step'], d['roofline_k_ba_solve']['avg_launch_us'])"
  done
done
