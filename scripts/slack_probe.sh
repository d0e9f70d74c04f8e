#!/bin/bash
# host slack per point of the step (5: start of the step, 0: before the IEKF enqueue, 4: after it, 3: before the insert, 1: before the LM, 2: before the margi) (VG_HOST_DELAY, pipeline.cpp host_delay): ms/scan with 0 and 40 us delays
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --no-tile1 --multi= --multi-1m= > gpurun_out/slack.json 2>/dev/null || { echo "bench failed"; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/slack.json')); print('$1', d['ms_per_step'])"; }
for rep in 1 2; do
  unset VG_HOST_DELAY; run base
  for pt in 5 0 4 3 1 2; do export VG_HOST_DELAY=$pt,40; run "pt$pt+40us"; done
done
