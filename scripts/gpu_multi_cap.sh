#!/bin/bash
# multi-sequence children (fresh process per B) under several context capacities
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cap in "--hash-log2 20" "--max-nodes 1000000 --max-fix 4000000" "--max-nodes 1000000 --max-fix 4000000 --hash-log2 20"; do
  timeout -k 10 300 python bench.py --no-cpu --target-steps 0 --no-h2d --stage-scans 0 --steps 20 --multi=4,8 $cap > gpurun_out/mc.json 2> gpurun_out/mc.err || { tail -5 gpurun_out/mc.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/mc.json')); print('$cap', d['value'], d['multi_sequence']['by_B'])"
done
