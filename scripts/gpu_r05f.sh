#!/bin/bash
# round 5 evidence: the default bench line, a 20-step line (the roofline ratios
# must not depend on --steps), rocprofv3 kernel stats of the bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05f}
( while sleep 30; do echo "bench running"; done ) & HB=$!
timeout -k 10 700 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { kill $HB; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu --multi= --multi-1m= --no-h2d > gpurun_out/bench_${TAG}_s20.json 2> gpurun_out/bench_${TAG}_s20.err || { kill $HB; tail -30 gpurun_out/bench_${TAG}_s20.err; exit 1; }
kill $HB
BENCH_ARGS="--steps 40 --multi= --multi-1m= --no-h2d" TAG=$TAG bash scripts/gpu_prof.sh || exit 1
python3 -c "
import json
for f in ['gpurun_out/bench_$TAG.json', 'gpurun_out/bench_${TAG}_s20.json']:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], {k: (d[k].get('frac'), d[k].get('traffic_ratio')) for k in d if k.startswith('roofline')})
"
