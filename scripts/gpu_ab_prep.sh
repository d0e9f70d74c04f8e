#!/bin/bash
# same-box A/B of the bench's step call (prepped arguments vs per-step conversion), then lib vs lib_alt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in P U; do
    if [ $v = U ]; then export VG_BENCH_UNPREPPED=1; else unset VG_BENCH_UNPREPPED; fi
    timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi= > gpurun_out/abp_$v$i.json 2>gpurun_out/abp.err || { echo "bench $v failed"; tail -5 gpurun_out/abp.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abp_$v$i.json')); print('$v', d['value'], d['ms_per_step'], d['host_ms_per_scan'])"
  done
done
unset VG_BENCH_UNPREPPED
AB_ARGS="--multi=" bash scripts/ab.sh || exit 1
