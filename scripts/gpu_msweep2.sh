#!/bin/bash
# multi-sequence experiments: concurrent child processes, wait policies (64-line)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-cpu --steps 4 --warmup 12 --stage-scans 0 --target-steps 0 --no-h2d --multi=${MULTI:-4,8} --multi-1m= > gpurun_out/ms2_$tag.json 2> gpurun_out/ms2_$tag.err || { echo "bench $tag failed"; tail -20 gpurun_out/ms2_$tag.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ms2_$tag.json').read().strip().splitlines()[-1]); print('$tag', d['multi_sequence']['by_B'])"
}
run procs2 VG_MULTI_PROCS=2 || exit 1
run sleep VG_MULTI_WAIT=20,20 || exit 1
run procs2sleep VG_MULTI_PROCS=2 VG_MULTI_WAIT=20,20 || exit 1
