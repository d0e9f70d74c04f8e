#!/bin/bash
# rocprofv3 kernel-trace stats of the bench command -> gpurun_out/prof_<tag>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
mkdir -p gpurun_out
( while sleep 30; do echo "prof running"; done ) & HB=$!
timeout -k 10 ${PROF_TIMEOUT:-500} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 -u bench.py --no-cpu --workers 1 ${BENCH_ARGS} > gpurun_out/prof_$TAG.log 2>&1 || { kill $HB; echo "prof failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
kill $HB
tail -2 gpurun_out/prof_$TAG.log
find gpurun_out/prof_$TAG -name '*stats*'
