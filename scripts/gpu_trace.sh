#!/bin/bash
# rocprofv3 kernel trace (per-dispatch timestamps) of a short bench -> gpurun_out/trace_<tag>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/trace_$TAG -o run -- python3 -u bench.py --no-cpu --steps 20 --warmup 12 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --no-tile1 --multi= --multi-1m= ${BENCH_ARGS} > gpurun_out/trace_$TAG.log 2>&1 || { echo "trace failed"; tail -30 gpurun_out/trace_$TAG.log; exit 1; }
tail -1 gpurun_out/trace_$TAG.log
find gpurun_out/trace_$TAG -name '*.csv' | xargs ls -la
