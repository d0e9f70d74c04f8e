#!/bin/bash
# the default bench line, then the rocprofv3 kernel-trace stats of the same command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03f}
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -c 600 gpurun_out/bench_$TAG.json
TAG=$TAG bash scripts/gpu_prof.sh
