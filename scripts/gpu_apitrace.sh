#!/bin/bash
# rocprofv3 kernel + HIP API trace of a short bench -> gpurun_out/api_<tag>/ (host-side launch costs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/api_$TAG -o run -- python3 -u bench.py --no-cpu --steps 12 --warmup 12 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --multi= ${BENCH_ARGS} > gpurun_out/api_$TAG.log 2>&1 || { echo "trace failed"; tail -30 gpurun_out/api_$TAG.log; exit 1; }
tail -1 gpurun_out/api_$TAG.log
find gpurun_out/api_$TAG -name '*.csv' | xargs ls -la
