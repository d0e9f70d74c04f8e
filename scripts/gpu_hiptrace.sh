#!/bin/bash
# kernel trace + HIP runtime API trace of a short bench: when the host launched
# each kernel against when it ran (scripts/launch_lag.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/htrace_$TAG -o run -- python3 -u bench.py --no-cpu --steps 20 --warmup 12 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --no-tile1 --multi= --multi-1m= > gpurun_out/htrace_$TAG.log 2>&1 || { echo "trace failed"; tail -30 gpurun_out/htrace_$TAG.log; exit 1; }
find gpurun_out/htrace_$TAG -name '*.csv' | xargs ls -la
