#!/bin/bash
# round-end evidence: full gpu test suite, smoke, the default bench line, then
# rocprofv3 kernel stats of the same bench command (each step time-limited)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r05final}
BENCH_ARGS="" bash scripts/gpu_check.sh || exit 1
cp gpurun_out/bench.json gpurun_out/bench_$TAG.json
TAG=$TAG bash scripts/gpu_prof.sh || exit 1
