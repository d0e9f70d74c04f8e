#!/bin/bash
# rocprofv3 kernel stats of the metric workload (bench without the multi-sequence sweep)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="--multi=" TAG=r02f bash scripts/gpu_prof.sh || exit 1
