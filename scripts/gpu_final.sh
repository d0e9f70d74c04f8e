#!/bin/bash
# round-end GPU call: full gpu test suite, smoke, bench line, then rocprofv3 kernel stats of the bench command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_ARGS="" bash scripts/gpu_check.sh || exit 1
TAG=r02f bash scripts/gpu_prof.sh || exit 1
