#!/bin/bash
# Round-3 GPU call: every -m gpu test, the default bench line, then the
# rocprofv3 kernel-trace stats of the bench command (scripts/gpu_prof.sh,
# host-input leg included). Each step under its own limit, stop at the first
# failure. Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03a}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gputest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$TAG.log
  [ $rc -ne 0 ] && { tail -30 gpurun_out/gputest_$TAG.log; exit $rc; }
  tail -2 gpurun_out/gputest_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  head -c 400 gpurun_out/bench_$TAG.json; echo
fi
[ -n "$SKIP_PROF" ] && exit 0
TAG=$TAG BENCH_ARGS="--multi= --multi-1m=" bash scripts/gpu_prof.sh
