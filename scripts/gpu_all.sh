#!/bin/bash
# One GPU call: -m gpu tests, the default bench line, then (TAG set) the
# rocprofv3 kernel-trace stats and the two PMC passes of the bench command.
# Outputs under gpurun_out/. Each step under its own time limit; stops at the
# first failure.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gputest.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest.log
  [ $rc -ne 0 ] && { tail -30 gpurun_out/gputest.log; exit $rc; }
fi
timeout -k 10 420 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json | head -c 600; echo
[ -z "$TAG" ] && exit 0
D=gpurun_out/pmc_$TAG
mkdir -p $D
ARGS="--no-cpu --steps 12 --warmup 12 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --multi= --multi-1m="
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/stats -o run -- python3 bench.py --no-cpu --target-steps 0 --workers 1 --no-h2d --multi= --multi-1m= > $D/stats.log 2>&1 || { echo "stats pass failed"; tail -20 $D/stats.log; exit 1; }
VG_BENCH_DEBUG=14=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- python3 bench.py $ARGS > $D/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $D/fetch.log; exit 1; }
VG_BENCH_DEBUG=14=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- python3 bench.py $ARGS > $D/write.log 2>&1 || { echo "write pass failed"; tail -20 $D/write.log; exit 1; }
python3 scripts/pmc_summary.py $D $D/pmc_traffic.json > /dev/null
find $D -name '*stats*.csv'
