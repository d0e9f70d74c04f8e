#!/bin/bash
# HBM traffic of the roofline kernels: two separate rocprofv3 --pmc passes
# (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2; MI355X_MICROARCH.md) plus the
# kernel-trace stats of the same bench command. Outputs under gpurun_out/pmc_<tag>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
D=gpurun_out/pmc_$TAG
mkdir -p $D
ARGS="--no-cpu --steps 12 --warmup 12 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --multi= --multi-1m="
VG_BENCH_DEBUG=14=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- python3 bench.py $ARGS > $D/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $D/fetch.log; exit 1; }
VG_BENCH_DEBUG=14=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- python3 bench.py $ARGS > $D/write.log 2>&1 || { echo "write pass failed"; tail -20 $D/write.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $D/stats -o run -- python3 bench.py --no-cpu --target-steps 0 --workers 1 --no-h2d --multi= --multi-1m= > $D/stats.log 2>&1 || { echo "stats pass failed"; tail -20 $D/stats.log; exit 1; }
find $D -name '*.csv' | head -20
