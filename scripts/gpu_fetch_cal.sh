#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration: two separate --pmc passes over scripts/micro/fetch_cal (built here)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/fetch_cal
mkdir -p $D
timeout -k 10 60 ./scripts/micro/fetch_cal > $D/bytes.csv || { echo "fetch_cal run failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- ./scripts/micro/fetch_cal > $D/fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $D/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- ./scripts/micro/fetch_cal > $D/write.log 2>&1 || { echo "write pass failed"; tail -20 $D/write.log; exit 1; }
python3 scripts/fetch_cal.py $D $D/bytes.csv $D/fetch_calibration.json
