#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the access shapes (scripts/micro/fetch_cal,
# built on the host: hipcc --offload-arch=gfx950 -O3), then the PMC traffic passes
# of the bench workload (scripts/gpu_pmc.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/cal6; mkdir -p $D/fetch $D/write
./scripts/micro/fetch_cal > $D/bytes.csv || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $D/fetch -o run -- ./scripts/micro/fetch_cal > $D/f.log 2>&1 || { echo fetch pass failed; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $D/write -o run -- ./scripts/micro/fetch_cal > $D/w.log 2>&1 || { echo write pass failed; exit 1; }
python3 scripts/fetch_cal.py $D $D/bytes.csv $D/fetch_calibration.json > /dev/null && echo cal ok
TAG=${TAG:-cal} bash scripts/gpu_pmc.sh
