#!/bin/bash
# IEKF phase clocks (probe build), the bench line without the multi legs, then
# the two PMC passes + kernel stats of the bench command -> pmc_traffic.json
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03k}
VINA_GPU_LIB=$PWD/vina-slam_amd/lib_probe/libvina_gpu.so timeout -k 10 200 python -u scripts/probe_ba.py iekf > gpurun_out/probe_iekf_$TAG.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_iekf_$TAG.txt; exit 1; }
cat gpurun_out/probe_iekf_$TAG.txt
TAG=$TAG SKIP_TESTS=1 SKIP_PROF=1 BENCH_ARGS="--multi= --multi-1m=" bash scripts/gpu_r03.sh || exit 1
[ -n "$SKIP_PMC" ] && exit 0
TAG=$TAG bash scripts/gpu_pmc.sh > gpurun_out/pmc_$TAG.out 2>&1 || { tail -5 gpurun_out/pmc_$TAG.out; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_$TAG gpurun_out/pmc_$TAG/pmc_traffic.json | tail -5
