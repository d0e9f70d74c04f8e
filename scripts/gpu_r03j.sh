#!/bin/bash
# kd-LIO exactness + cold start + the sharded test + solve probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03j}
timeout -k 10 500 python -u -m pytest tests/test_kdlio.py tests/test_cold_start.py tests/test_shard_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "valid|map " gpurun_out/gputest_$TAG.log | head -20; tail -3 gpurun_out/gputest_$TAG.log
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" gpurun_out/gputest_$TAG.log | head -60; exit $rc; }
VINA_GPU_LIB=$PWD/vina-slam_amd/lib_probe/libvina_gpu.so timeout -k 10 200 python -u scripts/probe_ba.py > gpurun_out/probe_$TAG.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_$TAG.txt; exit 1; }
head -11 gpurun_out/probe_$TAG.txt
