#!/bin/bash
# k_ba_solve rework: its numpy parity + the pipeline parity set, the phase
# clocks (probe build), then a same-box A/B against lib_alt (the previous build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-solve}
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_ba_solve_gpu.py tests/test_pipeline_gpu.py tests/test_ba_hessian_gpu.py} -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_$TAG.log
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|assert" gpurun_out/gputest_$TAG.log | head -80; exit $rc; }
VINA_GPU_LIB=$PWD/vina-slam_amd/lib_probe/libvina_gpu.so timeout -k 10 200 python -u scripts/probe_ba.py > gpurun_out/probe_$TAG.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_$TAG.txt; exit 1; }
head -9 gpurun_out/probe_$TAG.txt
[ -n "$SKIP_AB" ] && exit 0
AB_ARGS="--multi= --multi-1m=" timeout -k 10 600 bash scripts/ab.sh > gpurun_out/ab_$TAG.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
