#!/bin/bash
# the sharded parity test under the current build and under lib_alt2 (bisect)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/shard_A.log 2>&1; echo "A rc=$?"; tail -3 gpurun_out/shard_A.log
VINA_GPU_LIB=$PWD/vina-slam_amd/lib_alt2/libvina_gpu.so timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/shard_C.log 2>&1; echo "C rc=$?"; tail -3 gpurun_out/shard_C.log
