#!/bin/bash
# the sharded parity test (exchange logs per rank) under the current build, then under lib_alt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/arA gpurun_out/arB
VG_AR_LOG=$PWD/gpurun_out/arA/log timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/shard_A.log 2>&1; echo "A rc=$?"; tail -4 gpurun_out/shard_A.log
VG_AR_LOG=$PWD/gpurun_out/arB/log VINA_GPU_LIB=$PWD/vina-slam_amd/lib_alt/libvina_gpu.so timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/shard_B.log 2>&1; echo "B rc=$?"; tail -4 gpurun_out/shard_B.log
