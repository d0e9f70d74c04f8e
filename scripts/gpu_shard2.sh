#!/bin/bash
# the sharded parity test with per-exchange digests (current build), once
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ar${TAG:-C}
PYTHONHASHSEED=0 VG_AR_LOG=$PWD/gpurun_out/ar${TAG:-C}/log timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py -m gpu -v --timeout 300 --timeout-method thread ${K:+-k $K} > gpurun_out/shard_${TAG:-C}.log 2>&1; echo "rc=$?"; tail -4 gpurun_out/shard_${TAG:-C}.log
