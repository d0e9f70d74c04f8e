#!/bin/bash
# shard parity (host transport, desync, one-rank RCCL) + pipeline/stage parity, then the tile leg A/B across builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05cc}
timeout -k 10 700 python -u -m pytest tests/test_shard_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
for i in 1 2 3; do
  for v in A B; do
    if [ $v = B ]; then export VINA_GPU_LIB=$PWD/vina-slam_amd/lib_alt/libvina_gpu.so; else unset VINA_GPU_LIB; fi
    timeout -k 10 240 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi= --multi-1m= > gpurun_out/tile_$v$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tile_$v$i.json')); t=d['tile_path_1gpu']; print('$v', d['value'], t['value'], t['overhead_ms_per_scan'])"
  done
done
