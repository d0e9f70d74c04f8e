#!/bin/bash
# sharded parity tests, then a cross-build A/B of the tile leg (lib/ = working tree, lib_alt/ = HEAD)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05tl}
timeout -k 10 600 python -u -m pytest tests/test_shard_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
for i in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=vina-slam_amd/lib/libvina_gpu.so; else L=vina-slam_amd/lib_alt/libvina_gpu.so; fi
    VINA_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi= --multi-1m= > gpurun_out/tl_$v$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/tl_$v$i.json')); t=d['tile_path_1gpu']; print('$v', d['value'], t['value'], t['overhead_ms_per_scan'])"
  done
done
