#!/bin/bash
# full GPU suite, cross-build A/B (lib/ = working tree, lib_alt/ = HEAD), then kernel stats of both builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05pw}
timeout -k 10 600 python -u -m pytest tests/test_ba_hessian_gpu.py tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_shard_gpu.py tests/test_multi_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_ARGS="--no-tile1 --multi= --multi-1m=" bash scripts/ab.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
for v in lib lib_alt; do
  VINA_GPU_LIB=vina-slam_amd/$v/libvina_gpu.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ks_${TAG}_$v -o run -- python3 bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --no-tile1 --multi= --multi-1m= > gpurun_out/ks_${TAG}_$v.log 2>&1 || { tail -5 gpurun_out/ks_${TAG}_$v.log; exit 1; }
  f=$(find gpurun_out/ks_${TAG}_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -E "k_ba_hfinal|k_ba_prep|k_ba_solve|k_push_window" "$f" | cut -d, -f1-6
done
