#!/bin/bash
# the full GPU suite, the recut phase clocks of the working tree and of HEAD (lib_probe_alt), then a cross-build A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05rc}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
for v in "" _alt; do
  VINA_GPU_LIB=vina-slam_amd/lib_probe$v/libvina_gpu.so timeout -k 10 120 python3 -u scripts/probe_recut.py > gpurun_out/probe_recut_${TAG}$v.txt 2>&1 || { cat gpurun_out/probe_recut_${TAG}$v.txt; exit 1; }
  echo "== probe$v"; cat gpurun_out/probe_recut_${TAG}$v.txt
done
AB_ARGS="--no-tile1 --multi= --multi-1m=" bash scripts/ab.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
