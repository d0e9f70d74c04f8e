#!/bin/bash
# A/B/C of three builds of the library on the same box: A = lib/, B = lib_alt/, C = lib_alt2/ (3 rounds)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in A B C; do
    case $v in
      A) unset VINA_GPU_LIB ;;
      B) export VINA_GPU_LIB=$PWD/vina-slam_amd/lib_alt/libvina_gpu.so ;;
      C) export VINA_GPU_LIB=$PWD/vina-slam_amd/lib_alt2/libvina_gpu.so ;;
    esac
    timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d ${AB_ARGS} > gpurun_out/ab_$v$i.json 2>/dev/null || { echo "bench $v failed"; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$v$i.json')); print('$v', d['value'], d['ms_per_step'])"
  done
done
