#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/probe_ba.py iekf > gpurun_out/probe_iekf.log 2>&1 || { cat gpurun_out/probe_iekf.log; exit 1; }
cat gpurun_out/probe_iekf.log
bash scripts/gpu_check.sh
