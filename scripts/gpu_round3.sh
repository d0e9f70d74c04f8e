#!/bin/bash
# one GPU call: the pipeline/stage/multi/node parity tests, a scan timeline and a same-box A/B (lib vs lib_alt)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py tests/test_node_core.py tests/test_cold_start.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
TAG=${TAG:-r02l} bash scripts/gpu_trace.sh > gpurun_out/trace.out 2>&1 || { tail -5 gpurun_out/trace.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_${TAG:-r02l}/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_${TAG:-r02l}.txt && tail -1 gpurun_out/scan_timeline_${TAG:-r02l}.txt
grep -E "k_ba_init|k_ins_prep" gpurun_out/scan_timeline_${TAG:-r02l}.txt
AB_ARGS="--multi=" bash scripts/ab.sh || exit 1
