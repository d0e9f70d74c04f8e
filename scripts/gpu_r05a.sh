#!/bin/bash
# round 5, first call: the -m gpu suite on the deferred-LM build, a same-build
# A/B of the deferral (vgx_debug 26), the kernel-trace timeline, and the
# environment rocprofv3 --pmc hands to its target (serial-kernel detection)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r05a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { tail -40 gpurun_out/gputest_$TAG.log; exit 1; }
tail -1 gpurun_out/gputest_$TAG.log
AB_DEBUG="26=0" AB_ROUNDS=3 bash scripts/ab_env.sh > gpurun_out/ab_$TAG.txt 2>&1 || { cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES -d gpurun_out/pmcenv_$TAG -o run -- python3 -c "import os, json; print(json.dumps({k: v for k, v in os.environ.items() if 'ROC' in k or 'HSA' in k or 'AMD' in k}))" > gpurun_out/pmcenv_$TAG.txt 2>&1 || true
