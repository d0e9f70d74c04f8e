#!/bin/bash
# full -m gpu suite with the sharded test's exchange log, then (even if a test
# failed) the three-way A/B and the kernel-trace timeline
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03d}
VG_AR_LOG=$PWD/gpurun_out/arlog timeout -k 10 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_$TAG.log
[ $rc -eq 124 ] || [ $rc -eq 137 ] && exit $rc
AB_ARGS="--multi= --multi-1m=" timeout -k 10 900 bash scripts/${AB_SCRIPT:-ab3.sh} > gpurun_out/ab_$TAG.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_$TAG.txt; exit 1; }
cat gpurun_out/ab_$TAG.txt
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
