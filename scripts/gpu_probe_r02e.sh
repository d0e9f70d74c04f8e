#!/bin/bash
# one GPU call: multi-sequence probe (B sweep, sized contexts) and the phase
# clocks of the probed kernels (instrumented build in lib_probe/)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u scripts/multi_probe.py 64line 0,0 -- 1 2 4 8 > gpurun_out/multi_probe.jsonl 2> gpurun_out/multi_probe.err || { tail -5 gpurun_out/multi_probe.err; exit 1; }
cat gpurun_out/multi_probe.jsonl
timeout -k 10 200 python -u scripts/probe_ba.py > gpurun_out/probe_ba.txt 2>&1 || { tail -5 gpurun_out/probe_ba.txt; exit 1; }
cat gpurun_out/probe_ba.txt
