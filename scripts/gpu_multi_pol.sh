#!/bin/bash
# multi-sequence wait-policy sweep (scripts/multi_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
nproc > gpurun_out/multi_pol_env.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/multi_pol_env.txt 2>/dev/null
GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python -u scripts/multi_probe.py 64line 0,0 20,20 50,50 -- 2 4 8 > gpurun_out/multi_pol.jsonl 2> gpurun_out/multi_pol.err || { tail -5 gpurun_out/multi_pol.err; exit 1; }
cat gpurun_out/multi_pol_env.txt gpurun_out/multi_pol.jsonl
