#!/bin/bash
# multi-sequence B sweep under several hardware-queue limits (one stream per sequence)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
: > gpurun_out/multi_q.jsonl
for Q in 4 6 8; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python -u scripts/multi_probe.py 64line 0,0 -- 2 4 8 16 4 >> gpurun_out/multi_q.jsonl 2> gpurun_out/multi_q.err || { tail -5 gpurun_out/multi_q.err; exit 1; }
done
cat gpurun_out/multi_q.jsonl
