#!/bin/bash
# kernel trace of a multi-sequence leg (B from $B) -> busy fraction + per-kernel shares
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=${B:-8}
TAG=${TAG:-mt$B}
timeout -k 10 400 rocprofv3 --kernel-trace ${EXTRA} --output-format csv -d gpurun_out/trace_$TAG -o run_%pid% -- python3 -u bench.py --no-cpu --steps 10 --stage-scans 0 --target-steps 0 --workers 1 --no-h2d --multi=$B --multi-1m= > gpurun_out/trace_$TAG.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/trace_$TAG.log; exit 1; }
tail -1 gpurun_out/trace_$TAG.log | cut -c1-300
for f in $(find gpurun_out/trace_$TAG -name '*kernel_trace.csv'); do
  n=$(wc -l < $f); echo "$f $n"
  if [ $n -gt 20000 ]; then python3 scripts/busy_union.py $f 0.5; python3 scripts/kernel_share.py $f 30; fi
done
