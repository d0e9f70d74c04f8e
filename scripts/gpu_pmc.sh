#!/bin/bash
# HBM traffic of the roofline kernels: two separate rocprofv3 --pmc passes of
# scripts/pmc_run.py (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2:
# MI355X_MICROARCH.md), each with its own per-scan log, then
# scripts/pmc_summary.py pairs every dispatch with its scan. Outputs under
# gpurun_out/pmc_<tag>/ and gpurun_out/pmc_traffic_<tag>.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-cur}
D=gpurun_out/pmc_$TAG
mkdir -p $D/fetch $D/write
# P_k of every scan (per-stage profiling), outside the counter passes
timeout -k 10 300 python3 scripts/pmc_run.py --stages --out $D/scans_pk.json > $D/pk.log 2>&1 || { echo "P_k run failed"; tail -20 $D/pk.log; exit 1; }
for P in fetch write; do
  C=$([ $P = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $D/$P -o run -- python3 scripts/pmc_run.py --out $D/$P/scans.json > $D/$P.log 2>&1 || { echo "$P pass failed"; tail -20 $D/$P.log; exit 1; }
done
python3 scripts/pmc_summary.py $D gpurun_out/pmc_traffic_$TAG.json > $D/summary.out 2>&1 || { echo "summary failed"; tail -20 $D/summary.out; exit 1; }
head -c 3000 $D/summary.out
