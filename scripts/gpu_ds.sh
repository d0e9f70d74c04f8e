#!/bin/bash
# downsample rework: parity set (downsample, pipeline, cold start, deskew), then
# the 1M-ray single-sequence line and the default line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-ds}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_downsample_gpu.py tests/test_pipeline_gpu.py tests/test_cold_start.py tests/test_deskew.py tests/test_ba_solve_gpu.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_$TAG.log
[ $rc -ne 0 ] && { grep -B5 -A40 "Error\|assert" gpurun_out/gputest_$TAG.log | head -80; exit $rc; }
timeout -k 10 300 python3 -u bench.py --lidar 1M --no-cpu --steps 20 --stage-scans 4 --target-steps 0 --no-h2d --multi= --multi-1m=1,2,4 > gpurun_out/bench1m_$TAG.json 2> gpurun_out/bench1m_$TAG.err || { echo "1M bench failed"; tail -20 gpurun_out/bench1m_$TAG.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench1m_$TAG.json').read().strip().splitlines()[-1]); print('1M', d['value'], d['roofline']['stage_ms_per_scan'], d['multi_sequence_1M']['by_B'])"
