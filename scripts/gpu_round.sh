#!/bin/bash
# one GPU call: map/BA parity tests, phase clocks (lib_probe), same-box A/B
# (lib vs lib_alt), the bench line with the multi-sequence children
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_multi_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
tail -1 gpurun_out/rt.log
timeout -k 10 200 python -u scripts/probe_ba.py > gpurun_out/probe_ba.txt 2>&1 || { tail -5 gpurun_out/probe_ba.txt; exit 1; }
grep -A7 k_rc_apply gpurun_out/probe_ba.txt
AB_ARGS="--multi=" bash scripts/ab.sh || exit 1
timeout -k 10 400 python bench.py --no-cpu --target-steps 0 --no-h2d --stage-scans 0 --multi=2,4,8,4 > gpurun_out/bm.json 2> gpurun_out/bm.err || { tail -5 gpurun_out/bm.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bm.json')); print(d['value'], d['multi_sequence'])"
