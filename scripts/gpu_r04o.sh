set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/probe_recut.py > gpurun_out/probe_recut_r04t.txt 2>&1 &&
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline_gpu.py tests/test_stage_api_gpu.py tests/test_memo_gpu.py > gpurun_out/test_r04t.txt 2>&1 &&
for i in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi= --multi-1m= > gpurun_out/bench_r04t_$i.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/bench_r04t_$i.json')); print(d['value'], d['ms_per_step'])"; done
