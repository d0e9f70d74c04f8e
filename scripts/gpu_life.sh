set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${TAG:-a}
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_lifetime_gpu.py > gpurun_out/life_r05$T.log 2>&1 || { tail -60 gpurun_out/life_r05$T.log; exit 1; }
grep -E "PASS|FAIL|peak|max_nodes|shrink|compacted" gpurun_out/life_r05$T.log | tail -20
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stage_api_gpu.py tests/test_pipeline_gpu.py -k "fused or resident or nodrain or long or path" > gpurun_out/life2_r05$T.log 2>&1 || { tail -60 gpurun_out/life2_r05$T.log; exit 1; }
tail -5 gpurun_out/life2_r05$T.log
