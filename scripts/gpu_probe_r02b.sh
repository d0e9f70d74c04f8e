set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
TAG=r02b bash scripts/gpu_trace.sh > gpurun_out/trace.out 2>&1 || exit 1
python3 scripts/trace_scan.py gpurun_out/trace_r02b/run_kernel_trace.csv 20 > gpurun_out/trace_summary.txt || exit 1
for B in 1 2 4 8; do timeout -k 10 200 python -u scripts/mp_probe.py $B 64line 150 >> gpurun_out/mp.jsonl 2>> gpurun_out/mp.err || exit 1; done
GPU_MAX_HW_QUEUES=4 timeout -k 10 200 python -u scripts/batch_probe.py 64line 1 2 4 > gpurun_out/batch4.jsonl 2> gpurun_out/batch4.err
