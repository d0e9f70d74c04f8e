#!/bin/bash
# Round-3 GPU call: every -m gpu test, the default bench line, the k_ba_solve
# phase clocks (probe build), a same-box A/B (lib = A vs lib_alt = B) and the
# rocprofv3 kernel-trace stats of the bench command. Each step under its own
# limit, stop at the first failure. Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03b}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TEST_ARGS} > gpurun_out/gputest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$TAG.log
  [ $rc -ne 0 ] && { tail -30 gpurun_out/gputest_$TAG.log; exit $rc; }
  tail -2 gpurun_out/gputest_$TAG.log
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  head -c 400 gpurun_out/bench_$TAG.json; echo
fi
if [ -z "$SKIP_PROBE" ]; then
  VINA_GPU_LIB=$PWD/vina-slam_amd/lib_probe/libvina_gpu.so timeout -k 10 200 python -u scripts/probe_ba.py > gpurun_out/probe_$TAG.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/probe_$TAG.txt; exit 1; }
  head -12 gpurun_out/probe_$TAG.txt
fi
if [ -z "$SKIP_AB" ]; then
  AB_ARGS="--multi= --multi-1m=" bash scripts/${AB_SCRIPT:-ab.sh} > gpurun_out/ab_$TAG.txt 2>&1 || { echo "ab failed"; cat gpurun_out/ab_$TAG.txt; exit 1; }
  cat gpurun_out/ab_$TAG.txt
fi
[ -n "$SKIP_PROF" ] && exit 0
TAG=$TAG BENCH_ARGS="--multi= --multi-1m=" bash scripts/gpu_prof.sh || exit 1
[ -n "$SKIP_TRACE" ] && exit 0
TAG=$TAG bash scripts/gpu_trace.sh > gpurun_out/trace_$TAG.out 2>&1 || { tail -5 gpurun_out/trace_$TAG.out; exit 1; }
python3 scripts/scan_timeline.py gpurun_out/trace_$TAG/run_kernel_trace.csv 4 > gpurun_out/scan_timeline_$TAG.txt && tail -1 gpurun_out/scan_timeline_$TAG.txt
