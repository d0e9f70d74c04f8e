#!/bin/bash
# rehearsal of the driver's N > 1 bench flow on a one-GPU box: torch.distributed.run
# with N ranks, every rank on GPU 0, gloo for the barriers / max over ranks
# (VG_BENCH_REHEARSE=1; replica mode). Checks the launch, rendezvous, per-rank
# sequences, timing and rank-0 line; RCCL itself needs one GPU per rank.
set -o pipefail
mkdir -p gpurun_out
N=${N:-2}
VG_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port ${PORT:-29533} bench.py --gpus $N --steps 20 --warmup 12 \
  > gpurun_out/rehearse_$N.json 2> gpurun_out/rehearse_$N.log
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/rehearse_$N.log
python -c "import json; d=json.load(open('gpurun_out/rehearse_$N.json')); print(d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'], d.get('rehearsal'))"
