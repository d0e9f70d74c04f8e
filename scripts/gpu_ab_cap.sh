#!/bin/bash
# one GPU call: same-box A/B (lib/ vs lib_alt/) then the context-capacity probe
# (default capacities vs sized ones) on the single-sequence and B=4 legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AB_ARGS="--multi=" bash scripts/ab.sh || exit 1
for cap in "" "--max-nodes 1000000 --max-fix 3000000 --hash-log2 20"; do
  timeout -k 10 200 python bench.py --no-cpu --stage-scans 0 --target-steps 0 --no-h2d --multi=4 $cap > gpurun_out/cap.json 2>/dev/null || { echo "cap bench failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/cap.json')); print('cap[$cap]', d['value'], d['ms_per_step'], d['multi_sequence']['by_B'], d['config'].get('nodes_used_end'), d['config'].get('fix_used_end'))"
done
