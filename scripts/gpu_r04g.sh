#!/bin/bash
# tests + probe + same-box A/B + kernel trace (gpu_r04d.sh), then the
# multi-sequence counters and the PMC traffic passes (gpu_r04f.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r04d.sh || exit 1
TAG=${TAG}f bash scripts/gpu_r04f.sh
