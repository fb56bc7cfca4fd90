#!/bin/bash
# full GPU suite + inference kernel trace (fold GEMM back on the 32-deep tile)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r4m tests profinf || exit 1
