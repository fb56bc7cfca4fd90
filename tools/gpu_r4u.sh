#!/bin/bash
# rebuilt closing library: smoke + GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r4u smoke tests || exit 1
