#!/bin/bash
# round-4 final record: smoke, default bench (live PMC passes, CPU baseline, latency, streaming,
# large, training), inference / B=1 / training kernel traces, training GEMM breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu_round.sh r4final smoke bench profinf latprof trainprof || exit 1
timeout -k 10 300 python -u tools/train_gemm_breakdown.py 16 > gpurun_out/r4final/train_gemm_breakdown.txt 2>&1 || { tail -30 gpurun_out/r4final/train_gemm_breakdown.txt; exit 1; }
head -30 gpurun_out/r4final/train_gemm_breakdown.txt
