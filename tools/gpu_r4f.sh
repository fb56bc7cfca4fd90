#!/bin/bash
# round-4 training profile: kernel trace of base-640 B=16 training steps + per-shape GEMM breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4f; mkdir -p $OUT
bash tools/gpu_round.sh r4f trainprof || exit 1
timeout -k 10 300 python -u tools/train_gemm_breakdown.py 16 > $OUT/train_gemm_breakdown.txt 2>&1 || { tail -30 $OUT/train_gemm_breakdown.txt; exit 1; }
head -45 $OUT/train_gemm_breakdown.txt
