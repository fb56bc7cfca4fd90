#!/bin/bash
# round-4: coalesced 128-deep fold GEMM, composed SE gate, default prefetching gradient epilogue,
# prefetching column reductions: tests, inference kernel trace (k_pg3), training kernel trace +
# per-shape training GEMM breakdown
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4h; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_prep.py tests/test_gpu_kernels.py tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "prep or se_ or train or colsum or bn or rownorm or grad or wgrad" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
bash tools/gpu_round.sh r4h profinf || exit 1
bash tools/gpu_round.sh r4h trainprof || exit 1
timeout -k 10 300 python -u tools/train_gemm_breakdown.py 16 > $OUT/train_gemm_breakdown.txt 2>&1 || { tail -30 $OUT/train_gemm_breakdown.txt; exit 1; }
head -40 $OUT/train_gemm_breakdown.txt
