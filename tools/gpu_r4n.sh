#!/bin/bash
# wgrad two-step register prefetch: training tests, training kernel trace, step time; inference
# trace (fold GEMM back in hardware order)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4n; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_prep.py -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
bash tools/gpu_round.sh r4n trainprof profinf || exit 1
timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/train_time.txt 2>&1 || { tail -20 $OUT/train_time.txt; exit 1; }
tail -1 $OUT/train_time.txt
