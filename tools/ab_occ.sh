#!/bin/bash
# Register-budget launch bounds on every LDS-DMA GEMM instantiation: full GPU tests, inference A/B
# of the HEAD build (ab_libs/libhvs_head.so) vs this build, one training step timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-occ}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2 3; do
  HV_LIB_PATH=$GRAFT_REPO_ROOT/ab_libs/libhvs_head.so timeout -k 10 120 python tools/quick_bench.py head >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/quick_bench.py new >> $OUT/ab.txt 2>&1 || exit 1
done
cat $OUT/ab.txt
timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/train.txt 2>&1 || { tail -20 $OUT/train.txt; exit 1; }
tail -1 $OUT/train.txt
