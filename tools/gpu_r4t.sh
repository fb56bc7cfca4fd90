#!/bin/bash
# one-hash dropout mask: training tests (bf16 anchors), then
# training step vs the previous build (abl/libhvs_prev.so), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4t; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -k "train or drop or attention or act or norm" -q --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1; tail -2 $OUT/tests.log
grep -E "^E .*(Assertion|Error)" $OUT/tests.log | cut -c1-300 | head -5
for r in 1 2; do
  HV_LIB_PATH=$GRAFT_REPO_ROOT/abl/libhvs_prev.so timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/prev_$r.txt 2>&1 || { tail -20 $OUT/prev_$r.txt; exit 1; }
  echo "prev:     $(tail -1 $OUT/prev_$r.txt)"
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/hash_$r.txt 2>&1 || { tail -20 $OUT/hash_$r.txt; exit 1; }
  echo "onehash:  $(tail -1 $OUT/hash_$r.txt)"
done
