#!/bin/bash
# training regression bisection: determinism (eager vs eager vs graph) per GEMM variant, and the
# two failing tests with the per-pass gradient epilogue (HV_GV_TRAIN_NOPF)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4i; mkdir -p $OUT
for v in 0 0x100000; do
  timeout -k 10 200 python -u tools/train_bisect.py $v bf16 > $OUT/bisect_$v.txt 2>&1 || { tail -20 $OUT/bisect_$v.txt; exit 1; }
  grep variant $OUT/bisect_$v.txt
done
timeout -k 10 200 python -u tools/train_bisect.py 0 fp32 > $OUT/bisect_fp32.txt 2>&1 || { tail -20 $OUT/bisect_fp32.txt; exit 1; }
grep variant $OUT/bisect_fp32.txt
HV_TEST_GEMM_VARIANT=0x100000 timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "base_train_step_bf16 or graph_step_equals" > $OUT/tests_nopf.log 2>&1; tail -4 $OUT/tests_nopf.log
