#!/bin/bash
# bisection: previous column reduction, the failing training tests + determinism probe
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "base_train_step_bf16 or graph_step_equals" > $OUT/tests.log 2>&1; tail -4 $OUT/tests.log
grep -E "^E .*AssertionError" $OUT/tests.log | cut -c1-300
timeout -k 10 200 python -u tools/train_bisect.py 0 fp32 > $OUT/bisect_fp32.txt 2>&1 || { tail -20 $OUT/bisect_fp32.txt; exit 1; }
grep variant $OUT/bisect_fp32.txt
