#!/bin/bash
# graph-training fix check: byte-upload test, probe (first-replay predictions / histories), the
# training tests and the model capture tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4l; mkdir -p $OUT; rm -f $OUT/probe_*.txt
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q --timeout 100 --timeout-method thread -k "write_bytes" > $OUT/tests_wb.log 2>&1 || { tail -30 $OUT/tests_wb.log; exit 1; }
tail -1 $OUT/tests_wb.log
for args in "0 bf16 4" "0 fp32 4" "0 bf16 0"; do
  f=$OUT/probe_$(echo $args | tr ' ' '_').txt
  timeout -k 10 200 python -u tools/train_bisect.py $args > $f 2>&1 || { tail -20 $f; exit 1; }
  grep -h "variant\|AccumulateGrad" $f | cut -c1-200
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread > $OUT/tests_train.log 2>&1; tail -4 $OUT/tests_train.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -q --timeout 200 --timeout-method thread -k "capture or graph or stream" > $OUT/tests_model.log 2>&1; tail -2 $OUT/tests_model.log
