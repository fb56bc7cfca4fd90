#!/bin/bash
# round-4 batch: tests first (fused SE gate, prep, manifold regulariser, model parity), then the
# D=256 split-hidden A/B and the default bench (live PMC passes, B=16 CPU baseline, graph training)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prep.py tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "se_ or prep or wprep or manifold_regularization" > $OUT/prep_tests.log 2>&1 || { tail -30 $OUT/prep_tests.log; exit 1; }
tail -3 $OUT/prep_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -q --timeout 200 --timeout-method thread > $OUT/model_tests.log 2>&1 || { tail -30 $OUT/model_tests.log; exit 1; }
tail -3 $OUT/model_tests.log
bash tools/ab_mhc256.sh m256 || exit 1
bash tools/gpu_round.sh r4e bench || exit 1
