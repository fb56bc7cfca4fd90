#!/bin/bash
# round-4 batch: D=256 split-hidden A/B, the default bench (live PMC passes, B=16 CPU baseline,
# graph training), prep tests (vectorised cast, XCD-local fold tiles) + manifold regulariser test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4e; mkdir -p $OUT
bash tools/ab_mhc256.sh m256 || exit 1
bash tools/gpu_round.sh r4e bench || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_prep.py tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -k "prep or wprep or manifold_regularization" > $OUT/prep_tests.log 2>&1
tail -3 $OUT/prep_tests.log
