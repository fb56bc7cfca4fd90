#!/bin/bash
# A/B of the software-pipelined per-wave fused mHC kernel (HV_MV shape 8/9) against the per-wave
# kernel (shape 10): bitwise tests (kernel and whole model), in-model graph replay.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-mhcpipe}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread -k "pipelined" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 300 python -u tools/model_ab.py mhc_variant=10 mhc_variant=9 > $OUT/model_ab.txt 2>&1 || { tail -20 $OUT/model_ab.txt; exit 1; }
cat $OUT/model_ab.txt
