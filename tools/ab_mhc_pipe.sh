#!/bin/bash
# A/B of the fused mHC kernel restructurings: the software-pipelined per-wave kernel (HV_MV shape
# 8/9, D = 32/64) against the per-wave kernel (shape 10), and the split-hidden D = 128 kernel with
# untracked DMAs; bitwise tests (kernel and whole model), kernel timings, in-model graph replay.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-mhcpipe}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -v --timeout 200 --timeout-method thread -k "pipelined or survives or split_hidden or workgroup_shapes or fused_kernel_matches" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
HV_MHC_VARIANTS=10,8,9 timeout -k 10 300 python -u tools/mhc_ab.py 32:1638400 64:1638400 64:409600 128:102400 128:25600 > $OUT/mhc_ab.txt 2>&1 || { tail -20 $OUT/mhc_ab.txt; exit 1; }
grep "ms" $OUT/mhc_ab.txt
timeout -k 10 300 python -u tools/model_ab.py mhc_variant=10 mhc_variant=9 > $OUT/model_ab.txt 2>&1 || { tail -20 $OUT/model_ab.txt; exit 1; }
cat $OUT/model_ab.txt
