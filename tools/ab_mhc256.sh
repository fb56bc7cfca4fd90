#!/bin/bash
# Split-hidden fused mHC at D = 256 (HV_MV_SPLIT256) and the split-wait chunk loop (variant 12):
# kernel tests, per-shape A/B against the unfused chain, in-model A/B (B=16 and B=1 graphs).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-m256}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread -k "split_hidden or fused" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
HV_MHC_VARIANTS=0,512,524 timeout -k 10 300 python -u tools/mhc_ab.py 256:401:2 256:6416:2 256:25600:2 256:102400:2 > $OUT/mhc_ab256.txt 2>&1 || { tail -20 $OUT/mhc_ab256.txt; exit 1; }
grep "TF/s" $OUT/mhc_ab256.txt
HV_MHC_VARIANTS=0,12 timeout -k 10 300 python -u tools/mhc_ab.py 128:102400:4 128:25600:4 > $OUT/mhc_ab128.txt 2>&1 || { tail -20 $OUT/mhc_ab128.txt; exit 1; }
grep "TF/s" $OUT/mhc_ab128.txt
timeout -k 10 300 python -u tools/model_ab.py default mhc_variant=512 > $OUT/model_ab_512.txt 2>&1 || { tail -20 $OUT/model_ab_512.txt; exit 1; }
tail -4 $OUT/model_ab_512.txt
timeout -k 10 300 python -u tools/model_ab.py mhc_variant=512 mhc_variant=524 > $OUT/model_ab_524.txt 2>&1 || { tail -20 $OUT/model_ab_524.txt; exit 1; }
tail -4 $OUT/model_ab_524.txt
timeout -k 10 300 python -u tools/model_ab.py default mhc_variant=512 1 > $OUT/model_ab_b1.txt 2>&1 || { tail -20 $OUT/model_ab_b1.txt; exit 1; }
tail -4 $OUT/model_ab_b1.txt
