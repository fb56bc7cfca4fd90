#!/bin/bash
# round-3 A/B: conv address path (libhvs.so vs libhvs_base.so), fused-mHC NOMERGE variant, kernel tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r3e; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv or gemm or pingpong" > $OUT/ktests.log 2>&1 || { tail -30 $OUT/ktests.log; exit 1; }
tail -2 $OUT/ktests.log
for i in 1 2 3; do
  HV_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-vision-system_amd/hv_amd/libhvs_base.so timeout -k 10 120 python tools/quick_bench.py base >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/quick_bench.py new >> $OUT/ab.txt 2>&1 || exit 1
done
cat $OUT/ab.txt
HV_MHC_VARIANTS=0,7 timeout -k 10 300 python tools/mhc_ab.py 32:1638400 32:409600 64:409600 64:1638400 64:102400 > $OUT/mhc_ab.txt 2>&1 || exit 1
grep "ms" $OUT/mhc_ab.txt
timeout -k 10 200 python tools/model_ab.py default mhc_variant=7 > $OUT/model_ab.txt 2>&1 || exit 1
cat $OUT/model_ab.txt
timeout -k 10 200 python tools/gemm_breakdown.py > $OUT/gemm_breakdown.txt 2>&1 || exit 1
head -60 $OUT/gemm_breakdown.txt
HV_SWEEP_ONLY=conv3x3 timeout -k 10 300 python tools/tile_sweep.py > $OUT/tile_sweep_conv.txt 2>&1 || exit 1
cat $OUT/tile_sweep_conv.txt
