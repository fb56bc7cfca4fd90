#!/bin/bash
# Epilogue load batching (GEMM + fused mHC) and the B-resident small-K kernel: kernel tests,
# small-K probe, same-box A/B of the HEAD build (libhvs_base.so) vs this build, in-model variant A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-epi}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread -k "gemm or conv or smallk or pingpong or mhc or survives or train or layernorm or norm" > $OUT/ktests.log 2>&1 || { tail -30 $OUT/ktests.log; exit 1; }
tail -2 $OUT/ktests.log
HV_SK_EXTRA=res3=0x8006,res4=0x10006 timeout -k 10 300 python -u tools/sk_probe.py > $OUT/sk_probe.txt 2>&1 || { tail -20 $OUT/sk_probe.txt; exit 1; }
cat $OUT/sk_probe.txt
for i in 1 2 3; do
  HV_LIB_PATH=$GRAFT_REPO_ROOT/humanoid-vision-system_amd/hv_amd/libhvs_base.so timeout -k 10 120 python tools/quick_bench.py base >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/quick_bench.py new >> $OUT/ab.txt 2>&1 || exit 1
done
cat $OUT/ab.txt
timeout -k 10 300 python -u tools/model_ab.py default gemm_variant=0x10000 > $OUT/model_ab.txt 2>&1 || { tail -20 $OUT/model_ab.txt; exit 1; }
cat $OUT/model_ab.txt
timeout -k 10 300 python -u tools/model_ab.py default gemm_variant=0x10000 1 > $OUT/model_ab_b1.txt 2>&1 || { tail -20 $OUT/model_ab_b1.txt; exit 1; }
cat $OUT/model_ab_b1.txt
