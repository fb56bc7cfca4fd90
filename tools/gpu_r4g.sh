#!/bin/bash
# round-4: SE gate (n > 4 fused mean) + D=256 token-count policy + prefetching gradient epilogue:
# tests, in-model A/Bs (B=16, B=1), training-step A/B of HV_GV_TRAIN_PF (alternating)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4g; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_prep.py -q --timeout 200 --timeout-method thread -k "se_ or staged_epilogue or seed_offset or prep" > $OUT/tests_k.log 2>&1 || { tail -30 $OUT/tests_k.log; exit 1; }
tail -2 $OUT/tests_k.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py -q --timeout 200 --timeout-method thread > $OUT/tests_model.log 2>&1 || { tail -30 $OUT/tests_model.log; exit 1; }
tail -2 $OUT/tests_model.log
timeout -k 10 300 python -u tools/model_ab.py default fused_se_gate=0 > $OUT/ab_se16.txt 2>&1 || { tail -20 $OUT/ab_se16.txt; exit 1; }
tail -2 $OUT/ab_se16.txt
timeout -k 10 300 python -u tools/model_ab.py default mhc256_min_tokens=1000000000 > $OUT/ab_m256_16.txt 2>&1 || { tail -20 $OUT/ab_m256_16.txt; exit 1; }
tail -2 $OUT/ab_m256_16.txt
timeout -k 10 300 python -u tools/model_ab.py default fused_se_gate=0 1 > $OUT/ab_se1.txt 2>&1 || { tail -20 $OUT/ab_se1.txt; exit 1; }
tail -2 $OUT/ab_se1.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/train_def_$r.txt 2>&1 || { tail -20 $OUT/train_def_$r.txt; exit 1; }
  tail -1 $OUT/train_def_$r.txt
  HV_GEMM_VARIANT=0x100000 timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/train_pf_$r.txt 2>&1 || { tail -20 $OUT/train_pf_$r.txt; exit 1; }
  tail -1 $OUT/train_pf_$r.txt
done
bash tools/gpu_round.sh r4g profinf || exit 1
