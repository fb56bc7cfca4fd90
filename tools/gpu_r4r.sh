#!/bin/bash
# training-step A/B of GEMM tile forcing (HV_GEMM_VARIANT: 4 = 64x64 everywhere) vs default, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4r; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/def_$r.txt 2>&1 || { tail -20 $OUT/def_$r.txt; exit 1; }
  echo "default: $(tail -1 $OUT/def_$r.txt)"
  HV_GEMM_VARIANT=4 timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/v4_$r.txt 2>&1 || { tail -20 $OUT/v4_$r.txt; exit 1; }
  echo "64x64:   $(tail -1 $OUT/v4_$r.txt)"
done
