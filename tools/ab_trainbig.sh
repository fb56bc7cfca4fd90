#!/bin/bash
# Training GEMMs on the 256x256 ping-pong kernel (opt-in HV_GV_TRAIN_BIG; default the 64x128 ring): bitwise tests, train step A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tb}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread -k "staged_epilogue or train_modes" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/t_def_$i.txt 2>&1 || { tail -20 $OUT/t_def_$i.txt; exit 1; }
  tail -1 $OUT/t_def_$i.txt
  HV_GEMM_VARIANT=0x20000 timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/t_big_$i.txt 2>&1 || { tail -20 $OUT/t_big_$i.txt; exit 1; }
  tail -1 $OUT/t_big_$i.txt
done
