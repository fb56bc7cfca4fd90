#!/bin/bash
# Training step A/B of two library builds (HV_LIB_PATH): wall time per step and the training-GEMM kernel averages.
# usage: ab_trainlib.sh OUT OLD_LIB [HV_GEMM_VARIANT of a third leg]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-tl}; OLD=${2:-ab_libs/libhvs_pre.so}; mkdir -p $OUT
for i in 1 2; do
  HV_LIB_PATH=$PWD/$OLD timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/t_old_$i.txt 2>&1 || { tail -20 $OUT/t_old_$i.txt; exit 1; }
  echo "old: $(tail -1 $OUT/t_old_$i.txt)"
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/t_new_$i.txt 2>&1 || { tail -20 $OUT/t_new_$i.txt; exit 1; }
  echo "new: $(tail -1 $OUT/t_new_$i.txt)"
  if [ -n "$3" ]; then
    HV_GEMM_VARIANT=$3 timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/t_var_$i.txt 2>&1 || { tail -20 $OUT/t_var_$i.txt; exit 1; }
    echo "new+variant $3: $(tail -1 $OUT/t_var_$i.txt)"
  fi
done
HV_LIB_PATH=$PWD/$OLD timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_old -o run --output-format csv -- python tools/train_diag.py time 16 640 > $OUT/prof_old.log 2>&1 || { tail -30 $OUT/prof_old.log; exit 1; }
f=$(find $OUT/prof_old -name 'run_kernel_stats.csv' | head -1); python tools/prof_summary.py $(dirname $f) 6 45 > $OUT/prof_old_summary.txt; head -8 $OUT/prof_old_summary.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_new -o run --output-format csv -- python tools/train_diag.py time 16 640 > $OUT/prof_new.log 2>&1 || { tail -30 $OUT/prof_new.log; exit 1; }
f=$(find $OUT/prof_new -name 'run_kernel_stats.csv' | head -1); python tools/prof_summary.py $(dirname $f) 6 45 > $OUT/prof_new_summary.txt; head -8 $OUT/prof_new_summary.txt
