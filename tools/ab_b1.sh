#!/bin/bash
# Batch-1 (config E) diagnostics: fused mHC workgroup shapes at the B=1 token counts, frozen
# graph p50 and its rocprofv3 kernel trace.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-b1}; mkdir -p $OUT
HV_MHC_VARIANTS=0,5,2,10 timeout -k 10 300 python -u tools/mhc_ab.py 128:6400 128:1600 64:25600 64:102400 32:102400 > $OUT/mhc_ab_b1.txt 2>&1 || { tail -20 $OUT/mhc_ab_b1.txt; exit 1; }
grep "ms" $OUT/mhc_ab_b1.txt
timeout -k 10 120 python -u tools/lat_prof.py 50 > $OUT/lat.txt 2>&1 || { tail -20 $OUT/lat.txt; exit 1; }
cat $OUT/lat.txt
bash tools/gpu_round.sh $1 latprof
