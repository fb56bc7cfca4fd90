#!/bin/bash
# Same-box A/B of two builds of libhvs.so: B=16 graph step (tools/quick_bench.py) and B=1 frozen
# frame p50 (tools/lat_prof.py), alternating runs.  usage: bash tools/ab_libs.sh <out dir> <lib A> [rounds]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; A=$2; R=${3:-2}
mkdir -p $OUT
for i in $(seq $R); do
  for lib in "$A" ""; do
    tag=${lib:-current}
    if [ -n "$lib" ]; then export HV_LIB_PATH=$lib; else unset HV_LIB_PATH; fi
    timeout -k 10 200 python -u tools/quick_bench.py $tag >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
    echo -n "$tag: " >> $OUT/ab.txt
    timeout -k 10 200 python -u tools/lat_prof.py 200 >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
  done
done
unset HV_LIB_PATH
cat $OUT/ab.txt
