#!/bin/bash
# Same-box A/B of the per-forward prep kernels (rocprofv3 over tools/prep_time.py) + tools/ab_libs.sh; usage: bash tools/ab_prep.sh <out dir> <lib A>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; A=$2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_prep.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -2 $O/t.log
for lib in "$A" ""; do
  tag=${lib:+prev}; tag=${tag:-cur}
  if [ -n "$lib" ]; then export HV_LIB_PATH=$lib; else unset HV_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv -- python tools/prep_time.py > $O/$tag.log 2>&1 || exit 1
  python tools/prof_summary.py $(dirname $(find $O/$tag -name run_kernel_stats.csv | head -1)) 30 6
done
unset HV_LIB_PATH
bash tools/ab_libs.sh $O "$A" 2
