#!/bin/bash
# Same-box A/B of two HVOptions settings (HV_OPTS, parsed by tools/quick_bench.py and tools/lat_prof.py):
# B=16 graph step and B=1 frozen p50, alternating.  usage: bash tools/ab_opts.sh <out dir> <opts A> <opts B> [rounds]
# (AB_VAR=HV_SET: the arms are hv_amd module switches instead, e.g. detect.LATERALS_BESIDE_VIT=False)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; A=$2; B=$3; R=${4:-2}
mkdir -p $OUT
for i in $(seq $R); do
  for o in "$A" "$B"; do
    export ${AB_VAR:-HV_OPTS}="$o"
    timeout -k 10 200 python -u tools/quick_bench.py "[$o]" >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
    echo -n "[$o]: " >> $OUT/ab.txt
    timeout -k 10 200 python -u tools/lat_prof.py 200 >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
    if [ -n "$AB_RECOMPUTE" ]; then
      echo -n "[$o]: " >> $OUT/ab.txt
      HV_LAT_RECOMPUTE=1 timeout -k 10 200 python -u tools/lat_prof.py 200 >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
    fi
  done
done
unset HV_OPTS HV_SET
cat $OUT/ab.txt
