#!/bin/bash
# wgrad split plan: >= 512 (built) vs >= 640 / >= 768 workgroups (abl/), alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4w; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/w512_$r.txt 2>&1 || { tail -20 $OUT/w512_$r.txt; exit 1; }
  echo ">=512: $(tail -1 $OUT/w512_$r.txt)"
  for W in 640 768; do
    HV_LIB_PATH=$GRAFT_REPO_ROOT/abl/libhvs_wg$W.so timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/w${W}_$r.txt 2>&1 || { tail -20 $OUT/w${W}_$r.txt; exit 1; }
    echo ">=$W: $(tail -1 $OUT/w${W}_$r.txt)"
  done
done
