#!/bin/bash
# HBM ceiling probe; wgrad split plan >= 512 workgroups (abl/libhvs_wg512.so) vs >= 1024, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4o; mkdir -p $OUT
timeout -k 10 120 python -u tools/bw_probe.py > $OUT/bw.txt 2>&1 || { tail -10 $OUT/bw.txt; exit 1; }
tail -1 $OUT/bw.txt
for r in 1 2; do
  timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/def_$r.txt 2>&1 || { tail -20 $OUT/def_$r.txt; exit 1; }
  echo "default: $(tail -1 $OUT/def_$r.txt)"
  HV_LIB_PATH=$GRAFT_REPO_ROOT/abl/libhvs_wg512.so timeout -k 10 300 python -u tools/train_diag.py time 16 640 > $OUT/wg512_$r.txt 2>&1 || { tail -20 $OUT/wg512_$r.txt; exit 1; }
  echo "wg512:   $(tail -1 $OUT/wg512_$r.txt)"
done
