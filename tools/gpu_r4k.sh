#!/bin/bash
# full GPU test suite on the current build + the training determinism probe (fp32, bf16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; tail -6 $OUT/tests.log
grep -E "^FAILED|^E .*Error" $OUT/tests.log | cut -c1-250 | head -20
for p in fp32 bf16; do
  timeout -k 10 200 python -u tools/train_bisect.py 0 $p > $OUT/bisect_$p.txt 2>&1 || { tail -20 $OUT/bisect_$p.txt; exit 1; }
  grep variant $OUT/bisect_$p.txt
done
