#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4q; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp.py -q -s --timeout 280 --timeout-method thread > $OUT/tests.log 2>&1; tail -3 $OUT/tests.log
grep -h "rank [01]:" $OUT/tests.log | cut -c1-200
