#!/bin/bash
# wgrad plan >= 512 workgroups: training tests (bf16 anchors), one-GPU 2-rank DDP test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4p; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_ddp.py -q --timeout 250 --timeout-method thread > $OUT/tests.log 2>&1; tail -4 $OUT/tests.log
grep -E "^E .*(Assertion|Error)" $OUT/tests.log | cut -c1-300 | head -5
