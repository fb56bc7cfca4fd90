#!/bin/bash
# Reproduction attempt of round 4's profiled-launch SIGSEGV (commit b016011): the pre-fix library
# constants (64 copy segments = 2.1 KiB of by-value kernel arguments, 2 KiB byte uploads; built
# from this tree with only those two constants changed, abl/libhvs_k64.so) under one rocprofv3
# --pmc pass of a base-640 B=4 training step.  Output: gpurun_out/b016011/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/b016011; mkdir -p $O
HV_LIB_PATH=abl/libhvs_k64.so timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES -d $O/pmc -o run --output-format csv -- python tools/train_diag.py time 4 640 > $O/run.log 2>&1
rc=$?
echo "exit status $rc" | tee -a $O/run.log
tail -25 $O/run.log
