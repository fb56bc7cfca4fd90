#!/bin/bash
# one SQ counter pass over the bench workload's eager forwards (bench.py --pmc-child), per-kernel
# summary for the next round's kernel work
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r4x; mkdir -p $OUT
trap 'find gpurun_out -name "*counter_collection.csv" -size +4M -delete; du -sh gpurun_out' EXIT
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --pmc-child --size 640 --batch 16 --precision bf16 > $OUT/pmc_sq.log 2>&1 || { tail -5 $OUT/pmc_sq.log; exit 1; }
python tools/pmc_kernel_summary.py $OUT/pmc_sq 14 > $OUT/pmc_sq_summary.txt; head -8 $OUT/pmc_sq_summary.txt | cut -c1-200
