#!/bin/bash
# round-4 closing record of the final build: full GPU suite, smoke, default bench (live PMC,
# CPU baseline, latency, streaming, large, training), inference / B=1 / training traces, and one
# SQ counter pass over a B=4 training run (the write-bound training GEMMs, for the next round)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# keep the merge-back under gpurun's 64 MiB whatever happens: summaries stay, raw CSVs go
trap 'find gpurun_out -name "*kernel_trace.csv" -delete; find gpurun_out -name "*counter_collection.csv" -size +4M -delete; du -sh gpurun_out' EXIT
bash tools/gpu_round.sh r4close tests smoke bench profinf latprof trainprof || exit 1
OUT=gpurun_out/r4close
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq -o run --output-format csv -- python tools/train_diag.py time 4 640 > $OUT/pmc_sq.log 2>&1 || { tail -5 $OUT/pmc_sq.log; exit 1; }
python tools/pmc_kernel_summary.py $OUT/pmc_sq 10 > $OUT/pmc_sq_summary.txt; head -20 $OUT/pmc_sq_summary.txt
