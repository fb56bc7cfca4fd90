#!/bin/bash
# One GPU validation pass: gpu parity tests, smoke, bench (with CPU baseline), rocprofv3 kernel trace.
# usage: bash tools/gpu_round.sh <tag> [tests|bench|prof ...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for step in "$@"; do
  case $step in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; } ; tail -3 $OUT/tests.log ;;
    ktests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/ktests.log 2>&1 || { tail -40 $OUT/ktests.log; exit 1; } ; tail -3 $OUT/ktests.log ;;
    vitprobe) timeout -k 10 300 python -u tools/vit_grad_probe.py > $OUT/vit_grad_probe.txt 2>&1 || { tail -30 $OUT/vit_grad_probe.txt; exit 1; } ; head -60 $OUT/vit_grad_probe.txt ;;
    streamab) timeout -k 10 600 python -u tools/vit_grad_probe.py stream_ab > $OUT/vit_stream_ab.txt 2>&1 || { tail -30 $OUT/vit_stream_ab.txt; exit 1; } ; grep seed $OUT/vit_stream_ab.txt ;;
    determinism) timeout -k 10 600 python -u tools/vit_grad_probe.py determinism > $OUT/determinism.txt 2>&1 || { tail -30 $OUT/determinism.txt; exit 1; } ; grep differ $OUT/determinism.txt ;;
    preptime) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/preptime -o run --output-format csv -- python tools/prep_time.py > $OUT/preptime.log 2>&1 || { tail -30 $OUT/preptime.log; exit 1; } ; f=$(find $OUT/preptime -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 32 20 > $OUT/preptime_summary.txt; head -14 $OUT/preptime_summary.txt ;;
    sweep) timeout -k 10 400 python -u tools/tile_sweep.py > $OUT/tile_sweep.txt 2>&1 || { tail -30 $OUT/tile_sweep.txt; exit 1; } ; cat $OUT/tile_sweep.txt ;;
    bisect640) timeout -k 10 900 python -u tools/vit_grad_probe.py bisect640 attn32+lin32+qkv32 > $OUT/bisect640.txt 2>&1 || { tail -30 $OUT/bisect640.txt; exit 1; } ; grep MEDIAN $OUT/bisect640.txt ;;
    nmstime) timeout -k 10 300 python -u tools/nms_time.py 1 > $OUT/nms_time.txt 2>&1 && timeout -k 10 300 python -u tools/nms_time.py 16 >> $OUT/nms_time.txt 2>&1 || { tail -30 $OUT/nms_time.txt; exit 1; } ; grep -v amdgpu.ids $OUT/nms_time.txt ;;
    vitbisect) for m in attn32 lin32 qkv32; do timeout -k 10 300 python -u tools/vit_grad_probe.py vit_encoder $m > $OUT/vit_grad_probe_$m.txt 2>&1 || { tail -30 $OUT/vit_grad_probe_$m.txt; exit 1; } ; grep "==" $OUT/vit_grad_probe_$m.txt ; done ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -30 $OUT/smoke.log; exit 1; } ; tail -2 $OUT/smoke.log ;;
    bench) timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; } ; cat $OUT/bench.json ;;
    benchq) timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --no-latency --no-stream --no-large > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; } ; cat $OUT/bench.json ;;
    prof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-latency --no-stream --no-large --steps 20 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; } ; f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 29 40 > $OUT/prof_summary.txt; head -25 $OUT/prof_summary.txt ;;
    profss) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/profss -o run --output-format csv -- python bench.py --single-stream --no-pmc --no-cpu-baseline --no-latency --no-train --no-stream --no-large --steps 20 > $OUT/profss.log 2>&1 || { tail -30 $OUT/profss.log; exit 1; } ; f=$(find $OUT/profss -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 24 40 > $OUT/profss_summary.txt; python tools/gemm_family_avg.py $f >> $OUT/profss_summary.txt; grep -h '"avg_launch_ms"' $OUT/profss.log | head -1; tail -2 $OUT/profss_summary.txt ;;
    profinf) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/profinf -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-latency --no-train --no-stream --no-large --steps 20 > $OUT/profinf.log 2>&1 || { tail -30 $OUT/profinf.log; exit 1; } ; f=$(find $OUT/profinf -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 29 40 > $OUT/profinf_summary.txt; head -25 $OUT/profinf_summary.txt ;;
    breakdown) timeout -k 10 300 python -u tools/gemm_breakdown.py > $OUT/gemm_breakdown.txt 2>&1 || { tail -30 $OUT/gemm_breakdown.txt; exit 1; } ; head -50 $OUT/gemm_breakdown.txt ;;
    pmc) for c in FETCH_SIZE WRITE_SIZE; do timeout -s KILL 300 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-latency --no-train --no-stream --no-large --steps 2 --warmup 1 > $OUT/pmc_$c.log 2>&1 || { tail -30 $OUT/pmc_$c.log; exit 1; } ; done ; python tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $OUT/pmc_traffic.json ;;
    mfma) timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
          i=0
          for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
                     "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
            i=$((i+1)); cs=""
            for c in $set; do if grep -qw "$c" $OUT/counters.txt; then cs="$cs $c"; else echo "counter $c not listed"; fi; done
            timeout -s KILL 240 rocprofv3 --pmc $cs -d $OUT/mfma_p$i -o run --output-format csv -- python bench.py --no-pmc --no-cpu-baseline --no-latency --no-train --no-stream --no-large --steps 2 --warmup 1 > $OUT/mfma_p$i.log 2>&1 || { tail -30 $OUT/mfma_p$i.log; exit 1; }
          done
          python tools/pmc_mfma.py $OUT/pmc_mfma.json $OUT/mfma_p1 $OUT/mfma_p2 > $OUT/pmc_mfma.txt; head -50 $OUT/pmc_mfma.txt ;;
    latprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/latprof -o run --output-format csv -- python tools/lat_prof.py > $OUT/latprof.log 2>&1 || { tail -30 $OUT/latprof.log; exit 1; } ; f=$(find $OUT/latprof -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 1 40 > $OUT/latprof_summary.txt; python tools/frame_kernels.py $OUT/latprof > $OUT/latprof_frame.txt; head -25 $OUT/latprof_frame.txt ;;
    trainprof) timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trainprof -o run --output-format csv -- python tools/train_diag.py time 16 640 > $OUT/trainprof.log 2>&1 || { tail -30 $OUT/trainprof.log; exit 1; } ; f=$(find $OUT/trainprof -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python tools/prof_summary.py $d 6 45 > $OUT/trainprof_summary.txt; head -30 $OUT/trainprof_summary.txt ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
