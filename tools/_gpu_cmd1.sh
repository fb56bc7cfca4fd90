cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pf
timeout -k 10 600 python -u -m pytest tests/test_gpu_prep.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-latency --no-train --steps 20 > gpurun_out/pf/prof.log 2>&1; echo "prof rc=$?"; tail -1 gpurun_out/pf/prof.log | cut -c1-120
f=$(find gpurun_out/pf/prof -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python3 tools/prof_summary.py $d 29 60 > gpurun_out/pf/prof_summary.txt; grep -E "GPU kernel|k_pg|k_wprep" gpurun_out/pf/prof_summary.txt
