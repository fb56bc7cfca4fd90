cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t8
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q --timeout 300 --timeout-method thread > gpurun_out/t8/train_tests.log 2>&1
echo "train tests rc=$?"
grep -E "FAIL|passed|failed|Error" gpurun_out/t8/train_tests.log | tail -10
timeout -k 10 300 python -u tools/train_diag.py time 16 640 > gpurun_out/t8/time16.log 2>&1; echo "time rc=$?"; tail -1 gpurun_out/t8/time16.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/t8/prof -o run --output-format csv -- python tools/train_diag.py time 16 640 > gpurun_out/t8/prof.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/t8/prof -name 'run_kernel_stats.csv' | head -1); python tools/prof_summary.py $(dirname $f) 5 30 > gpurun_out/t8/prof_summary.txt; head -32 gpurun_out/t8/prof_summary.txt
