cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t6
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q --timeout 300 --timeout-method thread > gpurun_out/t6/train_tests.log 2>&1
echo "train tests rc=$?"
grep -E "FAIL|passed|failed|Error" gpurun_out/t6/train_tests.log | tail -10
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/ddp_gpu_check.py > gpurun_out/t6/ddp.log 2>&1; echo "ddp rc=$?"; grep rank gpurun_out/t6/ddp.log | tail -4
timeout -k 10 300 python -u tools/train_diag.py time 16 640 > gpurun_out/t6/time16.log 2>&1; echo "time rc=$?"; tail -1 gpurun_out/t6/time16.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/t6/prof -o run --output-format csv -- python tools/train_diag.py time 8 640 > gpurun_out/t6/prof.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/t6/prof -name 'run_kernel_stats.csv' | head -1); python tools/prof_summary.py $(dirname $f) 5 30 > gpurun_out/t6/prof_summary.txt; head -32 gpurun_out/t6/prof_summary.txt
