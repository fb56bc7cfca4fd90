cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t3
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -v --timeout 300 --timeout-method thread -k "tiny or trainer" > gpurun_out/t3/train_tests.log 2>&1
echo "train tests rc=$?"
grep -E "FAIL|passed|failed|Error" gpurun_out/t3/train_tests.log | tail -30
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latency > gpurun_out/t3/bench.json 2> gpurun_out/t3/bench.err; echo "bench rc=$?"; cut -c1-200 gpurun_out/t3/bench.json
timeout -k 10 300 python -u tools/train_diag.py grads > gpurun_out/t3/diag.log 2>&1; echo "diag rc=$?"; cat gpurun_out/t3/diag.log | tail -32
timeout -k 10 300 python -u tools/train_diag.py time 2 640 > gpurun_out/t3/time.log 2>&1; echo "time rc=$?"; tail -5 gpurun_out/t3/time.log
