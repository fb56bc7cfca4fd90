cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t9
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_model.py -q --timeout 300 --timeout-method thread > gpurun_out/t9/tests.log 2>&1
echo "tests rc=$?"
grep -E "FAIL|passed|failed|Error" gpurun_out/t9/tests.log | tail -10
timeout -k 10 300 python -u tools/train_diag.py time 16 640 > gpurun_out/t9/time16.log 2>&1; echo "time rc=$?"; tail -2 gpurun_out/t9/time16.log
timeout -k 10 300 python -u tools/train_diag.py time 4 640 > gpurun_out/t9/time4.log 2>&1; echo "time rc=$?"; tail -2 gpurun_out/t9/time4.log
