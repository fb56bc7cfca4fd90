cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
timeout -k 10 200 python -u tools/train_diag.py time 16 640 2>&1 | grep -v amdgpu.ids
