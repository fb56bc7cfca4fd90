cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
timeout -k 10 300 python -u tools/model_ab.py ktail 0 1 2>&1 | grep -v amdgpu.ids
