cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p3
timeout -k 10 300 python -u tools/gemm256_check.py > gpurun_out/p3/g256.txt 2>&1; echo "rc=$?"; cat gpurun_out/p3/g256.txt | grep -v amdgpu.ids
