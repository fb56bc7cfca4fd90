cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t7
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t7/tests.log 2>&1
echo "gpu tests rc=$?"
grep -E "FAIL|passed|failed|Error" gpurun_out/t7/tests.log | tail -15
timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 tools/ddp_gpu_check.py > gpurun_out/t7/ddp.log 2>&1; echo "ddp rc=$?"; grep "rank [01]:" gpurun_out/t7/ddp.log | tail -2
timeout -k 10 600 python -u bench.py > gpurun_out/t7/bench.json 2> gpurun_out/t7/bench.err; echo "bench rc=$?"; cat gpurun_out/t7/bench.json; tail -3 gpurun_out/t7/bench.err
