cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-latency --no-train --steps 2 --warmup 1 > gpurun_out/pmc/fetch.log 2>&1; echo "fetch rc=$?"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-latency --no-train --steps 2 --warmup 1 > gpurun_out/pmc/write.log 2>&1; echo "write rc=$?"
python3 tools/pmc_traffic.py gpurun_out/pmc/fetch gpurun_out/pmc/write gpurun_out/pmc/pmc_traffic.json
