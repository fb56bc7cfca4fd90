cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vz
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/vz/tests.txt 2>&1; rc=$?; tail -2 gpurun_out/vz/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train > gpurun_out/vz/bench.json 2> gpurun_out/vz/bench.err; echo "bench rc=$?"; python -c "
import json;d=json.loads(open('gpurun_out/vz/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac'],d['latency']['frozen'])"
timeout -k 10 300 python -u tools/gemm_breakdown.py 16 640 bf16 > gpurun_out/vz/gb.txt 2>&1; grep -v amdgpu.ids gpurun_out/vz/gb.txt | sed -n 1,12p
