cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dr/tests.txt 2>&1; rc=$?; tail -2 gpurun_out/dr/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/tile_ab.py deep 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-train > gpurun_out/dr/bench.json 2> gpurun_out/dr/bench.err; echo "bench rc=$?"; python -c "
import json;d=json.loads(open('gpurun_out/dr/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['achieved'],d['roofline']['frac'],d['latency']['frozen'])"
timeout -k 10 200 python -u tools/train_diag.py time 16 640 2>&1 | grep -v amdgpu.ids
