cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p5/tests.txt 2>&1; rc=$?; tail -5 gpurun_out/p5/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latency > gpurun_out/p5/bench.json 2> gpurun_out/p5/bench.err; echo "bench rc=$?"; python -c "
import json;d=json.loads(open('gpurun_out/p5/bench.json').read().strip().splitlines()[-1]);print(d['value'],d.get('training'))"
