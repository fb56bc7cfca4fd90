cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r14
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r14/tests.txt 2>&1; rc=$?; tail -2 gpurun_out/r14/tests.txt; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r14/bench.json 2> gpurun_out/r14/bench.err; echo "bench rc=$?"; python -c "
import json;d=json.loads(open('gpurun_out/r14/bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline'],d['latency']['frozen'],d['training']['value'],d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r14/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-latency --no-train --steps 20 > gpurun_out/r14/prof.log 2>&1; echo "prof rc=$?"
f=$(find gpurun_out/r14/prof -name 'run_kernel_stats.csv' | head -1); d=$(dirname $f); python3 tools/prof_summary.py $d 29 40 > gpurun_out/r14/prof_summary.txt; head -16 gpurun_out/r14/prof_summary.txt
