#!/bin/bash
# 8-stage 64x64 ring for small grids: kernel tests, small-GEMM probe, B=1 latency and B=16 A/B
# against the HEAD build (abl/libhvs_head.so).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-d8}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "pingpong or gemm or conv" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python tools/small_gemm_probe.py > $OUT/sg_probe.txt 2>&1 || { tail -20 $OUT/sg_probe.txt; exit 1; }
cat $OUT/sg_probe.txt
for i in 1 2; do
  HV_LIB_PATH=$GRAFT_REPO_ROOT/abl/libhvs_head.so timeout -k 10 120 python tools/quick_bench.py head >> $OUT/ab.txt 2>&1 || exit 1
  timeout -k 10 120 python tools/quick_bench.py new >> $OUT/ab.txt 2>&1 || exit 1
  HV_LIB_PATH=$GRAFT_REPO_ROOT/abl/libhvs_head.so timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline --no-train --no-stream --no-large --steps 5 > $OUT/lat_head_$i.json 2>> $OUT/lat.err || exit 1
  timeout -k 10 200 python -u bench.py --no-pmc --no-cpu-baseline --no-train --no-stream --no-large --steps 5 > $OUT/lat_new_$i.json 2>> $OUT/lat.err || exit 1
  python -c "import json,sys; [print(f, json.load(open(f))['latency']) for f in sys.argv[1:]]" $OUT/lat_head_$i.json $OUT/lat_new_$i.json
done
grep -v amdgpu.ids $OUT/ab.txt
