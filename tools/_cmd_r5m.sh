cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5m
for tag in prev cur; do
  if [ $tag = prev ]; then export HV_LIB_PATH=abl/libhvs_prev.so; else unset HV_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5m/$tag -o run --output-format csv -- python tools/prep_time.py > gpurun_out/r5m/$tag.log 2>&1 || exit 1
  f=$(find gpurun_out/r5m/$tag -name 'run_kernel_stats.csv' | head -1)
  echo "== $tag"; python tools/prof_summary.py $(dirname $f) 30 12
done
