#!/bin/bash
# One GPU session: parity tests; then, only if they ran without a fault, one bench
# line per config and a rocprofv3 kernel-trace summary of the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for cfg in ${BENCH_CONFIGS:-deit_base}; do
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  brc=$?
  echo "bench $cfg rc=$brc"; cat gpurun_out/bench_$cfg.json; tail -3 gpurun_out/bench_$cfg.err
  [ $brc -eq 0 ] || exit $brc
done
if [ -n "${PROFILE:-}" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity ${PROFILE_ARGS:-} > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  prc=$?
  echo "rocprof rc=$prc"; find gpurun_out/prof -name "*stats*" | head
  for f in $(find gpurun_out/prof -name "*kernel_stats.csv"); do cut -c1-220 $f | head -12; done
fi
