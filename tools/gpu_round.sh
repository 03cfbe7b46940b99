#!/bin/bash
# One round-end GPU session: parity suite; then per bench config a kernel-trace
# profile, the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) and the
# bench line carrying the measured traffic.  Every GPU step has its own time limit;
# the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in ${BENCH_CONFIGS:-deit_base dit_xl2 pixart_cross}; do
  rm -rf $O/prof_$cfg $O/pmc_fetch_$cfg $O/pmc_write_$cfg
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- \
    python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity > $O/prof_bench_$cfg.json 2> $O/prof_$cfg.err || exit $?
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$cfg -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_fetch_$cfg.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$cfg -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_write_$cfg.log 2>&1 || exit $?
  python tools/hbm_traffic.py $O/pmc_fetch_$cfg $O/pmc_write_$cfg $O/traffic_$cfg.json > /dev/null || exit $?
  find $O/prof_$cfg -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$cfg.csv \;
  timeout -k 10 600 python bench.py --config $cfg --traffic-json $O/traffic_$cfg.json > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  brc=$?; echo "bench $cfg rc=$brc"; tail -1 $O/bench_$cfg.json; [ $brc -eq 0 ] || exit $brc
done
echo done
