#!/bin/bash
# One round-end GPU session: parity suite, kernel-trace profile, HBM PMC passes,
# bench lines (with measured HBM traffic) for every config.  Every GPU step has
# its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r01}
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
rm -rf $O/prof $O/pmc_fetch $O/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity > $O/prof_bench.json 2> $O/prof.err || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o p --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o p --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/pmc_write.log 2>&1 || exit $?
python tools/hbm_traffic.py $O/pmc_fetch $O/pmc_write $O/traffic_deit_base.json || exit $?
for cfg in ${BENCH_CONFIGS:-deit_base dit_xl2 pixart_cross}; do
  extra=""; [ "$cfg" = deit_base ] && extra="--traffic-json $O/traffic_deit_base.json"
  timeout -k 10 600 python bench.py --config $cfg $extra > $O/bench_$cfg.json 2> $O/bench_$cfg.err
  brc=$?; echo "bench $cfg rc=$brc"; tail -1 $O/bench_$cfg.json; [ $brc -eq 0 ] || exit $brc
done
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
echo done
