#!/bin/bash
# Round-6 check 2: smoke, the whole GPU suite, then the config's lines LINES (default main,
# qkv, qkvproj) and a kernel trace of the qkvproj line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pt.log 2>&1
rc=$?; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-deit_base}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --lines ${LINES:-main,qkv,qkvproj} > gpurun_out/bb_$c.json 2> gpurun_out/bb_$c.err || { tail -5 gpurun_out/bb_$c.err; exit 1; }
  python tools/show_bench.py gpurun_out/bb_$c.json
  rm -rf gpurun_out/tq_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tq_$c -o run --output-format csv -- \
    python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline --no-parity --lines qkvproj > gpurun_out/tq_$c.log 2>&1 || exit $?
  find gpurun_out/tq_$c -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \;
done
echo done
