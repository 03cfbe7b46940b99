#!/bin/bash
# Round-6 check: smoke, the selection / dense / dtype GPU tests, then the DeiT-base and
# DiT-XL/2 main lines plus the dense secondaries (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "${PYK:-dense or packed_pass_fallback or special_rows or full_size or pixart_cross_full}" > gpurun_out/pt.log 2>&1
rc=$?; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-deit_base dit_xl2}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config $c --lines main,dense > gpurun_out/bd_$c.json 2> gpurun_out/bd_$c.err || { tail -5 gpurun_out/bd_$c.err; exit 1; }
  python tools/show_bench.py gpurun_out/bd_$c.json
done
echo done
