#!/bin/bash
# GPU parity suite (optional -k filter in PYK) then one bench line per config in CFGS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pt.log 2>&1
  rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
for c in ${CFGS:-deit_base dit_xl2 pixart_cross}; do
  timeout -k 10 300 python bench.py --config $c ${BARGS:---no-cpu-baseline} > gpurun_out/b_$c.json 2> gpurun_out/b_$c.err || exit 1
done
echo ok
