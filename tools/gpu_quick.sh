#!/bin/bash
# Quick GPU check: smoke, then the GPU suite (optional -k filter PYK), then bench lines
# (no CPU baseline) for CFGS under each library in LIBS (MXA_LIB paths; "default" = libmxa.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo smoke ok
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pt.log 2>&1
  rc=$?; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in ${LIBS:-default}; do
  [ "$lib" = default ] && lib=""
  for c in ${CFGS:-deit_base dit_xl2}; do
    MXA_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline --config $c --lines main > gpurun_out/bq_$c.json 2> gpurun_out/bq_$c.err || { tail -5 gpurun_out/bq_$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bq_$c.json'));print('${lib##*/}','$c',round(d['value']/1e6,2),'Mtok/s',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()},d['parity']['idx_bitmatch'])"
  done
done
echo done
