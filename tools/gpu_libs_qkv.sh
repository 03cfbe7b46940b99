#!/bin/bash
# qkv / qkvproj bench lines of CFGS under each library of LIBS (MXA_LIB; "default" = libmxa.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-default}; do
  [ "$lib" = default ] && lib=""
  for c in ${CFGS:-deit_base}; do
    MXA_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline --no-parity --config $c --lines ${LINES:-qkv} --steps 10 > gpurun_out/bl_$c.json 2> gpurun_out/bl_$c.err || { tail -5 gpurun_out/bl_$c.err; exit 1; }
    python -c "
import json;d=json.load(open('gpurun_out/bl_$c.json'))
for s in d.get('secondary',[]): print('${lib##*/}', s['config'], round(s['value']/1e6,2), 'Mtok/s', round(s['ms_per_step'],3), {k:round(v,3) for k,v in s['stages_ms'].items()})"
  done
done
echo done
