#!/bin/bash
# Bench lines (no CPU baseline) for each config under each library variant in LIBS
# (MXA_LIB paths; "default" = the product libmxa.so).  Summary to stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${LIBS:-default}; do
  [ "$lib" = default ] && lib=""
  for c in ${CFGS:-deit_base dit_xl2 pixart_cross}; do
    MXA_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -3 gpurun_out/bc.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bc.json'));print('${lib##*/}','$c',round(d['value']/1e6,2),'Mtok/s',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()},d['parity']['idx_bitmatch']);[print('${lib##*/}',x['config'],round(x['value']/1e6,2),'Mtok/s',round(x['ms_per_step'],3),'ms',{k:round(v,3) for k,v in x['stages_ms'].items()}) for x in d.get('secondary',[]) if 'qkv' in x['config']]"
  done
done
