#!/bin/bash
# Full GPU suite, then main-line bench under LIBS, then qkv / qkv+proj lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/pt3.log 2>&1
rc=$?; tail -4 gpurun_out/pt3.log; [ $rc -eq 0 ] || exit $rc
for lib in ${LIBS:-default}; do
  [ "$lib" = default ] && lib=""
  for c in deit_base dit_xl2; do
    MXA_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline --no-parity --config $c --lines main > gpurun_out/bm_$c.json 2> gpurun_out/bm_$c.err || { tail -5 gpurun_out/bm_$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bm_$c.json'));print('${lib##*/}','$c',round(d['value']/1e6,2),'Mtok/s',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()})"
  done
done
LINES=qkv,qkvproj CFGS="deit_base dit_xl2" bash tools/gpu_libs_qkv.sh
