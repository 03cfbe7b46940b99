#!/bin/bash
# Same-box A/B of library variants (LIBS: tags of mx_quantization_amd/libmxa_<tag>.so,
# "default" = libmxa.so) on the main line of each config in CFGS; REPS rounds; stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
for lib in ${LIBS:-default}; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  for c in ${CFGS:-deit_base}; do
    MXA_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --config $c --lines ${LINES:-main} ${BARGS:-} > gpurun_out/abl_${lib}_$c.json 2> gpurun_out/abl_${lib}_$c.err || { tail -5 gpurun_out/abl_${lib}_$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abl_${lib}_$c.json'));print('$rep','$lib','$c',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()})"
  done
done
done
