#!/bin/bash
# Same-box A/B of the DeiT-base main line (with its parity check) under libmxa.so and LIBS variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do for lib in default ${LIBS:-}; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  MXA_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --config deit_base --lines main > gpurun_out/abt_$lib.json 2> gpurun_out/abt_$lib.err || { tail -5 gpurun_out/abt_$lib.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abt_$lib.json'));print('$lib',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['stages_ms'].items()},d['parity']['idx_bitmatch'])"
done; done
