#!/bin/bash
# Same-box A/B of the finishing kernel at small k: libmxa.so (finish16_kernel for k <= 64) against
# libmxa_fqk1.so (build_native -DMXA_FQ_KMIN=1: finish_qk_kernel, every key's QK^T on MFMA, at
# every k with T <= 256), DeiT-base k = 20 and 30, PixArt cross k = 20; two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for lib in default fqk1; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  for ck in deit_base:20 deit_base:30 pixart_cross:20; do
    c=${ck%%:*}; k=${ck##*:}
    MXA_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --config $c --k $k --lines main > gpurun_out/abf_${lib}_${c}_$k.json 2> gpurun_out/abf_${lib}_${c}_$k.err || { tail -5 gpurun_out/abf_${lib}_${c}_$k.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abf_${lib}_${c}_$k.json'));print('$rep','$lib','$c','k=$k',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()},d['roofline']['mfma']['engine']['kernel'],d['parity']['idx_bitmatch'],round(d['parity']['out_normwise_rel_err_max'],6))"
  done
done
done
