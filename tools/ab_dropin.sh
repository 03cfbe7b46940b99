cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out
for rep in 1 2; do for lib in default gs; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  MXA_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity --config deit_base --lines dropin > gpurun_out/abd_$lib.json 2> gpurun_out/abd_$lib.err || { tail -5 gpurun_out/abd_$lib.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/abd_$lib.json'));print('$lib',[(x['config'],round(x['ms_per_step'],3),x.get('idx_equal_fused')) for x in d['secondary']])"
done; done
