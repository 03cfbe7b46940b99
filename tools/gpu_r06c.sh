#!/bin/bash
# Round-6 A/B: the whole GPU suite on every library of LIBS (tags of
# mx_quantization_amd/libmxa_<tag>.so, "default" = libmxa.so), then the same-box main-line
# A/B of tools/ab_libs.sh (CFGS, REPS) and a kernel trace of each library's main lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in ${PTLIBS-${LIBS:-default}}; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  MXA_LIB=$L timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pt_$lib.log 2>&1
  rc=$?; echo "pytest $lib rc=$rc: $(tail -1 gpurun_out/pt_$lib.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/pt_$lib.log; exit $rc; }
done
bash tools/ab_libs.sh || exit $?
for lib in ${TRACE:-}; do
  L=""; [ $lib != default ] && L=mx_quantization_amd/libmxa_$lib.so
  for c in ${CFGS:-deit_base}; do
    rm -rf gpurun_out/tr_${lib}_$c
    MXA_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr_${lib}_$c -o run --output-format csv -- \
      python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-parity --lines main > gpurun_out/tr_${lib}_$c.log 2>&1 || exit $?
    echo "== trace $lib $c"; find gpurun_out/tr_${lib}_$c -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \; | head -8
  done
done
echo done
