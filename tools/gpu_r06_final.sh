#!/bin/bash
# Round-6 profiling session, in two parts (each within one gpurun call):
#   PART=a: smoke, the whole GPU suite (TAG_pytest_gpu.log), then tools/gpu_round.sh for
#           deit_base (rocprof, HBM traffic and instruction PMC, qkv / qkvproj profiles, bench line)
#   PART=b: tools/gpu_round.sh for dit_xl2 and pixart_cross; the dense branch's MFMA counters and
#           trace (deit_base, dit_xl2); the drop-in line's trace; the float32 top-k A/B
# Outputs under gpurun_out/ (TAG_*), copied to profiles/ by hand.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r06v1}
mkdir -p $O
if [ "${PART:-a}" = a ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
  echo "smoke: $(tail -1 $O/${T}_smoke.log)"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $O/${T}_pytest_gpu.log)"; [ $rc -eq 0 ] || exit $rc
  TAG=$T NOTEST=1 BENCH_CONFIGS="deit_base" bash tools/gpu_round.sh || exit $?
else
  TAG=$T NOTEST=1 BENCH_CONFIGS="dit_xl2 pixart_cross" bash tools/gpu_round.sh || exit $?
  for cfg in deit_base dit_xl2; do
    rm -rf $O/pdt_$cfg $O/pdm_$cfg
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pdt_$cfg -o run --output-format csv -- \
      python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-parity --lines dense > $O/pdt_$cfg.json 2> $O/pdt_$cfg.err || exit $?
    find $O/pdt_$cfg -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_dense_$cfg.csv \;
    timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS \
      -d $O/pdm_$cfg -o p --output-format csv -- python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines dense > $O/pdm_$cfg.log 2>&1 || exit $?
    python tools/pmc_summary.py "$O/pdm_$cfg/**/*counter_collection.csv" --json $O/${T}_pmc_dense_$cfg.json > $O/${T}_pmc_dense_$cfg.txt || exit $?
  done
  rm -rf $O/pdr
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pdr -o run --output-format csv -- \
    python bench.py --config deit_base --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines dropin > $O/${T}_bench_dropin_deit_base.json 2> $O/pdr.err || exit $?
  find $O/pdr -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_dropin_deit_base.csv \;
  timeout -k 10 300 python tools/ab_topk_fp32.py > $O/${T}_ab_topk_fp32.txt 2>&1 || { tail -5 $O/${T}_ab_topk_fp32.txt; exit 1; }
  cat $O/${T}_ab_topk_fp32.txt
fi
echo done
