#!/bin/bash
# A/B on one box: the GPU suite on the default library (optional: NOTEST=1), then the main
# bench line of every config in CFGS for every library in LIBS (MXA_LIB paths; "default" =
# libmxa.so), then (PMC=1) the SQ counters of the first config's main line per library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pt.log 2>&1
  rc=$?; tail -4 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in ${LIBS:-default}; do
  tag=${lib##*/}; [ "$lib" = default ] && { lib=""; tag=default; }
  for c in ${CFGS:-deit_base dit_xl2}; do
    MXA_LIB=$lib timeout -k 10 240 python bench.py --no-cpu-baseline --config $c --lines main > gpurun_out/ab_${tag}_$c.json 2> gpurun_out/ab_${tag}_$c.err || { tail -5 gpurun_out/ab_${tag}_$c.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_$c.json'));print('$tag','$c',round(d['value']/1e6,2),'Mtok/s',round(d['ms_per_step'],3),'ms',{k:round(v,3) for k,v in d['stages_ms'].items()},d['parity']['idx_bitmatch'])"
  done
done
if [ -n "${PMC:-}" ]; then
  c=${CFGS%% *}; c=${c:-deit_base}
  for lib in ${LIBS:-default}; do
    tag=${lib##*/}; [ "$lib" = default ] && { lib=""; tag=default; }
    for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT"; do
      rm -rf gpurun_out/pmc_$tag
      MXA_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/pmc_$tag -o p --output-format csv -- \
        python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines main > gpurun_out/pmc_$tag.log 2>&1 || exit 1
    done
    python tools/pmc_summary.py "gpurun_out/pmc_$tag/**/*counter_collection.csv" > gpurun_out/pmc_${tag}_$c.txt
    grep -A10 "select" gpurun_out/pmc_${tag}_$c.txt | head -24
  done
fi
echo done
