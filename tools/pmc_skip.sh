#!/bin/bash
# SALU / VALU / LDS instruction counts of the selection kernel with phases skipped
# (instrumented build libmxa_prof.so, MXA_DBG_SKIP bits: 1 top-k, 4 scores).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-deit_base}
for sk in ${SKIPS:-0 1 5}; do
  rm -rf gpurun_out/pmcs_${CFG}_$sk
  MXA_LIB=mx_quantization_amd/libmxa_prof.so MXA_DBG_SKIP=$sk timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES \
    -d gpurun_out/pmcs_${CFG}_$sk -o p --output-format csv -- python tools/probe_once.py $CFG > gpurun_out/pmcs_${CFG}_$sk.log 2>&1 || exit $?
  echo "== skip $sk"; python tools/pmc_summary.py "gpurun_out/pmcs_${CFG}_$sk/*counter_collection.csv" | grep -A7 "true, false, 1\|true, true, 1" | grep -E "SALU|VALU|waves"
done
