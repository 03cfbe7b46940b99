#!/bin/bash
# Instruction counts of the fused row kernel with phases switched off
# (instrumented build libmxa_prof.so; MXA_DBG_SKIP bits as in tools/skip_prof.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-deit_base}
for sk in ${SKIPS:-0 1 16 4 8 2}; do
  rm -rf gpurun_out/pmcs_${CFG}_$sk
  MXA_LIB=$PWD/mx_quantization_amd/libmxa_prof.so MXA_DBG_SKIP=$sk timeout -k 10 300 \
    rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/pmcs_${CFG}_$sk -o p \
    --output-format csv -- python tools/probe_once.py $CFG > gpurun_out/pmcs_${CFG}_$sk.log 2>&1 || exit $?
done
echo pmc skips done
