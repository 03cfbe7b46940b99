#!/bin/bash
# PMC passes over tools/probe_attn.py (one rocprofv3 invocation per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-deit_base}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_$CFG_$i
  timeout -k 10 300 rocprofv3 --pmc $grp -d gpurun_out/pmc_${CFG}_$i -o p --output-format csv -- \
      python tools/probe_attn.py $CFG ${PATHS:-rows,tiles} > gpurun_out/pmc_${CFG}_$i.log 2>&1 || exit $?
done
echo pmc done
