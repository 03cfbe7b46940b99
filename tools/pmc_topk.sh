#!/bin/bash
# Instruction counters of the standalone top-k (one rocprofv3 pass per group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-deit_base}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  rm -rf gpurun_out/pmct_${CFG}_$i
  timeout -k 10 120 rocprofv3 --pmc $grp -d gpurun_out/pmct_${CFG}_$i -o p --output-format csv -- \
      python tools/probe_topk_only.py $CFG > gpurun_out/pmct_${CFG}_$i.log 2>&1 || exit $?
done
echo pmc done
