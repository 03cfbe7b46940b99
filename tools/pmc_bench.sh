#!/bin/bash
# Instruction / stall / MFMA PMC passes over bench.py (one rocprofv3 run per counter
# group, at most 8 SQ counters each); summary per kernel: tools/pmc_summary.py.
#   tools/pmc_bench.sh <config> [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-deit_base}
TAG=${2:-x}
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
# MFMA group: only the counters this box lists
MF=""
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_MFMA SQ_BUSY_CU_CYCLES; do
  grep -qw "$c" gpurun_out/pmc_avail.txt && MF="$MF $c"
done
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU" \
           "SQ_WAVES$MF GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${TAG}_${CFG}_$i
  timeout -k 10 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_${CFG}_$i -o p --output-format csv -- \
      python bench.py --config $CFG --steps 2 --warmup 1 --no-parity --no-cpu-baseline --no-secondary > gpurun_out/pmc_${TAG}_${CFG}_$i.log 2>&1 || exit $?
done
python tools/pmc_summary.py "gpurun_out/pmc_${TAG}_${CFG}_*/**/*counter_collection.csv" > gpurun_out/pmc_${TAG}_${CFG}.txt || exit $?
echo pmc done
