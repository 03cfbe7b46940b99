#!/bin/bash
# Instruction / stall PMC passes over bench.py (one rocprofv3 run per counter group,
# at most 8 SQ counters each); summary per kernel: tools/pmc_summary.py.
#   tools/pmc_bench.sh <config> [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${1:-deit_base}
TAG=${2:-x}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU"; do
  i=$((i+1))
  rm -rf gpurun_out/pmc_${TAG}_${CFG}_$i
  timeout -k 10 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_${TAG}_${CFG}_$i -o p --output-format csv -- \
      python bench.py --config $CFG --steps 2 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/pmc_${TAG}_${CFG}_$i.log 2>&1 || exit $?
done
python tools/pmc_summary.py "gpurun_out/pmc_${TAG}_${CFG}_*/**/*counter_collection.csv" > gpurun_out/pmc_${TAG}_${CFG}.txt || exit $?
echo pmc done
