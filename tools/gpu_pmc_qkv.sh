#!/bin/bash
# Counters of the fused qkv line of CFG (default deit_base): instruction / wait passes,
# an L2 hit / miss pass and the HBM fetch pass, each its own run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; cfg=${CFG:-deit_base}; T=${TAG:-q}; L=${LINES:-qkv}
mkdir -p $O
pmc() {  # pmc <dir> <counters...>
  local d=$1; shift
  rm -rf $O/$d
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $O/$d -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines $L > $O/$d.log 2>&1
}
pmc ${T}k1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY || exit $?
pmc ${T}k2 SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_ACTIVE_INST_ANY || exit $?
pmc ${T}k3 TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit $?
pmc ${T}k4 FETCH_SIZE || exit $?
python tools/pmc_summary.py "$O/${T}k[1234]/**/*counter_collection.csv" > $O/${T}_pmcq_$cfg.txt || exit $?
grep -A30 "qkv_proj_kernel" $O/${T}_pmcq_$cfg.txt | head -40
