#!/bin/bash
# Instruction / wait counters of the main line of CFG (default deit_base), two passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; cfg=${CFG:-deit_base}; T=${TAG:-q}
mkdir -p $O
pmc() {  # pmc <dir> <counters...>
  local d=$1; shift
  rm -rf $O/$d
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $O/$d -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines main > $O/$d.log 2>&1
}
pmc ${T}pi1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES || exit $?
pmc ${T}pi2 SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU || exit $?
python tools/pmc_summary.py "$O/${T}pi[12]/**/*counter_collection.csv" > $O/${T}_pmc_$cfg.txt || exit $?
cat $O/${T}_pmc_$cfg.txt
