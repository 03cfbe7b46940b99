#!/bin/bash
# Quick PMC look at one bench line (iteration tool; tools/gpu_round.sh makes the
# committed profiles): CFG (deit_base), LINES (qkv), TAG (x).  Two instruction/wait
# passes and the two HBM passes, each its own rocprofv3 run with its own time limit.
# Outputs gpurun_out/<TAG>_pmc.txt, <TAG>_traffic.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-x}
cfg=${CFG:-deit_base}
l=${LINES:-qkv}
mkdir -p $O
pmc() {  # pmc <dir> <counters...>
  local d=$1; shift
  rm -rf $O/$d
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $O/$d -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines $l > $O/$d.log 2>&1
}
pmc ${T}_p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_WAVE_CYCLES SQ_WAIT_ANY || exit $?
pmc ${T}_p2 SQ_WAVES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES || exit $?
python tools/pmc_summary.py "$O/${T}_p[12]/**/*counter_collection.csv" > $O/${T}_pmc.txt || exit $?
if [ -z "${NOHBM:-}" ]; then
  pmc ${T}_pf FETCH_SIZE || exit $?
  pmc ${T}_pw WRITE_SIZE || exit $?
  python tools/hbm_traffic.py $O/${T}_pf $O/${T}_pw $O/${T}_traffic.json || exit $?
fi
echo done
