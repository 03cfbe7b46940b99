#!/bin/bash
# One GPU profiling session: parity suite; then per bench config a kernel-trace
# profile, the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs), the
# instruction-counter passes, and the bench line reading them.  Every PMC pass runs
# the config's main line ALONE (--lines main: no DiT or qkv secondary, so each stage
# has one kernel instantiation), plus a separate pass for the fused qkv line.
# Outputs: gpurun_out/<TAG>_{rocprof,traffic,pmc,bench}_<cfg>.*; copy to profiles/.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r04v3}
mkdir -p $O
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/${T}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
pmc() {  # pmc <dir> <lines> <counters...>
  local d=$1 l=$2; shift 2
  rm -rf $O/$d
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" -d $O/$d -o p --output-format csv -- \
    python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-parity --lines $l > $O/$d.log 2>&1
}
for cfg in ${BENCH_CONFIGS:-deit_base dit_xl2 pixart_cross}; do
  rm -rf $O/prof_$cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$cfg -o run --output-format csv -- \
    python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-parity --lines main \
    > $O/prof_bench_$cfg.json 2> $O/prof_$cfg.err || exit $?
  find $O/prof_$cfg -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_$cfg.csv \;
  pmc pf_$cfg main FETCH_SIZE || exit $?
  pmc pw_$cfg main WRITE_SIZE || exit $?
  python tools/hbm_traffic.py $O/pf_$cfg $O/pw_$cfg $O/${T}_traffic_$cfg.json || exit $?
  pmc pi1_$cfg main SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES || exit $?
  pmc pi2_$cfg main SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU || exit $?
  pmc pi3_$cfg main SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_MFMA GRBM_GUI_ACTIVE || exit $?
  python tools/pmc_summary.py "$O/pi[123]_$cfg/**/*counter_collection.csv" --json $O/${T}_pmc_$cfg.json > $O/${T}_pmc_$cfg.txt || exit $?
  if [ "$cfg" != pixart_cross ] && [ -z "${NOQKV:-}" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profq_$cfg -o run --output-format csv -- \
      python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-parity --lines qkv \
      > $O/profq_bench_$cfg.json 2> $O/profq_$cfg.err || exit $?
    find $O/profq_$cfg -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_qkv_$cfg.csv \;
    pmc pqf_$cfg qkv FETCH_SIZE || exit $?
    pmc pqw_$cfg qkv WRITE_SIZE || exit $?
    python tools/hbm_traffic.py $O/pqf_$cfg $O/pqw_$cfg $O/${T}_traffic_qkv_$cfg.json || exit $?
    pmc pq1_$cfg qkv SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_WAVE_CYCLES SQ_WAIT_ANY || exit $?
    python tools/pmc_summary.py "$O/pq1_$cfg/**/*counter_collection.csv" --json $O/${T}_pmc_qkv_$cfg.json > $O/${T}_pmc_qkv_$cfg.txt || exit $?
    # x -> qkv Linear -> attention -> proj Linear (the GEMM kernel's own passes)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profp_$cfg -o run --output-format csv -- \
      python bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-parity --lines qkvproj \
      > $O/profp_bench_$cfg.json 2> $O/profp_$cfg.err || exit $?
    find $O/profp_$cfg -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_qkvproj_$cfg.csv \;
    pmc ppf_$cfg qkvproj FETCH_SIZE || exit $?
    pmc ppw_$cfg qkvproj WRITE_SIZE || exit $?
    python tools/hbm_traffic.py $O/ppf_$cfg $O/ppw_$cfg $O/${T}_traffic_qkvproj_$cfg.json || exit $?
    pmc pp1_$cfg qkvproj SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_WAVE_CYCLES SQ_WAIT_ANY || exit $?
    python tools/pmc_summary.py "$O/pp1_$cfg/**/*counter_collection.csv" --json $O/${T}_pmc_qkvproj_$cfg.json > $O/${T}_pmc_qkvproj_$cfg.txt || exit $?
  fi
  timeout -k 10 300 python bench.py --config $cfg --traffic-json $O/${T}_traffic_$cfg.json --pmc-json $O/${T}_pmc_$cfg.json \
    > $O/${T}_bench_$cfg.json 2> $O/${T}_bench_$cfg.err
  brc=$?; echo "bench $cfg rc=$brc"; tail -c 600 $O/${T}_bench_$cfg.json; [ $brc -eq 0 ] || exit $brc
done
echo done
