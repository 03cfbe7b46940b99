#!/bin/bash
# Round-5 check: smoke + GPU suite + bench lines (gpu_quick.sh), a same-box A/B against the
# HEAD library (libmxa_head.so when present), and a kernel trace of the drop-in line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out; T=${TAG:-r05v2}
mkdir -p $O
bash tools/gpu_quick.sh || exit $?
if [ -f mx_quantization_amd/libmxa_head.so ]; then LIBS="default head" bash tools/ab_once.sh || exit $?; fi
rm -rf $O/profd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/profd -o run --output-format csv -- \
  python bench.py --config deit_base --steps 10 --warmup 2 --no-cpu-baseline --no-parity --lines dropin \
  > $O/${T}_bench_dropin_deit_base.json 2> $O/profd.err || exit $?
find $O/profd -name "*kernel_stats.csv" -exec cp {} $O/${T}_rocprof_dropin_deit_base.csv \;
head -25 $O/${T}_rocprof_dropin_deit_base.csv | cut -c1-150
