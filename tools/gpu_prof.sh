#!/bin/bash
# rocprofv3 kernel-trace summaries of the main bench line of every config in CFGS
# (default library or MXA_LIB), one profile per config under gpurun_out/prof_<tag>_<cfg>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-p}
for c in ${CFGS:-deit_base dit_xl2}; do
  rm -rf gpurun_out/prof_${T}_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_$c -o run --output-format csv -- \
    python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-parity --lines ${LINES:-main} > gpurun_out/prof_${T}_$c.json 2> gpurun_out/prof_${T}_$c.err || { tail -5 gpurun_out/prof_${T}_$c.err; exit 1; }
  f=$(find gpurun_out/prof_${T}_$c -name "*kernel_stats.csv" | head -1)
  echo "== $c"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(f\"{r['Name'][:90]:90s} n={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:9.1f}us tot%={float(r['Percentage']):5.1f}\")
"
done
