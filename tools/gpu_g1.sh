cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke ok && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "qkv or proj or linear" > gpurun_out/pt.log 2>&1; rc=$?; tail -5 gpurun_out/pt.log; [ $rc -eq 0 ] && \
for c in deit_base dit_xl2; do timeout -k 10 240 python bench.py --no-cpu-baseline --no-parity --config $c --lines qkv,qkvproj --steps 10 > gpurun_out/bq_$c.json 2> gpurun_out/bq_$c.err || exit 1; python -c "
import json;d=json.load(open('gpurun_out/bq_$c.json'))
for s in d.get('secondary',[]): print(s['config'], round(s['value']/1e6,2), 'Mtok/s', round(s['ms_per_step'],3), {k:round(v,3) for k,v in s['stages_ms'].items()})"; done
