# round 4, call 32: final checks -- the GPU suite, smoke, and the default bench line
set -o pipefail
O=gpurun_out/c32
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/bench_default.json') if l.startswith('{')][-1]); r=d['roofline']
print('default', round(d['ms_per_step'],4), '%.3e' % d['value'], r['kernel'], r['frac'], r.get('mfma_pipe'), r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'), (d.get('edge_cut_1m') or {}).get('ms_per_step'))"
