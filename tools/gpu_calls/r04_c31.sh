# round 4, call 31: N=2 rehearsal of bench.py --gpus 2 on the one-GPU box (gloo, both ranks on GPU 0)
# with the final tree: the RouteNet leg on the resident forward and the edge-cut leg
set -o pipefail
IGN_DIST_BACKEND=gloo IGN_BENCH_DEVICE=0 timeout -k 10 600 python -u bench.py --gpus 2 --no-cpu --steps 10 --warmup 3 > gpurun_out/n2.json 2> gpurun_out/n2.err || { tail -20 gpurun_out/n2.err; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/n2.json') if l.startswith('{')][-1]); e=d.get('edge_cut_1m') or {}
print('n_gpus', d['n_gpus'], 'ms', round(d['ms_per_step'],4), 'value %.3e' % d['value'], 'edge_cut', e.get('n_ranks'), e.get('value'), e.get('edges_match_whole_graph'), e.get('ms_per_step'))"
