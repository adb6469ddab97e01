# round 4, call 24: sub-batch stream count A/B (QARGS selects the workload: Q-size, then the headline)
set -o pipefail
QARGS=${QARGS:---model qsize}
mkdir -p gpurun_out/c24
for r in 1 2; do for s in 2 3 4; do
  timeout -k 10 200 python -u bench.py $QARGS --no-cpu --no-edge-cut --streams $s > gpurun_out/c24/q-$s-$r.json 2> gpurun_out/c24/q-$s-$r.err || { tail -5 gpurun_out/c24/q-$s-$r.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c24/q-$s-$r.json') if l.startswith('{')][-1]); print('streams $s', round(d['ms_per_step'],4))"
done; done
