# headline with the resident forward: 1 / 2 / 3 / 4 sub-batch streams, same box, two passes
set -o pipefail
mkdir -p gpurun_out/c51
for rep in 1 2; do
  for s in 1 2 3 4; do
    timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut --streams $s > gpurun_out/c51/routenet_s${s}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c51/routenet_s${s}_$rep.json') if l.startswith('{')][-1]); print('streams $s', d['ms_per_step'])"
  done
done
