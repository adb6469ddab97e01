# round 4, call 9: what the timed region's HIP event pairs cost (direct launches with events around
# the dominant kernel) against untimed hipGraph replay of each sub-batch
set -o pipefail
O=gpurun_out/c9
mkdir -p $O
for r in 1 2 3; do
  for mode in timed untimed; do
    extra=""; [ $mode = untimed ] && extra="--no-timing"
    timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut --steps 40 $extra > $O/$mode-$r.json 2> $O/$mode-$r.err || { tail -20 $O/$mode-$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$mode-$r.json').read().splitlines()[-1]); print('$mode', round(d['ms_per_step'],4))"
  done
done
