# round 4, call 2: readout next-group input prefetch A/B (pf = default tree, nopf = without);
# GEANT2 sub-batch stream count
set -o pipefail
O=gpurun_out/c2
mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_lib.sh "pf nopf" 3 --steps 20 > $O/ab_prefetch.log 2>&1 || { tail -20 $O/ab_prefetch.log; exit 1; }
cat $O/ab_prefetch.log
for s in 1 2 3 4; do
  timeout -k 10 200 python -u bench.py --topology geant2 --streams $s --no-cpu --no-edge-cut --steps 20 \
    > $O/geant2_s$s.json 2> $O/geant2_s$s.err || { tail -20 $O/geant2_s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/geant2_s$s.json').read().splitlines()[-1]); print('geant2 streams $s', round(d['ms_per_step'],4))"
done
