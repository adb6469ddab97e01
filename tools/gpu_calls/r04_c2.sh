# round 4, call 2: parity tests after the sum-path changes; readout next-group input prefetch A/B
# (pf = default tree, nopf = without); segmented sum for every sum MP (IGN_SUM_WINDOW=2) against the
# auto rule on RouteNet synth50 / GEANT2, windowed against auto (segmented) on Q-size; GEANT2 streams
set -o pipefail
O=gpurun_out/c2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  > $O/test_parity.log 2>&1 || { tail -30 $O/test_parity.log; exit 1; }
tail -2 $O/test_parity.log
bash tools/ab_lib.sh "pf nopf" 3 --steps 20 > $O/ab_prefetch.log 2>&1 || { tail -20 $O/ab_prefetch.log; exit 1; }
cat $O/ab_prefetch.log
for spec in "rn|" "geant2|--topology geant2" "qsize|--model qsize"; do
  name=${spec%%|*}; args=${spec#*|}
  for w in -1 2 1; do
    [ $name != qsize ] && [ $w = 1 ] && continue
    IGN_SUM_WINDOW=$w timeout -k 10 200 python -u bench.py $args --no-cpu --no-edge-cut --steps 20 \
      > $O/${name}_w$w.json 2> $O/${name}_w$w.err || { tail -20 $O/${name}_w$w.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${name}_w$w.json').read().splitlines()[-1]); print('$name win $w', round(d['ms_per_step'],4), {k: round(v['ms_total']/max(1,v['launches']),4) for k,v in d['roofline']['warmup_kernels'].items()})"
  done
done
for s in 1 3 4; do
  timeout -k 10 200 python -u bench.py --topology geant2 --streams $s --no-cpu --no-edge-cut --steps 20 \
    > $O/geant2_s$s.json 2> $O/geant2_s$s.err || { tail -20 $O/geant2_s$s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/geant2_s$s.json').read().splitlines()[-1]); print('geant2 streams $s', round(d['ms_per_step'],4))"
done
