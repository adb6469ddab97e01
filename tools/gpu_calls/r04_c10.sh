# round 4, call 10: the graph-resident forward (resident.hip) -- parity (bitwise vs the batched
# launches, oracle, batch invariance) and GEANT2 / NSFNET x512 ms/step against IGN_RESIDENT=0
set -o pipefail
O=gpurun_out/c10
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "resident_forward_batch_invariance" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for topo in geant2 nsfnet; do
  for s in 2 4; do
    for v in 1 0; do
      f=$O/$topo-s$s-r$v
      IGN_RESIDENT=$v timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut --topology $topo --streams $s > $f.json 2> $f.err || { tail -20 $f.err; exit 1; }
      python3 - $f.json "$topo s$s resident=$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], r["kernel"], "avg %.4f" % r["avg_launch_ms"],
      " ".join("%s %.4f" % (k, v["ms_total"] / max(1, v["launches"])) for k, v in r["warmup_kernels"].items()))
PY
    done
  done
done
