#!/bin/bash
# A/B of an environment switch on the default bench (GPU box): ab_env.sh VAR "v1 v2" [reps] [bench args]
# prints the bench's per-kind warm-up kernel times and ms/step per run
VAR=$1; VALS=$2; REPS=${3:-2}; shift 3
mkdir -p gpurun_out/ab
for r in $(seq $REPS); do
  for v in $VALS; do
    f=gpurun_out/ab/$VAR-${v//\//_}-$r
    env $VAR=$v timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut "$@" > $f.json 2> $f.err || { echo "run $v failed"; exit 1; }
    python - "$VAR=$v" $f.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
wk = (d.get("roofline") or {}).get("warmup_kernels", {})
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], " ".join("%s %.4f" % (k, v["ms_total"] / max(1, v["launches"])) for k, v in wk.items()))
PY
  done
done
