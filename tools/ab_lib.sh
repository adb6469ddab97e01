#!/bin/bash
# A/B of library builds on the default bench (GPU box): ab_lib.sh "name1 name2 ..." [reps] [bench args]
# each name is ignnition_amd/ab/lib_<name>.so (IGN_LIB_PATH); prints ms/step and per-kind launch times
NAMES=$1; REPS=${2:-2}; shift 2
mkdir -p gpurun_out/ab
for r in $(seq $REPS); do
  for n in $NAMES; do
    f=gpurun_out/ab/lib-$n-$r
    IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python -u bench.py --no-cpu --no-edge-cut "$@" > $f.json 2> $f.err || { echo "run $n failed"; tail -5 $f.err; exit 1; }
    python - "$n" $f.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
wk = (d.get("roofline") or {}).get("warmup_kernels", {})
print("%-10s" % sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "dom %.4f" % (d.get("roofline") or {}).get("avg_launch_ms", 0),
      " ".join("%s %.4f" % (k, v["ms_total"] / max(1, v["launches"])) for k, v in wk.items()), flush=True)
PY
  done
done
