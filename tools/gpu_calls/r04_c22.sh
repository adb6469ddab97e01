# round 4, call 22: one bench line per workload (tools/bench_sweep.sh) on the round's tree
set -o pipefail
bash tools/bench_sweep.sh && for f in gpurun_out/sweep/*.json; do python3 - $f <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d.get("roofline") or {}
e = d.get("edge_cut_1m") or {}
print(sys.argv[1].split("/")[-1], "ms/step %.4f" % d["ms_per_step"], "value %.3e" % d["value"], r.get("kernel"), r.get("frac"),
      "edge_cut_1m %.3e %.3f ms" % (e["value"], e["ms_per_step"]) if e else "")
PY
done
