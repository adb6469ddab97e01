"""Summarise bench.py JSON lines: ms/step and average per-launch ms per kernel kind."""
import json
import sys

for path in sys.argv[1:]:
    try:
        line = [l for l in open(path) if l.startswith("{")][-1]
        d = json.loads(line)
    except Exception as exc:  # noqa: BLE001
        print(path, "no result:", exc)
        continue
    r = d.get("roofline") or {}
    k = r.get("warmup_kernels", r.get("kernels", {}))
    per = {a: round(b["ms_total"] / b["launches"], 4) for a, b in k.items()}
    print("%-28s %.3e edges/s %.3f ms/step" % (path.split("/")[-1], d["value"], d["ms_per_step"]), per,
          "| %s %s %.3f ms frac %.3f" % (r.get("kernel"), r.get("bound"), r.get("avg_launch_ms", 0), r.get("frac", 0)))
