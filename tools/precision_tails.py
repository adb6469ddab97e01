"""Full-batch error tails of the engine's contraction variants vs the float64 C++ restatement,
with the plain IEEE float32 evaluation (oracle/cpu_forward.cpp without -ffast-math) and the
-ffast-math float32 one as yardsticks.  Usage (GPU box):
    python tools/precision_tails.py [routenet:synth50 qsize:synth50 routenet:geant2] [--graphs 512]
Prints one JSON line per workload: {variant: {max, p9999, mean}}."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ignnition_amd import workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402
from oracle import cpu_oracle  # noqa: E402

VARIANTS = {   # name: (IGN_SEQ_VARIANT, IGN_READOUT_VARIANT, IGN_SUM_VARIANT)
    "default": (None, None, None),
    "bf16x6": ("4", "2", "7"),
    "f32mfma": ("2", "1", "3"),
}


def tails(got, ref):
    e = np.abs(np.asarray(got, np.float64).reshape(-1) - ref) / np.maximum(1.0, np.abs(ref))
    return {"max": float(e.max()), "p9999": float(np.quantile(e, 0.9999)), "mean": float(e.mean()),
            "n_over_1e-4": int((e > 1e-4).sum())}


def run(model, topo, n, seed=1, variants=VARIANTS):
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs(model, topo, n)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(seed, bias_scale=0.05)
    t = time.time()
    ref = cpu_oracle.cpu_forward(plan, graphs, prm, 0, float64=True).astype(np.float64)
    res = {"workload": "%s_%s_x%d" % (model, topo, n), "predictions": int(ref.size),
           "t_ref_s": round(time.time() - t, 1)}
    res["ieee_f32"] = tails(cpu_oracle.cpu_forward(plan, graphs, prm, 0, ieee=True), ref)
    res["fastmath_f32"] = tails(cpu_oracle.cpu_forward(plan, graphs, prm, 0), ref)
    for name, (sq, ro, sm) in variants.items():
        for k, v in (("IGN_SEQ_VARIANT", sq), ("IGN_READOUT_VARIANT", ro), ("IGN_SUM_VARIANT", sm)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        eng = Engine(plan, 0)
        eng.set_params(prm)
        b = Batch(eng, graphs)
        out = b.forward().reshape(-1)
        b.close()
        eng.close()
        res[name] = tails(out, ref)
    for k in ("IGN_SEQ_VARIANT", "IGN_READOUT_VARIANT", "IGN_SUM_VARIANT"):
        os.environ.pop(k, None)
    return res


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["routenet:synth50", "qsize:synth50", "routenet:geant2"])
    ap.add_argument("--graphs", type=int, default=512)
    a = ap.parse_args()
    cpu_oracle.build()
    for w in a.workloads:
        m, t = w.split(":")
        print(json.dumps(run(m, t, a.graphs)), flush=True)
