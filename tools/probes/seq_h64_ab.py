"""Probe (GPU box): ordered-update variants at H = 64 (no bench config has a 64-wide ordered MP):
RouteNet with hidden 64 on 256 synth50 graphs, forward time per variant (median of reps), split-fp16
(6) vs split-bf16 (4).  python tools/probes/seq_h64_ab.py [reps]"""
import copy
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from ignnition_amd import model_examples, synthetic, workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402
from ignnition_amd.json_operations import Model_information  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    desc = model_examples.routenet(hidden=64, iterations=8)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("synth50", g) for g in range(256)])
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(0)
    for rnd in range(2):
        for v in ("4", "6"):
            os.environ["IGN_SEQ_VARIANT"] = v
            eng = Engine(plan, 0)
            eng.set_params(prm)
            b = Batch(eng, graphs)
            b.forward(to_host=False)
            b.forward()
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                b.forward()
                ts.append(time.perf_counter() - t)
            print("H=64 seq variant %s: %.3f ms per forward (median of %d)" % (v, 1e3 * float(np.median(ts)), reps),
                  flush=True)
            b.close()
            eng.close()


if __name__ == "__main__":
    main()
