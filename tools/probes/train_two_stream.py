"""Probe (GPU box): does the training step gain from two half-batches on two plans / streams?

(a) one engine, the 512 x synth50 RouteNet batch: forward_train, mse, backward, adam per step;
(b) two engines with 256 graphs each, each running the same step on its own stream, launched back to
    back before one wait (no gradient sum and no parameter sync: an upper bound on the gain).
python tools/probes/train_two_stream.py [steps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ignnition_amd import workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402


def setup(plan, prm, graphs, labels):
    e = Engine(plan, 0)
    e.set_params(prm)
    b = Batch(e, graphs)
    b.enable_training()
    y = torch.from_numpy(np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels])).cuda()
    d = torch.empty_like(y)
    g = torch.zeros(e.n_params, dtype=torch.float32, device="cuda")
    m, v = torch.zeros_like(g), torch.zeros_like(g)
    torch.cuda.synchronize()
    it = [0]

    def step():
        b.forward_train(to_host=False)
        e.mse_loss(b.predictions_ptr(), y, d, want_loss=False)
        b.backward(d, g)
        e.adam_step(g, m, v, it[0], 1e-3)
        it[0] += 1
    return e, step


def timed(steps_fns, engines, n):
    for f in steps_fns:
        f()
    for e in engines:
        e.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        for f in steps_fns:
            f()
    for e in engines:
        e.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "synth50", 512)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(0, bias_scale=0.05)
    e0, s0 = setup(plan, prm, graphs, labels)
    print("one batch           %.3f ms/step" % timed([s0], [e0], n), flush=True)
    e1, s1 = setup(plan, prm, graphs[:256], labels[:256])
    e2, s2 = setup(plan, prm, graphs[256:], labels[256:])
    print("two halves, 2 strm  %.3f ms/step" % timed([s1, s2], [e1, e2], n), flush=True)
    print("two halves, serial  %.3f ms/step" % timed([lambda: (s1(), e1.synchronize()), lambda: (s2(), e2.synchronize())],
                                                     [e1, e2], n), flush=True)


if __name__ == "__main__":
    main()
