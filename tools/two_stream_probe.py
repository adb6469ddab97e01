"""Probe (GPU box): does the GPU overlap two independent halves of the headline batch?

Runs the 512 x synth50 RouteNet forward (a) as one batch on one engine and (b) as two batches of
256 graphs on two engines (two non-blocking streams), both launched before one synchronisation.
If the compute-bound ordered update of one half co-runs with the memory-bound sum update of the
other, (b) beats (a).  python tools/two_stream_probe.py [reps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from ignnition_amd import workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "synth50", 512)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(0)
    e0 = Engine(plan, 0)
    e0.set_params(prm)
    whole = Batch(e0, graphs)

    def one():
        whole.forward(to_host=False)
        e0.synchronize()

    engines, halves = [], []
    for k in range(2):
        e = Engine(plan, 0)
        e.set_params(prm)
        engines.append(e)
        halves.append(Batch(e, graphs[256 * k:256 * (k + 1)]))

    def two():
        for b in halves:
            b.forward(to_host=False)
        for e in engines:
            e.synchronize()

    def two_serial():
        for e, b in zip(engines, halves):
            b.forward(to_host=False)
            e.synchronize()

    for name, fn in (("one batch", one), ("two halves, two streams", two), ("two halves, serial", two_serial)):
        print("%-28s %.3f ms" % (name, timed(fn, reps)), flush=True)


if __name__ == "__main__":
    main()
