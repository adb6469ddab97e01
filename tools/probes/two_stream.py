"""Probe: 512 synth50 graphs as one batch vs two 256-graph batches on two plans/streams
(concurrent hipGraph replays), to see whether the HBM-bound sum update of one half overlaps the
issue-bound ordered update of the other.  Prints ms per 512-graph forward for each layout."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np
import torch

from ignnition_amd import workloads
from ignnition_amd.engine import Batch, Engine, MPPlan

G = 512
desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "synth50", G)
plan = MPPlan.from_model_info(mi)
prm = plan.init_params(seed=0, bias_scale=0.05)


def timeit(fn, sync, n=20):
    for _ in range(3):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    sync()
    return (time.perf_counter() - t) / n * 1e3


res = {}
e1 = Engine(plan, 0)
e1.set_params(prm)
s1 = torch.cuda.Stream()
e1.set_stream(s1.cuda_stream)
full = Batch(e1, graphs)
res["one_512"] = timeit(lambda: full.forward(to_host=False), torch.cuda.synchronize)
outs_full = full.forward(to_host=True).reshape(-1)
for parts in (2, 4):
    engs, bats = [], []
    step = G // parts
    for p in range(parts):
        e = Engine(plan, 0)
        e.set_params(prm)
        s = torch.cuda.Stream()
        e.set_stream(s.cuda_stream)
        engs.append((e, s))
        bats.append(Batch(e, graphs[p * step:(p + 1) * step]))

    def fwd():
        for b in bats:
            b.forward(to_host=False)
    res["%dx%d_streams" % (parts, step)] = timeit(fwd, torch.cuda.synchronize)
    got = np.concatenate([b.forward(to_host=True).reshape(-1) for b in bats])
    res["%dx%d_maxdiff" % (parts, step)] = float(np.abs(got - outs_full).max())
    # same split, one stream (serial): isolates the overlap from the size effect
    for e, s in engs:
        e.set_stream(s1.cuda_stream)
    res["%dx%d_serial" % (parts, step)] = timeit(fwd, torch.cuda.synchronize)
print(res)
