"""Is the training forward's fused readout (readout_h16 with activation saves) independent of which
rows share a 16-row tile?  The edge-cut test's synthetic graph alone, and after an 8-node graph in
the same batch (its rows shifted by 8): training predictions with the fused readout and with the
per-layer path (IGN_TRAIN_FUSED_READOUT, set by the caller), and the inference forward (GPU box)."""
import copy
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ignnition_amd import synthetic, workloads  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402
from ignnition_amd.json_operations import Model_information  # noqa: E402


def run(eng, graphs, train):
    import torch
    from ignnition_amd.partition import _DeviceRows
    b = Batch(eng, graphs)
    s = None
    if train:
        b.enable_training()
        p = b.forward_train().reshape(-1).copy()
        n = sum(int(g["num_node"]) for g in graphs)
        s = torch.as_tensor(_DeviceRows(b.train_buffers("node")[0], n, 32), device="cuda").cpu().numpy().copy()
    else:
        p = b.forward().reshape(-1).copy()
    b.close()
    return p, s


def main():
    desc, dims, _, graphs, labels = workloads.make_synthetic_inputs(n_nodes=2000, hidden=32, iterations=2, window=96)
    small = synthetic.synthetic_graph_arrays(n_nodes=8, window=4, graph_id=7)
    small.pop("target")
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(21, bias_scale=0.1))
    for train in (True, False):
        alone, sa = run(eng, graphs, train)
        shifted, ss = run(eng, [small] + graphs, train)
        shifted = shifted[8:]
        if sa is not None:
            ds = np.nonzero((sa != ss[8:]).any(axis=1))[0]
            print("  final states: rows differing", len(ds), ds[:10].tolist(), "max |h| %.3g" % float(np.abs(sa).max()))
        d = np.nonzero(alone != shifted)[0]
        print("train" if train else "inference", "fused=%s" % os.environ.get("IGN_TRAIN_FUSED_READOUT", "1"),
              "rows differing after an 8-row shift:", len(d), d[:10].tolist(),
              "max abs diff %.3g" % (float(np.abs(alone - shifted).max())))


if __name__ == "__main__":
    main()
