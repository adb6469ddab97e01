"""Bitwise A/B of two library builds (GPU box): the default RouteNet synth50 batch (or --model /
--topology / --graphs) through each ignnition_amd/ab/lib_<name>.so in its own process
(IGN_LIB_PATH), predictions compared bit for bit.  --train compares the parameter gradients of one backward instead (dpred = a
fixed seeded vector).
    python tools/ab_bitwise.py base new [--graphs 512] [--model routenet] [--topology synth50] [--train]"""
import argparse
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, numpy as np
sys.path.insert(0, %r)
from ignnition_amd import workloads
from ignnition_amd.engine import Batch, Engine, MPPlan
desc, dims, mi, graphs, _ = workloads.make_batch_inputs(%r, %r, %d)
plan = MPPlan.from_model_info(mi)
prm = plan.init_params(1, bias_scale=0.05)
eng = Engine(plan, 0); eng.set_params(prm)
b = Batch(eng, graphs)
if not %r:
    np.save(%r, b.forward().reshape(-1))
else:
    import torch
    b.enable_training()
    pred = b.forward_train(to_host=False)
    n = b.predictions * b.output_units
    dpred = torch.from_numpy(np.random.default_rng(3).standard_normal(n).astype(np.float32)).cuda()
    grads = torch.zeros(eng.n_params, dtype=torch.float32, device="cuda")
    b.backward(dpred, grads)
    torch.cuda.synchronize()
    np.save(%r, grads.cpu().numpy())
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--graphs", type=int, default=512)
    ap.add_argument("--model", default="routenet")
    ap.add_argument("--topology", default="synth50")
    ap.add_argument("--train", action="store_true")
    a = ap.parse_args()
    outs = {}
    os.makedirs(os.path.join(REPO, "gpurun_out", "ab"), exist_ok=True)
    for name in a.libs:
        f = os.path.join(REPO, "gpurun_out", "ab", "pred_%s.npy" % name)
        env = dict(os.environ, IGN_AB_LIB="1", IGN_LIB_PATH=os.path.join(REPO, "ignnition_amd", "ab", "lib_%s.so" % name))
        subprocess.run([sys.executable, "-c", CHILD % (REPO, a.model, a.topology, a.graphs, a.train, f, f)], env=env, check=True,
                       timeout=300)
        outs[name] = np.load(f)
    base = a.libs[0]
    for name in a.libs[1:]:
        d = outs[name] != outs[base]
        print("%s vs %s: %d of %d values differ (max |diff| %.3g)" % (name, base, int(d.sum()), d.size,
              float(np.abs(outs[name].astype(np.float64) - outs[base]).max())), flush=True)


if __name__ == "__main__":
    main()
