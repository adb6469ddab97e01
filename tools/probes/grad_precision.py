"""Gradient precision of the training step's contraction paths vs torch autograd of the float64
restatement (oracle/train_oracle.py): relative L2 error of the whole gradient vector and of the
worst parameter tensor, per environment setting (GPU box).
    python tools/probes/grad_precision.py [n_graphs]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CHILD = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, %r)
sys.path.insert(0, %r + "/tests")
from ignnition_amd import workloads
from ignnition_amd.engine import MPPlan
from oracle.train_oracle import TorchOracle
from test_gpu_training import _engine_grads
desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "synth50", %d)
prm = MPPlan.from_model_info(mi).init_params(13, bias_scale=0.1)
eng, b, pred, loss, g, _ = _engine_grads(desc, dims, graphs, labels, prm)
_, _, og, _ = TorchOracle(desc, dims, prm).loss_and_grads(graphs, labels)
num = sum(float(np.sum((g[k].astype(np.float64) - v) ** 2)) for k, v in og.items())
den = sum(float(np.sum(v ** 2)) for v in og.values())
worst = max((np.linalg.norm(g[k].astype(np.float64) - v) / max(np.linalg.norm(v), 1e-30), k) for k, v in og.items())
print(json.dumps({"rel_l2": (num / den) ** 0.5, "worst": worst}))
'''

SETTINGS = {"default": {}, "train_seq_bf16": {"IGN_TRAIN_SEQ_H16": "0"}, "f32_recompute": {"IGN_BWD_BF": "0"},
            "unfused": {"IGN_BWD_FUSE": "0"}}

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    for name, env in SETTINGS.items():
        r = subprocess.run([sys.executable, "-c", CHILD % (REPO, REPO, n)], env=dict(os.environ, **env),
                           capture_output=True, text=True, timeout=600)
        out = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(name, out[-1] if out else r.stderr[-800:], flush=True)
