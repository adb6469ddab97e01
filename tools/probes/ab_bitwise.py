"""Bitwise A/B of the forward between library builds (GPU box): RouteNet synth50 x8 and GEANT2 x4
predictions with the default library and with each ignnition_amd/ab/lib_<name>.so (IGN_LIB_PATH),
each in its own process.  python tools/probes/ab_bitwise.py name [name...]"""
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import sys, numpy as np
sys.path.insert(0, %r)
from ignnition_amd import synthetic, workloads
from ignnition_amd.engine import Batch, Engine, MPPlan
desc, dims, mi = workloads.model("routenet")
plan = MPPlan.from_model_info(mi)
prm = plan.init_params(7, bias_scale=0.2)
out = []
for topo, n in (("synth50", 8), ("geant2", 4)):
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample(topo, g) for g in range(n)])
    eng = Engine(plan, 0); eng.set_params(prm)
    b = Batch(eng, graphs)
    out.append(b.forward().reshape(-1).copy())
    b.close(); eng.close()
np.save(sys.argv[1], np.concatenate(out))
''' % REPO


def run(lib, path):
    env = dict(os.environ)
    if lib:
        env["IGN_AB_LIB"] = "1"
        env["IGN_LIB_PATH"] = os.path.join(REPO, "ignnition_amd", "ab", "lib_%s.so" % lib)
    subprocess.run([sys.executable, "-c", CHILD, path], env=env, check=True, timeout=300)
    return np.load(path)


def main():
    tmp = tempfile.mkdtemp(prefix="ign_ab_")
    ref = run(None, os.path.join(tmp, "default.npy"))
    for name in sys.argv[1:]:
        got = run(name, os.path.join(tmp, name + ".npy"))
        diff = np.abs(got.astype(np.float64) - ref)
        print("%s: %d predictions, %d differ, max |diff| %.3g" % (name, ref.size, int((got != ref).sum()), diff.max()))


if __name__ == "__main__":
    main()
