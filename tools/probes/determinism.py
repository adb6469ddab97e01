"""Repeat-run determinism of the forward (GPU box): RouteNet GEANT2 x2 at H = 32, every
seq/readout variant pair of tests/test_gpu_parity.py::test_split_fp16_scaling, N repeated forwards
each, per library build (ignnition_amd/ab/lib_<name>.so via IGN_LIB_PATH, or the default).
    python tools/probes/determinism.py [lib names...]"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import sys, copy, os, numpy as np
sys.path.insert(0, %r)
from ignnition_amd import model_examples, synthetic, workloads
from ignnition_amd.engine import Batch, Engine, MPPlan
from ignnition_amd.json_operations import Model_information
desc = model_examples.routenet(hidden=32, iterations=8)
_, dims, _ = workloads.model("routenet")
mi = Model_information(copy.deepcopy(desc), dims)
graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("geant2", g) for g in range(2)])
plan = MPPlan.from_model_info(mi)
prm = plan.init_params(11, bias_scale=0.2)
res = []
for seq, ro in (("2", "1"), ("6", "1"), ("7", "1"), ("2", "4"), ("6", "4")):
    os.environ["IGN_SEQ_VARIANT"] = seq; os.environ["IGN_READOUT_VARIANT"] = ro
    eng = Engine(plan, 0); eng.set_params(prm)
    b = Batch(eng, graphs)
    outs = [b.forward().reshape(-1).copy() for _ in range(6)]
    b.close(); eng.close()
    bad = sum(not np.array_equal(o, outs[0]) for o in outs[1:])
    res.append("%%s/%%s:%%d" %% (seq, ro, bad))
print(" ".join(res))
'''
names = sys.argv[1:] or ["default"]
for n in names:
    env = dict(os.environ)
    if n != "default":
        env["IGN_LIB_PATH"] = os.path.join(REPO, "ignnition_amd", "ab", "lib_%s.so" % n)
        env["IGN_AB_LIB"] = "1"   # an A/B build may predate symbols _lib.py binds (as tools/ab_bitwise.py)
    r = subprocess.run([sys.executable, "-c", CHILD % REPO], env=env, capture_output=True, text=True, timeout=300)
    print("%-10s %s" % (n, r.stdout.strip() or r.stderr[-500:]), flush=True)
