"""Per-stage host time of the training input pipeline for one 512 x synth50 batch (GPU box):
the native reader's gather, normalisation, ign_batch_create, ign_batch_enable_training, the
label copy.  python tools/host_pipeline_profile.py [graphs]"""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

from ignnition_amd import generate_model as gm  # noqa: E402
from ignnition_amd import synthetic, workloads  # noqa: E402
from ignnition_amd.dataset import NativeDataset, plan_keys  # noqa: E402
from ignnition_amd.engine import Batch, Engine, MPPlan  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    desc, dims, mi = workloads.model("routenet")
    tmp = tempfile.mkdtemp(prefix="ign_prof_")
    t = time.perf_counter()
    synthetic.write_tar_dataset(synthetic.dataset("synth50", n), os.path.join(tmp, "train"))
    print("write dataset %.2f s" % (time.perf_counter() - t))
    gm.register_user_functions(workloads.USER_FUNCTIONS)
    gm.set_model_info(mi)
    plan = MPPlan.from_model_info(mi)
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(0))
    t = time.perf_counter()
    ds = NativeDataset.for_model(os.path.join(tmp, "train"), mi)
    print("open + parse %.3f s" % (time.perf_counter() - t))
    keys = plan_keys(plan)
    rng = np.random.default_rng(0)
    for rep in range(3):
        ids = rng.permutation(n)
        t0 = time.perf_counter()
        bg, labels = ds.batch(ids, keys)
        t1 = time.perf_counter()
        for f in mi.get_all_features():
            if str(f.normalization) != "None" and f.name in bg:
                v, lens = bg.get(f.name)
                bg.arrays[f.name] = (np.asarray(gm._resolve(f.normalization)(v, f.name), np.float32), lens)
        t2 = time.perf_counter()
        b = Batch(eng, bg)
        t3 = time.perf_counter()
        b.enable_training()
        t4 = time.perf_counter()
        b.close()
        t5 = time.perf_counter()
        print("rep %d: gather %.1f ms, normalise %.1f ms, batch_create %.1f ms, enable_training %.1f ms, "
              "destroy %.1f ms" % (rep, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3),
                                   1e3 * (t5 - t4)))


if __name__ == "__main__":
    main()
