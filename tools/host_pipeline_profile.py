"""Per-stage host time of the training input pipeline for one 512 x synth50 batch (GPU box):
the native reader's gather, normalisation, ign_batch_create, ign_batch_enable_training, the
label copy.  python tools/host_pipeline_profile.py [graphs]; env REPS (per thread), THREADS (concurrent
builders, like the prefetch workers)."""
import os
import sys
import tempfile
import threading
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
    reps = int(os.environ.get("REPS", "3"))
    threads = int(os.environ.get("THREADS", "1"))
    stages = ("gather", "normalise", "batch_create", "enable_training", "destroy")
    times = {k: [] for k in stages}
    lock = threading.Lock()

    def work(seed):
        if os.environ.get("PIN") == "1":   # this builder thread on one CPU of the process's set
            cpus = sorted(os.sched_getaffinity(0))
            os.sched_setaffinity(0, {cpus[seed % len(cpus)]})
        rng = np.random.default_rng(seed)
        for rep in range(reps):
            ids = rng.permutation(n)
            t = [time.perf_counter()]
            bg, labels = ds.batch(ids, keys, narrow=os.environ.get("NARROW", "1") == "1")   # as NativeInput.load
            t.append(time.perf_counter())
            for f in mi.get_all_features():
                if str(f.normalization) != "None" and f.name in bg:
                    v, lens = bg.get(f.name)
                    bg.arrays[f.name] = (np.asarray(gm._resolve(f.normalization)(v, f.name), np.float32), lens)
            t.append(time.perf_counter())
            b = Batch(eng, bg)
            t.append(time.perf_counter())
            b.enable_training()
            t.append(time.perf_counter())
            b.close()
            t.append(time.perf_counter())
            with lock:
                for k, a, c in zip(stages, t[:-1], t[1:]):
                    times[k].append(1e3 * (c - a))
                if threads == 1:
                    print("rep %d: " % rep + ", ".join("%s %.1f ms" % (k, times[k][-1]) for k in stages))

    t0 = time.perf_counter()
    th = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    print("threads %d: %.1f ms per batch (wall / batches); mean per stage: %s" % (
        threads, 1e3 * wall / (threads * reps),
        ", ".join("%s %.1f" % (k, np.mean(times[k][threads:] or times[k])) for k in stages)))

if __name__ == "__main__":
    main()
