"""Native dataset reader (libignmp.so ign_dataset_*) vs the reference generator's own outputs
(tests/golden/gen_fixtures.json, bit-exact) and vs ignnition_amd.generator on synthetic
datasets.  CPU only: the reader is host code."""
import json
import time

import numpy as np
import pytest

from ignnition_amd import generator as G
from ignnition_amd import synthetic, workloads
from ignnition_amd.dataset import NativeDataset, plan_keys
from ignnition_amd.engine import BatchedGraphs, MPPlan


def _flat(v):
    return np.asarray(v, dtype=np.float64).reshape(-1)


@pytest.mark.parametrize("idx", range(8))
def test_native_reader_matches_reference_fixtures(gen_fixtures, idx, tmp_path):
    case = gen_fixtures[idx]
    synthetic.write_tar_dataset(case["samples"], str(tmp_path), per_file=len(case["samples"]))
    ds = NativeDataset(str(tmp_path), case["feature_names"], case["output_name"], case["adj_names"],
                       case["interleave_names"], [], case["training"], threads=2)
    assert len(ds) == len(case["expected"]), case["name"]
    for sid, exp in enumerate(case["expected"]):
        ds.gather([sid])
        for k, v in exp["data"].items():
            got, lens = ds.get(k)
            if got.dtype == np.int64:
                assert got.tolist() == np.asarray(v).reshape(-1).tolist(), (case["name"], k)
            else:
                np.testing.assert_array_equal(got, _flat(v).astype(np.float32), err_msg="%s %s" % (case["name"], k))
            assert lens.tolist() == [got.size]
        if case["training"]:
            lab, _ = ds.get("__label__")
            np.testing.assert_array_equal(lab, _flat(exp["output"]).astype(np.float32))
    ds.close()


def _compare_with_python(tmp_path, kind, topology, n):
    samples = synthetic.dataset(topology, n, qsize=(kind == "qsize"), first_id=3)
    synthetic.write_tar_dataset(samples, str(tmp_path), per_file=3)
    desc, dims, mi = workloads.model(kind)
    names = [f.name for f in mi.get_all_features()]
    out, _, _ = mi.get_output_info()
    py = list(G.generator(str(tmp_path), names, out, mi.get_adjecency_info(), mi.get_interleave_tensors(), [], True))
    ds = NativeDataset.for_model(str(tmp_path), mi, threads=4)
    assert len(ds) == len(py) == n
    plan = MPPlan.from_model_info(mi)
    keys = plan_keys(plan)
    bg, labels = ds.batch(list(range(n)), keys)
    ref = BatchedGraphs.from_dicts([x for x, _ in py])
    for k in keys:
        got, glen = bg.get(k)
        exp, elen = ref.get(k)
        assert glen.tolist() == elen.tolist(), k
        if got.dtype == np.int64:
            assert got.tolist() == np.asarray(exp, np.int64).tolist(), k
        else:
            np.testing.assert_array_equal(got, np.asarray(exp, np.float32), err_msg=k)
    np.testing.assert_array_equal(labels[0], np.concatenate([np.asarray(y, np.float32) for _, y in py]))
    # a shuffled subset keeps per-sample contents
    sub = [5, 0, 2]
    bg2, _ = ds.batch(sub, keys)
    one = BatchedGraphs.from_dicts([py[i][0] for i in sub])
    for k in keys:
        assert np.array_equal(bg2.get(k)[0], np.asarray(one.get(k)[0], bg2.get(k)[0].dtype)), k
    return ds


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_native_reader_matches_python_generator(tmp_path, kind):
    _compare_with_python(tmp_path, kind, "nsfnet", 7).close()


def test_native_reader_errors_abandon_file(tmp_path):
    good = synthetic.routenet_sample("nsfnet", 0)
    bad = dict(good)
    del bad["traffic"]
    synthetic.write_tar_dataset([good, bad, good], str(tmp_path), per_file=3)
    desc, dims, mi = workloads.model("routenet")
    ds = NativeDataset.for_model(str(tmp_path), mi)
    assert len(ds) == 1           # the first sample is kept, the rest of the file is abandoned
    assert ds.errors and "traffic" in ds.errors[0]


def test_native_reader_missing_data_json_is_fatal(tmp_path):
    import tarfile
    with tarfile.open(str(tmp_path / "x.tar.gz"), "w:gz") as tar:
        p = tmp_path / "other.json"
        p.write_text("[]")
        tar.add(str(p), arcname="other.json")
    desc, dims, mi = workloads.model("routenet")
    with pytest.raises(Exception, match="data.json"):
        NativeDataset.for_model(str(tmp_path), mi)


def test_native_reader_is_faster(tmp_path):
    samples = synthetic.dataset("geant2", 24, qsize=False, first_id=0)
    synthetic.write_tar_dataset(samples, str(tmp_path), per_file=4)
    desc, dims, mi = workloads.model("routenet")
    names = [f.name for f in mi.get_all_features()]
    out, _, _ = mi.get_output_info()
    t0 = time.perf_counter()
    py = list(G.generator(str(tmp_path), names, out, mi.get_adjecency_info(), mi.get_interleave_tensors(), [], True))
    t_py = time.perf_counter() - t0
    t0 = time.perf_counter()
    ds = NativeDataset.for_model(str(tmp_path), mi, threads=4)
    ds.batch(list(range(len(ds))), plan_keys(MPPlan.from_model_info(mi)))
    t_native = time.perf_counter() - t0
    assert len(ds) == len(py)
    assert t_native < t_py


def test_concurrent_batches_equal_serial(tmp_path):
    """ign_dataset_batch objects are independent: batches gathered on 4 threads at once hold
    exactly what one thread gathers (the training input pipeline's workers share one dataset)."""
    from concurrent.futures import ThreadPoolExecutor
    desc, dims, mi = workloads.model("qsize")
    synthetic.write_tar_dataset(synthetic.dataset("nsfnet", 12, qsize=True), str(tmp_path), per_file=5)
    ds = NativeDataset.for_model(str(tmp_path), mi)
    keys = plan_keys(MPPlan.from_model_info(mi))
    rng = np.random.default_rng(0)
    id_sets = [rng.choice(12, size=5, replace=False) for _ in range(16)]

    def one(ids):
        bg, y = ds.batch(ids, keys)
        return {k: (np.array(v), np.array(l)) for k, (v, l) in bg.arrays.items()}, y[0].copy()

    serial = [one(ids) for ids in id_sets]
    with ThreadPoolExecutor(4) as ex:
        par = list(ex.map(one, id_sets))
    for (a, ya), (b, yb) in zip(serial, par):
        np.testing.assert_array_equal(ya, yb)
        assert a.keys() == b.keys()
        for k in a:
            np.testing.assert_array_equal(a[k][0], b[k][0])
            np.testing.assert_array_equal(a[k][1], b[k][1])
    ds.close()


def test_recycled_gather_buffers_equal_fresh(tmp_path, monkeypatch):
    """Destroyed batches hand their concatenation buffers back to the dataset's pool; batches of
    other sizes and orders gathered into them (larger, smaller, repeated) hold exactly what an
    unpooled dataset (IGN_GATHER_POOL=0) gathers, and a batch may outlive its dataset's handle."""
    import gc
    desc, dims, mi = workloads.model("qsize")
    synthetic.write_tar_dataset(synthetic.dataset("nsfnet", 12, qsize=True), str(tmp_path), per_file=5)
    pooled = NativeDataset.for_model(str(tmp_path), mi)
    monkeypatch.setenv("IGN_GATHER_POOL", "0")
    fresh = NativeDataset.for_model(str(tmp_path), mi)
    keys = plan_keys(MPPlan.from_model_info(mi))
    rng = np.random.default_rng(3)
    for size in (3, 12, 2, 7, 12, 1, 5):
        ids = rng.choice(12, size=size, replace=False)
        a, ya = pooled.batch(ids, keys)
        b, yb = fresh.batch(ids, keys)
        np.testing.assert_array_equal(ya[0], yb[0])
        for k in keys:
            np.testing.assert_array_equal(a.get(k)[0], b.get(k)[0])
            np.testing.assert_array_equal(a.get(k)[1], b.get(k)[1])
        del a, b
        gc.collect()
    last, _ = pooled.batch([4, 0, 9], keys)
    pooled.close()
    fresh.close()
    ref = {k: np.array(last.get(k)[0]) for k in keys}
    del last   # destroyed after the dataset: its buffers go to the pool the batch still holds
    gc.collect()
    assert all(v.size for v in ref.values())


def test_narrow_gather_equals_wide(tmp_path):
    """``NativeDataset.batch(..., narrow=True)`` (``ign_dataset_batch_get_narrow``): the integer
    keys as int32 with the int64 gather's values and per-graph lengths, float keys and labels
    unchanged; the wide gather of the same batch still int64 (samples are stored narrow)."""
    desc, dims, mi = workloads.model("qsize")
    synthetic.write_tar_dataset(synthetic.dataset("nsfnet", 6, qsize=True), str(tmp_path), per_file=4)
    ds = NativeDataset.for_model(str(tmp_path), mi)
    keys = plan_keys(MPPlan.from_model_info(mi))
    ids = [4, 0, 5, 2]
    wide, yw = ds.batch(ids, keys)
    nar, yn = ds.batch(ids, keys, narrow=True)
    np.testing.assert_array_equal(yw[0], yn[0])
    n_int = 0
    for k in keys:
        (vw, lw), (vn, ln) = wide.get(k), nar.get(k)
        np.testing.assert_array_equal(lw, ln)
        np.testing.assert_array_equal(vw, vn)
        if vw.dtype == np.int64:
            assert vn.dtype == np.int32, k
            n_int += 1
        else:
            assert vn.dtype == vw.dtype == np.float32, k
    assert n_int >= 6
    ds.close()


class _FakeBatch:
    def __init__(self, v):
        self.v, self.closed = v, False

    def close(self):
        self.closed = True


class _FakeTrainer:
    """Trainer.prepare's contract for the prefetcher: (batch with close(), labels)."""

    def prepare(self, features, labels):
        import random
        time.sleep(random.uniform(0, 0.01))
        if features == "bad":
            raise ValueError("bad batch")
        return _FakeBatch(features), labels


def test_prefetcher_keeps_job_order_and_raises_in_place():
    from ignnition_amd.training import BatchPrefetcher
    jobs = [(k, -k) for k in range(40)]
    pf = BatchPrefetcher(_FakeTrainer(), jobs, depth=6, workers=4)
    got = [(b.v, y) for b, y in pf]
    assert got == jobs
    pf.close()
    pf = BatchPrefetcher(_FakeTrainer(), [(0, 0), ("bad", 1), (2, 2)], depth=3, workers=3,
                         load=lambda job: job)
    assert next(pf)[0].v == 0
    with pytest.raises(ValueError, match="bad batch"):
        next(pf)
    pf.close()


def test_batch_arrays_keep_their_buffers_alive(tmp_path):
    """NativeDataset.batch returns zero-copy views of the gather's buffers; an array taken out of
    the BatchedGraphs must stay valid after the BatchedGraphs is dropped."""
    import gc
    from examples.make_example import make
    from ignnition_amd import framework_operations as fo
    from ignnition_amd.dataset import NativeDataset, plan_keys
    from ignnition_amd.engine import MPPlan
    d = make("routenet", str(tmp_path / "rn"), "nsfnet", 3)
    fo.load_config(d + "/train_options.ini")
    mi = fo.create_model()
    ds = NativeDataset.for_model(fo.CONFIG["PATHS"]["train_dataset"], mi, training=True)
    keys = plan_keys(MPPlan.from_model_info(mi))
    bg, _ = ds.batch([0, 1, 2], keys)
    key = next(k for k in keys if k.startswith("src_"))
    arr = bg.arrays[key][0]
    ref = arr.copy()
    del bg
    gc.collect()
    for _ in range(3):   # reuse the freed memory if it were freed
        ds.batch([2, 1, 0], keys)
    np.testing.assert_array_equal(arr, ref)


def test_builder_cpus_are_disjoint_per_local_rank(monkeypatch):
    """Batch-builder pinning (IGN_PIN_BUILDERS): each builder gets CPUs of the process's affinity,
    local ranks take disjoint slices (or none when they do not fit), and the switch turns it off."""
    import os
    from ignnition_amd.training import builder_cpus
    monkeypatch.setenv("IGN_PIN_BUILDERS", "1")
    allowed = os.sched_getaffinity(0)
    seen = set()
    for lr in range(2):
        monkeypatch.setenv("LOCAL_RANK", str(lr))
        sets = builder_cpus(2)
        assert len(sets) == 2
        for c in sets:
            assert c <= allowed
            assert not (c & seen)
            seen |= c
    monkeypatch.setenv("LOCAL_RANK", "1000")
    assert builder_cpus(2) == [set(), set()]
    monkeypatch.setenv("IGN_PIN_BUILDERS", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    assert builder_cpus(3) == [set(), set(), set()]
