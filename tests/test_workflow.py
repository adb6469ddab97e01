"""User workflow through train_options.ini + model_description.json (FO:34-91, 169-268)."""
import json
import os

import numpy as np
import pytest

from ignnition_amd import framework_operations as fo
from ignnition_amd import generate_model as gm
from ignnition_amd import workloads
from examples.make_example import make


@pytest.fixture()
def example_dir(tmp_path):
    d = make("routenet", str(tmp_path / "rn"), "nsfnet", 3)
    fo.load_config(os.path.join(d, "train_options.ini"))
    gm.register_user_functions(workloads.USER_FUNCTIONS)
    return d


def test_create_model_and_debug(example_dir):
    mi = fo.create_model()
    assert mi.get_mp_iterations() == 8
    dims = fo.find_dataset_dimensions(fo.CONFIG["PATHS"]["train_dataset"])
    assert dims["traffic"] == 1 and dims["adj_links_paths"] == 0
    dump = fo.debug(mi, out_dir=os.path.join(example_dir, "debug_model"))
    plan = json.load(open(os.path.join(example_dir, "debug_model", "plan.json")))
    assert plan["iterations"] == 8 and len(plan["message_passings"]) == 2
    assert dump["cells"][0][0] == "path"


def test_input_fn_native_matches_python(example_dir):
    """The native input path yields the same normalised arrays and labels as input_fn."""
    from ignnition_amd.engine import BatchedGraphs
    mi = fo.create_model()
    gm.set_model_info(mi)
    path = fo.CONFIG["PATHS"]["train_dataset"]
    xs, ys = next(gm.input_fn(path, training=True, batch_size=3, repeat=False))
    bg, yn = next(gm.input_fn_native(path, training=True, batch_size=3, repeat=False))
    ref = BatchedGraphs.from_dicts(xs)
    for k in bg.arrays:
        np.testing.assert_allclose(bg.get(k)[0], np.asarray(ref.get(k)[0], bg.get(k)[0].dtype), rtol=1e-6, err_msg=k)
    np.testing.assert_allclose(yn[0], np.concatenate([np.asarray(y, np.float32) for y in ys]), rtol=1e-6)


def test_input_fn_batches(example_dir):
    mi = fo.create_model()
    gm.set_model_info(mi)
    it = gm.input_fn(fo.CONFIG["PATHS"]["train_dataset"], training=True, batch_size=2, repeat=False)
    xs, ys = next(it)
    assert len(xs) == 2 and len(ys) == 2
    # labels normalised with `log` (RNJ:107)
    assert np.all(np.asarray(ys[0]) < 5)


@pytest.mark.gpu
def test_predict_end_to_end(example_dir):
    from oracle.dense_forward import DenseOracle
    mi = fo.create_model()
    prm = __import__("ignnition_amd.engine", fromlist=["MPPlan"]).MPPlan.from_model_info(mi).init_params(3)
    preds = fo.predict(mi, params=prm, batch_size=2)
    assert len(preds) == 3
    gm.set_model_info(mi)
    graphs = [g for batch in gm.input_fn(fo.CONFIG["PATHS"]["predict_dataset"], training=False, repeat=False)
              for g in batch]
    desc = json.load(open(fo.CONFIG["PATHS"]["json_path"]))
    ref = DenseOracle(desc, fo.find_dataset_dimensions(fo.CONFIG["PATHS"]["train_dataset"]), prm).forward(graphs)
    got = np.concatenate(preds)   # no label_denormalization in RNJ -> normalised outputs
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_train_and_evaluate_end_to_end(example_dir):
    """FO:108-166: steps, checkpoints, eval metrics, warm start."""
    from ignnition_amd.checkpoint import load_params
    mi = fo.create_model()
    fo.CONFIG["TRAINING_OPTIONS"]["train_steps"] = "25"
    fo.CONFIG["TRAINING_OPTIONS"]["batch_size"] = "3"
    fo.CONFIG["TRAINING_OPTIONS"]["eval_samples"] = "3"
    fo.CONFIG["TRAINING_OPTIONS"]["keep_checkpoint_max"] = "2"
    res = fo.train_and_evaluate(mi, log_every=5)
    m = res["final_metrics"]
    assert m["step"] == 25 and m["samples"] == 3
    assert np.isfinite(m["loss"]) and np.isfinite(m["mae"]) and np.isfinite(m["r-squared"])
    assert res["trainer"].iterations == 25
    assert 1 <= len(res["checkpoints"]) <= 2 and all(os.path.exists(c) for c in res["checkpoints"])
    assert os.path.exists(os.path.join(res["model_dir"], "metrics.jsonl"))
    saved = load_params(res["checkpoints"][-1])
    now = res["trainer"].params()
    for k in now:
        np.testing.assert_array_equal(saved[k], now[k])
    # warm start from the checkpoint continues from those parameters
    fo.CONFIG["PATHS"]["warm_start_path"] = res["checkpoints"][-1]
    fo.CONFIG["TRAINING_OPTIONS"]["train_steps"] = "1"
    res2 = fo.train_and_evaluate(mi)
    assert res2["trainer"].iterations == 1
    del fo.CONFIG["PATHS"]["warm_start_path"]


@pytest.mark.gpu
def test_training_learns_on_repeated_batch(example_dir):
    from ignnition_amd.training import Trainer
    mi = fo.create_model()
    gm.set_model_info(mi)
    xs, ys = next(gm.input_fn(fo.CONFIG["PATHS"]["train_dataset"], batch_size=3))
    tr = Trainer(mi, seed=1)
    tr.lr.lr0 = 0.003
    first = tr.train_step(xs, ys)["loss"]
    for _ in range(40):
        last = tr.train_step(xs, ys)["loss"]
    assert last < 0.5 * first


@pytest.mark.gpu
def test_native_batches_equal_dict_batches(example_dir):
    """A batch built from the native reader's arrays predicts bit-identically to one built from
    the Python generator's dicts."""
    from ignnition_amd.engine import Batch, Engine, MPPlan
    mi = fo.create_model()
    gm.set_model_info(mi)
    path = fo.CONFIG["PATHS"]["train_dataset"]
    xs, _ = next(gm.input_fn(path, training=True, batch_size=3, repeat=False))
    bg, _ = next(gm.input_fn_native(path, training=True, batch_size=3, repeat=False))
    plan = MPPlan.from_model_info(mi)
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(2))
    np.testing.assert_array_equal(Batch(eng, xs).forward(), Batch(eng, bg).forward())


def test_native_batches_cross_epochs_like_the_reference(example_dir):
    """ds.repeat() before batching (GM:185-194): a batch may span the end of one epoch and the
    start of the next; the native stream and the Python input_fn cut the same batches."""
    mi = fo.create_model()
    gm.set_model_info(mi)
    path = fo.CONFIG["PATHS"]["train_dataset"]       # 3 samples
    nat = gm.input_fn_native(path, training=True, batch_size=2)
    py = gm.input_fn(path, training=True, batch_size=2)
    ids = []
    for _ in range(3):
        bg, yn = next(nat)
        xs, ys = next(py)
        ids.append(bg.sample_ids)
        np.testing.assert_allclose(yn[0], np.concatenate([np.asarray(y, np.float32) for y in ys]), rtol=1e-6)
    assert ids == [[0, 1], [2, 0], [1, 2]]


def test_data_parallel_slices_are_disjoint(example_dir):
    """World 2, one shared seed: the two ranks' batches of a step are the halves of one global
    batch of the single-rank stream (disjoint stream positions; every sample of an epoch used once)."""
    mi = fo.create_model()
    gm.set_model_info(mi)
    path = fo.CONFIG["PATHS"]["train_dataset"]
    whole = gm.input_fn_native(path, shuffle=True, batch_size=2, seed=11)
    ranks = [gm.input_fn_native(path, shuffle=True, batch_size=1, seed=11, rank=r, world=2) for r in range(2)]
    seen = []
    for _ in range(6):
        g = next(whole)[0].sample_ids
        parts = [next(r)[0].sample_ids for r in ranks]
        assert parts[0] + parts[1] == g   # (a global batch across an epoch end may repeat a sample)
        seen += g
    for e in range(4):   # 12 draws = 4 epochs of 3 samples, each a permutation
        assert sorted(seen[3 * e:3 * e + 3]) == [0, 1, 2]


def test_warm_start_overlays_matching_tensors():
    """FO:126-131: tensors whose variable name matches kernel.* / recurrent_kernel.* / bias.* come
    from the checkpoint (attention/kernel1 included), the rest keep their initial values, a
    partial checkpoint is fine, and a shape mismatch raises."""
    from ignnition_amd import model_examples
    from ignnition_amd.engine import MPPlan
    from ignnition_amd.json_operations import Model_information
    desc = model_examples.routenet_aggregation({"type": "attention"}, hidden=16, iterations=2)
    _, dims, _ = workloads.model("routenet")
    init = MPPlan.from_model_info(Model_information(desc, dims)).init_params(0)
    ckpt = {"attention/kernel1": np.full_like(init["attention/kernel1"], 2.0),
            "attention/attn_kernel": np.full_like(init["attention/attn_kernel"], 3.0),
            "path_update/recurrent_kernel": np.full_like(init["path_update/recurrent_kernel"], 4.0)}
    out = fo.warm_start(init, ckpt)
    assert set(out) == set(init)
    assert np.all(out["attention/kernel1"] == 2.0) and np.all(out["path_update/recurrent_kernel"] == 4.0)
    np.testing.assert_array_equal(out["attention/attn_kernel"], init["attention/attn_kernel"])   # attn_kernel !~ kernel.*
    np.testing.assert_array_equal(out["path_update/kernel"], init["path_update/kernel"])         # not in the checkpoint
    with pytest.raises(ValueError, match="shape"):
        fo.warm_start(init, {"path_update/kernel": np.zeros((3, 3), np.float32)})


def test_set_params_checks_names_and_shapes():
    from ignnition_amd.engine import Engine, MPPlan
    _, dims, mi = workloads.model("routenet")
    plan = MPPlan.from_model_info(mi)
    eng = Engine(plan, 0)
    prm = plan.init_params(0)
    missing = dict(prm)
    del missing["path_update/bias"]
    with pytest.raises(ValueError, match="missing"):
        eng.set_params(missing)
    bad = dict(prm)
    bad["path_update/kernel"] = np.zeros((5, 96), np.float32)
    with pytest.raises(ValueError, match="shape"):
        eng.set_params(bad)
    eng.close()


def test_warm_start_full_name_rule_is_tfs_anchored_match():
    """match="full": TF's get_collection(scope=regex) rule, re.match on the full variable name;
    the reference's patterns then select only top-level names (none in its models)."""
    init = {"path_update/kernel": np.zeros((2, 3), np.float32), "kernel_top": np.zeros(2, np.float32),
            "bias": np.zeros(1, np.float32)}
    ckpt = {k: np.ones_like(v) for k, v in init.items()}
    full = fo.warm_start(init, ckpt, match="full")
    assert np.all(full["kernel_top"] == 1) and np.all(full["bias"] == 1)
    assert np.all(full["path_update/kernel"] == 0)
    comp = fo.warm_start(init, ckpt)
    assert all(np.all(v == 1) for v in comp.values())
    with pytest.raises(ValueError, match="match"):
        fo.warm_start(init, ckpt, match="prefix")


def test_python_input_stream_has_its_own_rng(example_dir):
    """Data-parallel input_fn streams shuffle with random.Random(seed): draws from the global
    random between them (rank 0's eval generator) do not move one rank's order, so the two ranks'
    batches stay the halves of the one-rank stream's global batches."""
    import random
    mi = fo.create_model()
    gm.set_model_info(mi)
    path = fo.CONFIG["PATHS"]["train_dataset"]
    whole = gm.input_fn(path, shuffle=True, batch_size=2, seed=5)
    ranks = [gm.input_fn(path, shuffle=True, batch_size=1, seed=5, rank=r, world=2) for r in range(2)]
    lab = lambda ys: [float(np.asarray(y).reshape(-1)[0]) for y in ys]
    for _ in range(6):
        g = lab(next(whole)[1])
        random.random()                       # another thread's draw on the global generator
        r0 = lab(next(ranks[0])[1])
        random.shuffle(list(range(10)))
        r1 = lab(next(ranks[1])[1])
        assert r0 + r1 == g


def test_split_cuts_partition_graphs_evenly():
    """engine.SplitBatch's sub-batches: consecutive graphs, every graph once, sizes within one."""
    from ignnition_amd.engine import split_cuts
    for n in (1, 2, 3, 5, 16, 511, 512):
        for parts in (1, 2, 3, 4, 8):
            c = split_cuts(n, parts)
            assert c[0] == 0 and c[-1] == n and len(c) == min(parts, n) + 1
            sizes = [b - a for a, b in zip(c, c[1:])]
            assert min(sizes) >= 1 and max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        split_cuts(0, 2)
