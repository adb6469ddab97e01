"""Training step on the GPU vs the torch-autograd oracle (oracle/train_oracle.py, float64).

Tolerance: per parameter tensor, ||g_engine - g_oracle|| <= 1e-4 * ||g_oracle||
(+1e-7 absolute for tensors whose gradient is ~0); loss within 1e-5 relative; Adam update of
the parameters within 1e-6 relative of the float64 restatement."""
import copy

import numpy as np
import pytest
import torch

from ignnition_amd import model_examples, synthetic, workloads
from ignnition_amd.engine import Batch, Engine, MPPlan, device_count
from ignnition_amd.json_operations import Model_information
from oracle.train_oracle import TorchOracle, adam_step

pytestmark = pytest.mark.gpu

GTOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")


def _engine_grads(desc, dims, graphs, labels, prm, eng=None):
    if eng is None:
        mi = Model_information(copy.deepcopy(desc), dims)
        plan = MPPlan.from_model_info(mi)
        eng = Engine(plan, 0)
        eng.set_params(prm)
    b = Batch(eng, graphs)
    b.enable_training()
    pred = b.forward_train()
    y = torch.tensor(np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels]), device="cuda")
    dpred = torch.empty_like(y)
    loss = eng.mse_loss(b.predictions_ptr(), y, dpred)
    grads = torch.zeros(eng.n_params, dtype=torch.float32, device="cuda")
    b.backward(dpred, grads)
    torch.cuda.synchronize()
    g = grads.cpu().numpy()
    named = {name: g[off:off + int(np.prod(shape))].reshape(shape) for name, shape, off in eng.layout}
    return eng, b, pred, loss, named, grads


def _check(desc, dims, graphs, labels, prm):
    eng, b, pred, loss, g, _ = _engine_grads(desc, dims, graphs, labels, prm)
    o_loss, o_reg, o_g, o_pred = TorchOracle(desc, dims, prm).loss_and_grads(graphs, labels)
    np.testing.assert_allclose(pred.reshape(-1), o_pred, rtol=1e-4, atol=1e-4)
    assert loss == pytest.approx(o_loss, rel=1e-5)
    assert eng.l2_loss() == pytest.approx(o_reg, rel=1e-5)
    for name, og in o_g.items():
        err = np.linalg.norm(g[name].astype(np.float64) - og)
        assert err <= GTOL * np.linalg.norm(og) + 1e-7, "%s: rel err %.3g" % (name, err / max(np.linalg.norm(og), 1e-30))
    return eng, b


@pytest.mark.parametrize("kind,n", [("routenet", 1), ("routenet", 3), ("qsize", 2)])
def test_gradients_match_autograd(kind, n):
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "nsfnet", n)
    prm = MPPlan.from_model_info(mi).init_params(7, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


@pytest.mark.parametrize("hidden", [16, 64])
def test_gradients_hidden_sizes(hidden):
    desc = model_examples.routenet(hidden=hidden, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", 5)])
    prm = MPPlan.from_model_info(mi).init_params(2, bias_scale=0.2)
    _check(desc, dims, graphs, labels, prm)


def test_gradients_synthetic_graph():
    desc, dims, mi, graphs, labels = workloads.make_synthetic_inputs(n_nodes=1500, iterations=2, window=40)
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    _check(desc, dims, graphs, [np.asarray(l, np.float32) for l in labels], prm)


def test_backward_extreme_scales():
    """The ordered backward's split-fp16 dh = du U^T (train_kernels.hip) scales du per row by Sd and
    folds Uᵀ's pack scale sigma_t into the seed / unseed powers of two: with a tiny recurrent kernel
    (sigma_t ~ 2^76) and tiny path gradients (the output layer scaled by 2^-50, so du ~ 2^-50) their
    exponents must stay normal.  Every gradient tensor within 1e-4 relative of the float64
    oracle (no absolute slack: all of them are tiny here)."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "nsfnet", 1)
    prm = MPPlan.from_model_info(mi).init_params(3, bias_scale=0.1)
    prm["path_update/recurrent_kernel"] = prm["path_update/recurrent_kernel"] * np.float32(2.0 ** -60)
    prm["readout_model_0/Output_layer/kernel"] = prm["readout_model_0/Output_layer/kernel"] * np.float32(2.0 ** -50)
    eng, b, pred, loss, g, _ = _engine_grads(desc, dims, graphs, labels, prm)
    _, _, o_g, o_pred = TorchOracle(desc, dims, prm).loss_and_grads(graphs, labels)
    np.testing.assert_allclose(pred.reshape(-1), o_pred, rtol=1e-4, atol=1e-4)
    for name, og in o_g.items():
        assert np.all(np.isfinite(g[name])), name
        ref = np.linalg.norm(og)
        if ref == 0:
            continue
        err = np.linalg.norm(g[name].astype(np.float64) - og)
        assert err <= GTOL * ref, "%s: rel err %.3g (|g| %.3g)" % (name, err / ref, ref)


def test_adam_step_matches_keras_restatement():
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "nsfnet", 2)
    prm = MPPlan.from_model_info(mi).init_params(1, bias_scale=0.1)
    eng, b, pred, loss, g, grads = _engine_grads(desc, dims, graphs, labels, prm)
    m = torch.zeros_like(grads)
    v = torch.zeros_like(grads)
    ref = {k: np.asarray(x, np.float64) for k, x in prm.items()}
    rm = {k: np.zeros_like(x) for k, x in ref.items()}
    rv = {k: np.zeros_like(x) for k, x in ref.items()}
    for it in range(3):
        eng.adam_step(grads, m, v, it, 0.01)
        adam_step(ref, {k: g[k].astype(np.float64) for k in ref}, rm, rv, it, 0.01)
    got = eng.get_params()
    for k in ref:
        np.testing.assert_allclose(got[k], ref[k], rtol=1e-5, atol=1e-6)
    # the repacked fragments follow: a forward with the updated parameters equals a fresh plan's
    fresh = Engine(MPPlan.from_model_info(mi), 0)
    fresh.set_params(got)
    np.testing.assert_array_equal(Batch(fresh, graphs).forward(), Batch(eng, graphs).forward())


def test_backward_consumes_the_forward():
    """The readout backward writes the output layer's gradient rows over the saved activations
    (fuse_outer_bwd), so a second backward of one forward is refused (ign_backward, ignmp.h); after
    the next forward_train the backward runs again and gives the same bits."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "nsfnet", 1)
    prm = MPPlan.from_model_info(mi).init_params(1, bias_scale=0.1)
    eng, b, pred, loss, g, grads = _engine_grads(desc, dims, graphs, labels, prm)
    first = grads.clone()
    y = torch.tensor(np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels]), device="cuda")
    dpred = torch.empty_like(y)
    eng.mse_loss(b.predictions_ptr(), y, dpred)
    with pytest.raises(Exception, match="one backward per forward"):
        b.backward(dpred, grads)
    b.forward_train(to_host=False)
    eng.mse_loss(b.predictions_ptr(), y, dpred)
    b.backward(dpred, grads)
    torch.cuda.synchronize()
    assert torch.equal(grads, first)


@pytest.mark.parametrize("kind,topo,n", [("routenet", "nsfnet", 3), ("routenet", "synth50", 2), ("qsize", "nsfnet", 2),
                                         ("qsize", "synth50", 2), ("routenet", "holes", 2)])
def test_resident_training_forward_is_the_batched_one(monkeypatch, kind, topo, n):
    """The training forward's MP loop as one graph-resident launch (resident.hip's SAVE variant,
    IGN_RESIDENT_TRAIN=1, default) leaves the same state versions, per-step saves and message sums as
    the per-MP launches (=0): predictions, loss and every gradient bitwise equal, and within the
    autograd tolerance of the float64 restatement."""
    if topo == "holes":
        from tests.test_gpu_parity import _routenet_graph, _with_holes
        desc, dims, mi, g = _routenet_graph("geant2", 8)
        graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("geant2", 8),
                                                    synthetic.routenet_sample("nsfnet", 4)])
        graphs = [_with_holes(graphs[0], skip=5, count=6), graphs[1]]
    else:
        desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, topo, n)
    prm = MPPlan.from_model_info(mi).init_params(9, bias_scale=0.1)
    runs = {}
    for v in ("1", "0"):
        monkeypatch.setenv("IGN_RESIDENT_TRAIN", v)
        plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
        eng = Engine(plan, 0)
        eng.set_params(prm)
        eng.set_timing(True)
        eng, b, pred, loss, g, grads = _engine_grads(desc, dims, graphs, labels, prm, eng)
        st = eng.stats()
        assert st["mp_resident"]["launches"] == (1 if v == "1" else 0), st
        runs[v] = (pred.reshape(-1), loss, grads.cpu().numpy())
        b.close()
        eng.close()
    np.testing.assert_array_equal(runs["1"][0], runs["0"][0])
    assert runs["1"][1] == runs["0"][1]
    np.testing.assert_array_equal(runs["1"][2], runs["0"][2])
    if topo != "holes":
        # Q-size synth50: the training forward sums a node's 49-420 messages as one float32 chain (the
        # lane walk that keeps x_save, not the inference forward's segmented order), 1.37e-4 here
        e = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, runs["1"][2], eng.layout)
        assert e <= (2 * GTOL if (kind, topo) == ("qsize", "synth50") else GTOL), e


def test_deferred_weight_gradient_reduction(monkeypatch):
    """The sum and ordered MPs' per-instance weight gradients keep their partial tiles and are reduced
    once per backward (IGN_DEFER_WGRAD=1, default) instead of once per MP instance (=0): the same
    gradients up to fp32 reassociation, bitwise deterministic, and within the autograd tolerance."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("qsize", "nsfnet", 3)
    prm = MPPlan.from_model_info(mi).init_params(12, bias_scale=0.1)
    got = {}
    for v in ("1", "0"):
        monkeypatch.setenv("IGN_DEFER_WGRAD", v)
        eng, _, _, _, _, g = _engine_grads(desc, dims, graphs, labels, prm)
        got[v] = g.cpu().numpy()
        if v == "1":
            np.testing.assert_array_equal(got[v], _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy())
    assert np.linalg.norm(got["1"].astype(np.float64) - got["0"]) <= 1e-6 * np.linalg.norm(got["0"])
    assert _rel_err_vs_oracle(desc, dims, graphs, labels, prm, got["1"], eng.layout) <= GTOL


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_fused_sum_backward_weight_gradients(monkeypatch, kind):
    """The 32-wide sum MPs' backward forms dW = x^T da and dU = h^T du in the kernel (f32 MFMA through a
    per-wave transpose tile, IGN_SUM_BWD_FUSE=1, default) instead of writing da / du for two split-bf16
    row contractions (=0): every gradient within fp32 reassociation of the other form, bitwise
    deterministic, and within the autograd tolerance."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "nsfnet", 3)
    prm = MPPlan.from_model_info(mi).init_params(14, bias_scale=0.1)
    got = {}
    for v in ("1", "0"):
        monkeypatch.setenv("IGN_SUM_BWD_FUSE", v)
        eng, _, _, _, _, g = _engine_grads(desc, dims, graphs, labels, prm)
        got[v] = g.cpu().numpy()
        if v == "1":
            np.testing.assert_array_equal(got[v], _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy())
    named = {v: {n: got[v][off:off + int(np.prod(sh))] for n, sh, off in eng.layout} for v in got}
    for n in named["0"]:
        ref = np.linalg.norm(named["0"][n].astype(np.float64))
        assert np.linalg.norm(named["1"][n].astype(np.float64) - named["0"][n]) <= 1e-6 * ref + 1e-12, n
    assert _rel_err_vs_oracle(desc, dims, graphs, labels, prm, got["1"], eng.layout) <= GTOL


def test_training_reduces_loss():
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "nsfnet", 4)
    prm = MPPlan.from_model_info(mi).init_params(0)
    eng, b, pred, loss0, g, grads = _engine_grads(desc, dims, graphs, labels, prm)
    y = torch.tensor(np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels]), device="cuda")
    dpred = torch.empty_like(y)
    m = torch.zeros_like(grads)
    v = torch.zeros_like(grads)
    losses = []
    for it in range(30):
        b.forward_train(to_host=False)
        losses.append(eng.mse_loss(b.predictions_ptr(), y, dpred))
        b.backward(dpred, grads)
        eng.adam_step(grads, m, v, it, 0.003)
    assert losses[-1] < 0.5 * losses[0]


# ---------------------------------------------------------------------------------------------
# message-creation networks (GM:440-475): gradients through the per-edge Dense stack
def _msg_net_case(inputs, units, activation, ordered=False, l2=None):
    from ignnition_amd.framework_operations import dimensions_of_sample
    rng = np.random.default_rng(3)
    if ordered:   # network on the link -> path (ordered) messages
        desc = model_examples.routenet(iterations=3)
        src = desc["message_passing"]["stages"][0]["stage_mp"][0]["source_entities"][0]
        src["message"] = [{"type": "neural_network", "nn_name": "message_nn", "input": list(inputs)}]
        desc["neural_networks"].append({"nn_name": "message_nn", "nn_type": "feed_forward", "nn_architecture": [
            {"type_layer": "Dense", "units": u, "activation": activation} for u in units]})
    else:
        desc = model_examples.routenet_message_net(inputs=inputs, units=units, activation=activation, iterations=3)
    if l2:
        net = [n for n in desc["neural_networks"] if n["nn_name"] == "message_nn"][0]
        net["nn_architecture"][0]["kernel_regularizer"] = l2
    samples = [synthetic.routenet_sample("nsfnet", g) for g in range(2)]
    if "edge_params" in inputs:
        for s in samples:
            s["adj_paths_links"] = {l: [[p, [float(rng.uniform(0, 1)), float(rng.uniform(-1, 1))]] for p in ps]
                                    for l, ps in s["adj_paths_links"].items()}
    dims = dimensions_of_sample(samples[0])
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, samples)
    prm = MPPlan.from_model_info(mi).init_params(6, bias_scale=0.1)
    return desc, dims, graphs, labels, prm


@pytest.mark.parametrize("inputs,units,act,ordered,l2", [
    (("hs_source", "hs_dest"), (24, 32), "selu", False, 0.01),
    (("hs_dest", "hs_source", "edge_params"), (32,), "tanh", False, None),
    (("hs_source", "hs_dest"), (32,), "tanh", True, None),
])
def test_gradients_message_networks(inputs, units, act, ordered, l2):
    desc, dims, graphs, labels, prm = _msg_net_case(inputs, units, act, ordered, l2)
    _check(desc, dims, graphs, labels, prm)


@pytest.mark.parametrize("inputs", [("hs_source", "hs_dest"), ("hs_dest", "hs_source", "edge_params")])
def test_gradients_attention_over_message_network(inputs):
    """Attention (AUX:287-343) whose source rows are a message network's per-edge outputs
    (GM:440-475): the score and weighted-message gradients of each edge flow back through the
    network to the states it read."""
    desc, dims, graphs, labels, prm = _msg_net_case(inputs, (32,), "tanh")
    desc["message_passing"]["stages"][1]["stage_mp"][0]["aggregation"] = {"type": "attention"}
    prm = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims)).init_params(8, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


@pytest.mark.parametrize("aggr", [{"type": "convolution"}, {"type": "convolution", "activation_function": "tanh"},
                                  {"type": "convolution", "activation_function": "selu"}])
def test_gradients_convolution(aggr):
    """Convolution aggregation (AUX:384-401): x = act((sum_m h_src K + h) / deg) into the GRU."""
    desc = model_examples.routenet_aggregation(aggr, hidden=32, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


@pytest.mark.parametrize("axis", [1, 2])
def test_gradients_concat(axis):
    """{link, node} -> path concatenated on axis 1 (slots) or 2 (features, AUX:443-456)."""
    desc = model_examples.qsize_aggregation({"type": "concat", "concat_axis": axis}, iterations=3)
    _, dims, _ = workloads.model("qsize")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g, qsize=True) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


def test_gradients_attention_routenet():
    """Attention aggregation (AUX:287-343): scores, the axis-0 softmax over (graph, position)
    cells, the weighted sum, into the GRU; gradients reach K1, K2 and the attention vector."""
    desc = model_examples.routenet_aggregation({"type": "attention"}, hidden=32, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


def test_gradients_attention_two_sources():
    """{link, node} -> path attention: the combined edge list and the position quirk (GM:539-541)."""
    desc = model_examples.qsize_aggregation({"type": "attention"}, iterations=3)
    _, dims, _ = workloads.model("qsize")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g, qsize=True) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    _check(desc, dims, graphs, labels, prm)


@pytest.mark.parametrize("case", ["pool_sum", "pool_mean", "pool_max", "nn_pool_product", "product_width1",
                                  "extend_nn", "extend_pool", "shadow_entity_name"])
def test_gradients_readout_operations(case):
    """Readout operations before predict (GM:605-655): neural_network, pooling (max: tf's
    gradient split among ties), element-wise product with broadcasting, extend_adjacencies."""
    from oracle.dense_forward import DenseOracle
    from tests.readout_cases import READOUT_CASES
    ops, pin, nets = READOUT_CASES[case]
    desc = model_examples.routenet_readout(ops, pin, nets, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet" if g % 2 == 0 else "geant2", g)
                                            for g in range(3)])
    prm = MPPlan.from_model_info(mi).init_params(11, bias_scale=0.1)
    ora = DenseOracle(desc, dims, prm)
    rng = np.random.default_rng(5)   # labels shaped like each graph's predictions
    labels = [rng.normal(size=ora.forward_graph(g).size).astype(np.float32) for g in graphs]
    _check(desc, dims, graphs, labels, prm)


def _rel_err_vs_oracle(desc, dims, graphs, labels, prm, gflat, layout):
    """Relative L2 error of a flat engine gradient against torch autograd of the float64 restatement."""
    _, _, og, _ = TorchOracle(desc, dims, prm).loss_and_grads(graphs, labels)
    named = {name: gflat[off:off + int(np.prod(shape))].reshape(shape) for name, shape, off in layout}
    num = sum(float(np.sum((named[k].astype(np.float64) - v) ** 2)) for k, v in og.items())
    return (num / sum(float(np.sum(v ** 2)) for v in og.values())) ** 0.5


def test_fused_backward_is_deterministic_and_matches_unfused(monkeypatch):
    """The ordered backward forms dU from per-wave partials reduced in a fixed order: two runs are
    bitwise equal.  Against the du-buffer + row-contraction form (IGN_BWD_FUSE=0, which also runs
    the split-bf16 training forward): both within the same distance of float64 autograd.  (On
    synth50 batches every fp32 evaluation of this gradient sits ~7e-5 (relative L2) from float64,
    dominated by the forward's rounding, so two forms whose FORWARDS round differently differ by
    that much)"""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "synth50", 6)
    prm = MPPlan.from_model_info(mi).init_params(11, bias_scale=0.1)
    eng, _, _, _, _, g1 = _engine_grads(desc, dims, graphs, labels, prm)
    g1 = g1.cpu().numpy()
    g2 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    np.testing.assert_array_equal(g1, g2)
    monkeypatch.setenv("IGN_BWD_FUSE", "0")
    g3 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    e1 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g1, eng.layout)
    e3 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g3, eng.layout)
    print("vs float64 autograd: fused %.3g, unfused %.3g" % (e1, e3))
    assert e1 <= max(1.25 * e3, 1e-6) and e1 <= GTOL


@pytest.mark.parametrize("switch", ["IGN_BWD_BF", "IGN_TRAIN_SEQ_H16"])
def test_split_ordered_training_is_fp32_accurate(monkeypatch, switch):
    """The training forward's split-fp16 ordered update (seq_gru_h16<SAVE>) with the backward's
    bitwise gate recompute and split-fp16 dh = du . U^T (per-row du scales), against the split-bf16
    forward + f32 recompute (IGN_BWD_BF=0) and the split-bf16 forward + recompute
    (IGN_TRAIN_SEQ_H16=0): bitwise deterministic, and no farther from float64 autograd."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "synth50", 6)
    prm = MPPlan.from_model_info(mi).init_params(13, bias_scale=0.1)
    eng, _, _, _, _, g1 = _engine_grads(desc, dims, graphs, labels, prm)
    g1 = g1.cpu().numpy()
    np.testing.assert_array_equal(g1, _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy())
    monkeypatch.setenv(switch, "0")
    g0 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    assert not np.array_equal(g0, g1)   # the switch took effect
    e1 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g1, eng.layout)
    e0 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g0, eng.layout)
    print("%s: vs float64 autograd, default %.3g, off %.3g" % (switch, e1, e0))
    assert e1 <= max(1.25 * e0, 1e-6) and e1 <= GTOL


@pytest.mark.parametrize("switch", ["IGN_TSGEMM_BF", "IGN_TRAIN_DENSE_BF", "IGN_TRAIN_DENSE_H16"])
def test_split_bf16_backward_matches_f32(monkeypatch, switch):
    """The split-bf16 weight-gradient contractions (tsgemm_bf) against their f32-MFMA form, and the training
    Dense layers' split-fp16 row GEMMs (IGN_TRAIN_DENSE_H16, forward and backward) against their
    split-bf16 form: bitwise deterministic, and equal to fp32 reassociation (relative L2 <= 1e-5)
    on 24 synth50 graphs.  IGN_TRAIN_DENSE_BF=0 also puts the readout's first-layer input gradient
    (256 -> 32, on dense_bf since round 5) back on row_gemm_t's f32 MFMA."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "synth50", 24)
    prm = MPPlan.from_model_info(mi).init_params(13, bias_scale=0.1)
    monkeypatch.setenv(switch, "1")
    g1 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    g2 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    np.testing.assert_array_equal(g1, g2)
    monkeypatch.setenv(switch, "0")
    g0 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    assert not np.array_equal(g0, g1)   # the switch took effect
    assert np.linalg.norm(g1.astype(np.float64) - g0) <= 1e-5 * np.linalg.norm(g0)


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_output_layer_gradient_formed_on_the_fly(monkeypatch, kind):
    """The 1-unit output layer's backward rows (dz[r][k] = dz_out[r] w3[k] selu'(a2[r][k])) formed
    by the layer below's input-gradient kernel as it loads a2, and written over a2 for that layer's
    weight gradient (default), instead of by row_outer_t (IGN_FUSE_OUTER_BWD=0): the same
    arithmetic, bitwise-equal gradients, and within the tolerance of float64 autograd."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "nsfnet", 6)
    prm = MPPlan.from_model_info(mi).init_params(17, bias_scale=0.1)
    eng, _, _, _, _, g1 = _engine_grads(desc, dims, graphs, labels, prm)
    g1 = g1.cpu().numpy()
    monkeypatch.setenv("IGN_FUSE_OUTER_BWD", "0")
    g0 = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    np.testing.assert_array_equal(g1, g0)
    assert _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g1, eng.layout) <= GTOL


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_training_forward_fused_readout(monkeypatch, kind):
    """The training forward's readout on the inference kernel (readout_h16 writing both layers'
    activations, IGN_TRAIN_FUSED_READOUT, default on) against the per-layer row GEMMs: bitwise
    deterministic, the switch takes effect, and both within the tolerance of float64 autograd."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "nsfnet", 4)
    prm = MPPlan.from_model_info(mi).init_params(19, bias_scale=0.1)
    eng, _, p1, _, _, g1 = _engine_grads(desc, dims, graphs, labels, prm)
    g1 = g1.cpu().numpy()
    np.testing.assert_array_equal(g1, _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy())
    monkeypatch.setenv("IGN_TRAIN_FUSED_READOUT", "0")
    _, _, p0, _, _, g0 = _engine_grads(desc, dims, graphs, labels, prm)
    g0 = g0.cpu().numpy()
    assert not np.array_equal(g0, g1)
    np.testing.assert_allclose(p1, p0, rtol=1e-5, atol=1e-5)
    e1 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g1, eng.layout)
    e0 = _rel_err_vs_oracle(desc, dims, graphs, labels, prm, g0, eng.layout)
    print("vs float64 autograd: fused readout %.3g, per layer %.3g" % (e1, e0))
    assert e1 <= GTOL and e0 <= GTOL


def test_readout_bits_do_not_depend_on_the_row_tile():
    """A row's prediction is the same bits whichever rows share its 16-row tile: the synthetic graph
    alone and after an 8-node graph in the same batch (every row shifted by 8), for the training
    forward (readout_h16 with activation saves) and the inference forward.  (The SAVE form once
    lowered one tile's layer-2 multiply-add fused and the other's unfused; tools/probes/ro_save_probe.py.)"""
    desc, dims, _, graphs, _ = workloads.make_synthetic_inputs(n_nodes=2000, hidden=32, iterations=2, window=96)
    small = synthetic.synthetic_graph_arrays(n_nodes=8, window=4, graph_id=7)
    small.pop("target")
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(21, bias_scale=0.1))
    for train in (True, False):
        outs = []
        for gs in (graphs, [small] + graphs):
            b = Batch(eng, gs)
            if train:
                b.enable_training()
            outs.append((b.forward_train() if train else b.forward()).reshape(-1).copy())
            b.close()
        np.testing.assert_array_equal(outs[0], outs[1][8:])


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_pooled_buffers_reused_and_poisoned(monkeypatch, kind):
    """Batch and training buffers come from the plan's device-memory cache (devpool.cpp): a batch
    built after another was destroyed reuses its blocks.  With IGN_POOL_POISON=1 every scratch
    block starts as NaN, so predictions and gradients bitwise equal to those on uncached hipMalloc
    blocks (IGN_POOL=0) show that no kernel reads scratch it has not written, and that a reused
    block carries nothing over from the batch before (a smaller one in between)."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "synth50", 6)
    prm = MPPlan.from_model_info(mi).init_params(17, bias_scale=0.1)
    monkeypatch.setenv("IGN_POOL", "0")
    _, b0, p0, l0, _, g0 = _engine_grads(desc, dims, graphs, labels, prm)
    f0 = b0.forward()
    g0 = g0.cpu().numpy()
    b0.close()
    monkeypatch.setenv("IGN_POOL", "1")
    monkeypatch.setenv("IGN_POOL_POISON", "1")
    eng = Engine(MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims)), 0)
    eng.set_params(prm)
    for rep in range(3):
        gs, ls = (graphs, labels) if rep != 1 else (graphs[:2], labels[:2])
        _, b, pred, loss, _, g = _engine_grads(desc, dims, gs, ls, prm, eng=eng)
        fwd = b.forward()
        if rep != 1:
            np.testing.assert_array_equal(pred, p0)
            np.testing.assert_array_equal(fwd, f0)
            np.testing.assert_array_equal(g.cpu().numpy(), g0)
            assert loss == l0
        else:
            assert np.isfinite(pred).all() and np.isfinite(g.cpu().numpy()).all()
        b.close()
    # ign_plan_trim_cache hands every idle block back (batch destroy no longer waits on the
    # stream: the fences do); a batch built afterwards runs on fresh blocks, same bits
    eng.trim_cache()
    _, b, pred, loss, _, g = _engine_grads(desc, dims, graphs, labels, prm, eng=eng)
    np.testing.assert_array_equal(pred, p0)
    np.testing.assert_array_equal(g.cpu().numpy(), g0)
    b.close()
    eng.trim_cache()


@pytest.mark.parametrize("kind,topo,n", [("routenet", "synth50", 4), ("qsize", "geant2", 3), ("routenet", "nsfnet", 5)])
def test_gpu_transposed_csrs_equal_host(monkeypatch, kind, topo, n):
    """The training tables' transposed CSRs built on the GPU (train_csr.hip, a stable radix sort;
    the default) and on the host (IGN_TRAIN_CSR_GPU=0): the same gradients, bitwise -- the sort
    keeps every row's steps / destinations in the host's emission order.  Q-size: two source slots
    of its sum MP and an interleaved ordered MP."""
    desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, topo, n)
    prm = MPPlan.from_model_info(mi).init_params(17, bias_scale=0.1)
    g_gpu = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    monkeypatch.setenv("IGN_TRAIN_CSR_GPU", "0")
    g_host = _engine_grads(desc, dims, graphs, labels, prm)[5].cpu().numpy()
    assert np.abs(g_host).sum() > 0
    np.testing.assert_array_equal(g_gpu, g_host)
