"""The training oracle (oracle/train_oracle.py, torch autograd in float64) on CPU: its forward
is the dense oracle's, its gradients agree with finite differences, and the optimizer / metric
restatements follow the published Keras formulas."""
import copy

import numpy as np
import pytest
import torch

from ignnition_amd import model_examples, synthetic, workloads
from ignnition_amd.engine import MPPlan
from ignnition_amd.json_operations import Model_information
from oracle.dense_forward import DenseOracle, l2_regularization
from oracle.train_oracle import TorchOracle, adam_step, eval_metrics, exponential_decay


def _setup(kind, n=1, hidden=None, iterations=None):
    if hidden or iterations:
        desc = model_examples.routenet(hidden=hidden or 32, iterations=iterations or 8)
        _, dims, _ = workloads.model(kind)
        mi = Model_information(copy.deepcopy(desc), dims)
        graphs, labels = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g) for g in range(n)])
    else:
        desc, dims, mi, graphs, labels = workloads.make_batch_inputs(kind, "nsfnet", n)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(3, bias_scale=0.1)
    return desc, dims, graphs, labels, prm


@pytest.mark.parametrize("kind", ["routenet", "qsize"])
def test_torch_forward_matches_dense_oracle(kind):
    desc, dims, graphs, labels, prm = _setup(kind, 2)
    got = TorchOracle(desc, dims, prm).forward(graphs).detach().numpy()
    exp = DenseOracle(desc, dims, prm).forward(graphs)
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("inputs", [("hs_source", "hs_dest"), ("hs_dest", "hs_source", "edge_params")])
def test_torch_forward_message_network_matches_dense_oracle(inputs):
    from ignnition_amd.framework_operations import dimensions_of_sample
    rng = np.random.default_rng(1)
    desc = model_examples.routenet_message_net(inputs=inputs, units=(24, 32), activation="selu", iterations=3)
    samples = [synthetic.routenet_sample("nsfnet", g) for g in range(2)]
    if "edge_params" in inputs:
        for s in samples:
            s["adj_paths_links"] = {l: [[p, [float(rng.uniform(0, 1)), float(rng.uniform(-1, 1))]] for p in ps]
                                    for l, ps in s["adj_paths_links"].items()}
    dims = dimensions_of_sample(samples[0])
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, samples)
    prm = MPPlan.from_model_info(mi).init_params(2, bias_scale=0.1)
    got = TorchOracle(desc, dims, prm).forward(graphs).detach().numpy()
    exp = DenseOracle(desc, dims, prm).forward(graphs)
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("aggr", [{"type": "convolution"}, {"type": "convolution", "activation_function": "tanh"},
                                  {"type": "attention"}])
def test_torch_forward_convolution_matches_dense_oracle(aggr):
    desc = model_examples.routenet_aggregation(aggr, hidden=32, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    got = TorchOracle(desc, dims, prm).forward(graphs).detach().numpy()
    exp = DenseOracle(desc, dims, prm).forward(graphs)
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("aggr", [{"type": "concat", "concat_axis": 2}, {"type": "attention"}])
def test_torch_forward_qsize_aggregations_match_dense_oracle(aggr):
    desc = model_examples.qsize_aggregation(aggr, iterations=3)
    _, dims, _ = workloads.model("qsize")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g, qsize=True) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    got = TorchOracle(desc, dims, prm).forward(graphs).detach().numpy()
    exp = DenseOracle(desc, dims, prm).forward(graphs)
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12)


def test_regularization_matches():
    desc, dims, graphs, labels, prm = _setup("routenet")
    reg = float(TorchOracle(desc, dims, prm).regularization().detach())
    assert reg == pytest.approx(l2_regularization(desc, prm), rel=1e-12)
    assert reg > 0


def test_gradients_match_finite_differences():
    desc, dims, graphs, labels, prm = _setup("routenet", 1, hidden=16, iterations=2)
    ora = TorchOracle(desc, dims, prm)
    loss, reg, grads, _ = ora.loss_and_grads(graphs, labels)
    rng = np.random.default_rng(0)
    for name in ["path_update/recurrent_kernel", "link_update/kernel", "path_update/bias",
                 "readout_model_0/" + desc["neural_networks"][0]["nn_architecture"][0]["name"] + "/kernel"]:
        p0 = {k: np.asarray(v, np.float64).copy() for k, v in prm.items()}
        idx = tuple(rng.integers(0, s) for s in p0[name].shape)
        eps = 1e-6
        vals = []
        for sgn in (1, -1):
            p = copy.deepcopy(p0)
            p[name][idx] += sgn * eps
            l, r, _, _ = TorchOracle(desc, dims, p).loss_and_grads(graphs, labels)
            vals.append(l + r)
        fd = (vals[0] - vals[1]) / (2 * eps)
        assert fd == pytest.approx(grads[name][idx], rel=1e-5, abs=1e-9), name


def test_adam_and_decay_formulas():
    assert exponential_decay(0, 0.001, 80000, 0.6) == pytest.approx(0.001)
    assert exponential_decay(40000, 0.001, 80000, 0.6) == pytest.approx(0.001 * 0.6 ** 0.5)
    assert exponential_decay(100000, 0.001, 82000, 0.8, staircase="True") == pytest.approx(0.001 * 0.8)
    p = {"w": np.array([1.0, -2.0])}
    m = {"w": np.zeros(2)}
    v = {"w": np.zeros(2)}
    g = np.array([0.5, -0.25])
    adam_step(p, {"w": g}, m, v, 0, 0.1)
    # first step (t = 1): m = 0.1 g, v = 0.001 g^2, lr_t = lr sqrt(1 - 0.999) / (1 - 0.9)
    lr_t = 0.1 * np.sqrt(0.001) / 0.1
    exp = np.array([1.0, -2.0]) - lr_t * (0.1 * g) / (np.sqrt(0.001 * g * g) + 1e-7)
    np.testing.assert_allclose(p["w"], exp, rtol=1e-12)
    np.testing.assert_allclose(m["w"], 0.1 * g)
    np.testing.assert_allclose(v["w"], 0.001 * g * g)


def test_eval_metrics():
    m = eval_metrics([1.0, 2.0, 4.0], [1.5, 2.0, 3.0])
    assert m["mae"] == pytest.approx(0.5)
    assert m["mre"] == pytest.approx((0.5 + 0 + 0.25) / 3)
    assert m["r-squared"] == pytest.approx(1 - 1.25 / (((np.array([1, 2, 4]) - 7 / 3) ** 2).sum()))


@pytest.mark.parametrize("case", ["pool_sum", "pool_max", "nn_pool_product", "product_width1", "extend_nn",
                                  "extend_pool", "shadow_entity_name"])
def test_torch_forward_readout_operations_match_dense_oracle(case):
    from tests.readout_cases import READOUT_CASES
    ops, pin, nets = READOUT_CASES[case]
    desc = model_examples.routenet_readout(ops, pin, nets, iterations=3)
    _, dims, _ = workloads.model("routenet")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g) for g in range(2)])
    prm = MPPlan.from_model_info(mi).init_params(4, bias_scale=0.1)
    got = TorchOracle(desc, dims, prm).forward(graphs).detach().numpy()
    exp = DenseOracle(desc, dims, prm).forward(graphs)
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12)

