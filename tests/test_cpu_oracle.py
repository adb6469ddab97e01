"""The C++/OpenMP restatement (oracle/cpu_forward.cpp) against the float64 dense oracle (CPU):
the models of the benchmark configurations and the concat / interleave variants, and the same
run-time errors (K.rnn mask width, gather_nd(-1)).  Its float64 mode (the checker of the
engine's full-size outputs) agrees to float32 output rounding; its float32 mode (bench.py's
second CPU line) within plain float32 error of this model (the float32 dense oracle itself is
up to ~2e-4 off float64 on outlier predictions of 64 synth50 graphs)."""
import copy

import numpy as np
import pytest

from ignnition_amd import model_examples, synthetic, workloads
from ignnition_amd.engine import MPPlan
from ignnition_amd.json_operations import Model_information
from oracle import cpu_oracle
from oracle.dense_forward import DenseOracle

TOL64 = 1e-6   # float64 restatement, float32 outputs
TOL32 = 5e-4   # float32 restatement (plain float32 arithmetic, see above)


@pytest.fixture(scope="module", autouse=True)
def _built():
    cpu_oracle.build()


def _close(got, ref, tol):
    err = np.abs(got.astype(np.float64) - ref) / np.maximum(1.0, np.abs(ref))
    assert got.shape == ref.shape and err.max() <= tol, err.max()


def _check(desc, dims, graphs, seed=2, threads=4):
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    prm = plan.init_params(seed, bias_scale=0.1)
    ref = DenseOracle(desc, dims, prm).forward(graphs)
    got64 = cpu_oracle.cpu_forward(plan, graphs, prm, threads, float64=True)
    got32 = cpu_oracle.cpu_forward(plan, graphs, prm, threads)
    assert np.all(np.isfinite(got32)) and np.all(np.isfinite(got64))
    _close(got64, ref, TOL64)
    _close(got32, ref, TOL32)


@pytest.mark.parametrize("kind,topo,n", [("routenet", "nsfnet", 3), ("qsize", "nsfnet", 2), ("routenet", "geant2", 2)])
def test_examples_match_dense_oracle(kind, topo, n):
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs(kind, topo, n)
    _check(desc, dims, graphs)


@pytest.mark.parametrize("threads", [1, 3])
def test_one_large_graph_parallel_over_destinations(threads):
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=2000, iterations=3, window=64)
    _check(desc, dims, graphs, threads=threads)


@pytest.mark.parametrize("axis", [1, 2])
def test_concat(axis):
    desc = model_examples.qsize_aggregation({"type": "concat", "concat_axis": axis}, iterations=3)
    _, dims, _ = workloads.model("qsize")
    mi = Model_information(copy.deepcopy(desc), dims)
    graphs, _ = workloads.graph_inputs(mi, [synthetic.routenet_sample("nsfnet", g, qsize=True) for g in range(2)])
    _check(desc, dims, graphs)


def test_batch_is_per_graph():
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "synth50", 6)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(1)
    whole = cpu_oracle.cpu_forward(plan, graphs, prm, 4)
    alone = np.concatenate([cpu_oracle.cpu_forward(plan, [g], prm, 1) for g in graphs])
    np.testing.assert_array_equal(whole, alone)


def test_errors_like_the_reference():
    from tests.test_oracle import QS_DIMS, narrow_mask_input
    desc = model_examples.qsize(hidden=16, iterations=2)
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), QS_DIMS))
    with pytest.raises(cpu_oracle.OracleError, match="sequence_mask"):
        cpu_oracle.cpu_forward(plan, [narrow_mask_input()], plan.init_params(0))
    desc = model_examples.routenet(hidden=16, iterations=2)
    dims = {"link_capacity": 1, "traffic": 1, "adj_links_paths": 0, "adj_paths_links": 0}
    x = {"link_capacity": [0.5, -0.3, 0.8], "traffic": [0.2, -0.4, 0.1],
         "src_adj_links_paths": [0, 1], "dst_adj_links_paths": [0, 1], "seq_link_path": [0, 0],
         "src_adj_paths_links": [0, 1, 0], "dst_adj_paths_links": [0, 1, 2], "seq_path_link": [0, 0, 0],
         "num_link": 3, "num_path": 3}
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    with pytest.raises(cpu_oracle.OracleError, match="no message"):
        cpu_oracle.cpu_forward(plan, [x], plan.init_params(0))


def test_saturated_gates_stay_finite():
    """Inputs large enough to saturate every gate and overflow an unclamped exp (the restatement is
    built with -ffast-math, which assumes finite values): still finite and equal to the float64
    oracle (sigmoid / tanh saturate to their limits in both)."""
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "nsfnet", 2)
    big = [dict(g, traffic=np.asarray(g["traffic"], np.float32) * 400.0,
                link_capacity=np.asarray(g["link_capacity"], np.float32) * 400.0) for g in graphs]
    _check(desc, dims, big, seed=5)
