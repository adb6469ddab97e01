"""BASELINE.json's two headline workloads at their stated sizes (MI355X only).

configs[4] — the synthetic 1M-node / 10M-edge graph, H=64, T=8:
  * the whole graph on one GPU: finite, and bitwise deterministic run to run; all 1M predictions
    against the C++/OpenMP restatement in float64 (oracle/cpu_forward.cpp, itself checked against
    the float64 dense oracle in tests/test_cpu_oracle.py);
  * the 8-way edge-cut the driver's 8-GPU bench runs (contiguous id ranges, halo rows,
    interior/boundary overlap), all 8 partitions in this process over LoopbackComm: the
    concatenated predictions equal the whole-graph run bit for bit (each destination keeps its
    in-edges in order, so every sum associates identically);
  * the oracle on a 25 000-node instance of the same generator (same degree law and locality),
    at the full model size (H=64, T=8), within the §8c tolerance.

configs[2] — RouteNet on 512 synth50-size graphs batched into one CSR (the default bench):
  * deterministic; three graphs of the batch equal the same graph run alone (GM:712-724: the
    reference runs the model per graph); two graphs against the float64 oracle.

Full-batch precision (configs[1]-[3] at 512 graphs: RouteNet synth50, Q-size synth50, RouteNet
GEANT2): every prediction of the engine's default contractions against the float64 C++
restatement, held to plain IEEE float32 arithmetic of the same model (the restatement built
without -ffast-math: libm expf / tanhf) -- DESIGN §4 has the table, including the split-bf16 x6
and f32-MFMA variants this test also records.

Tolerance: |engine - oracle| <= 1e-4 * max(1, |oracle|).
"""
import copy

import numpy as np
import pytest
import torch

from ignnition_amd import partition, workloads
from ignnition_amd.engine import Batch, Engine, MPPlan, device_count
from ignnition_amd.json_operations import Model_information
from oracle import cpu_oracle
from oracle.dense_forward import DenseOracle

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _scaled(got, exp):
    got = np.asarray(got, np.float64).reshape(-1)
    exp = np.asarray(exp, np.float64).reshape(-1)
    assert got.shape == exp.shape
    return np.abs(got - exp) / np.maximum(1.0, np.abs(exp))


def _scaled_err(got, exp):
    got = np.asarray(got, np.float64).reshape(-1)
    exp = np.asarray(exp, np.float64).reshape(-1)
    assert got.shape == exp.shape
    return float((np.abs(got - exp) / np.maximum(1.0, np.abs(exp))).max())


@pytest.fixture(scope="module")
def big_graph():
    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=1_000_000)
    x = graphs[0]
    assert int(x["num_node"]) == 1_000_000
    assert 9_500_000 <= len(x["src_adj_nodes_nodes"]) <= 10_500_000
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    assert plan.hidden[0] == 64 and plan.iterations == 8
    prm = plan.init_params(3, bias_scale=0.1)
    eng = Engine(plan, 0)
    eng.set_params(prm)
    whole = Batch(eng, graphs)
    out = whole.forward().reshape(-1)
    edges = whole.edges_per_forward
    out2 = whole.forward().reshape(-1)
    whole.close()
    yield x, plan, eng, out, out2, edges, prm
    eng.close()


def test_1m_whole_graph_finite_and_deterministic(big_graph):
    x, plan, eng, out, out2, edges, _ = big_graph
    assert out.size == 1_000_000
    assert np.all(np.isfinite(out))
    assert edges == 8 * len(x["src_adj_nodes_nodes"])
    np.testing.assert_array_equal(out, out2)


def test_1m_eight_partition_edge_cut_bit_identical(big_graph):
    """The 8-rank layout of `bench.py --model synthetic --gpus 8`, in one process."""
    x, plan, eng, out, _, edges, _ = big_graph
    world = 8
    parts = [partition.local_part(x, plan, r, world) for r in range(world)]
    comm = partition.LoopbackComm(world)
    partition.exchange_requests(parts, comm)
    halo = [p.halos["node"].n_halo for p in parts]
    assert all(h > 0 for h in halo)
    fw = partition.EdgeCutForward(eng, parts, comm, overlap=True)
    try:
        assert fw.edges_per_forward == edges
        splits = [b.mp_split(0) for b in fw.batches]
        assert all(i > 0 and bd > 0 for i, bd in splits)
        got = np.concatenate([o.reshape(-1) for o in fw.forward()])
        np.testing.assert_array_equal(got, out)
    finally:
        fw.close()
        torch.cuda.synchronize()


def test_1m_whole_graph_matches_cpu_restatement(big_graph):
    """Every one of the 1M predictions (H=64, T=8, 10M edges) against the C++ restatement
    (float64, the box's CPU share)."""
    x, plan, eng, out, _, _, prm = big_graph
    ref = cpu_oracle.cpu_forward(plan, [x], prm, 0, float64=True)
    err = _scaled_err(out, ref)
    print("1M synthetic vs C++ restatement: max scaled error %.3g" % err)
    assert err <= TOL


def test_synthetic_full_model_25k_matches_oracle():
    """H=64, T=8 and the default generator settings, 25k nodes / ~250k edges."""
    if device_count() == 0:
        pytest.fail("no GPU visible")
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=25_000)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(4, bias_scale=0.1)
    eng = Engine(plan, 0)
    eng.set_params(prm)
    b = Batch(eng, graphs)
    out = b.forward().reshape(-1)
    b.close()
    eng.close()
    ref = DenseOracle(desc, dims, prm).forward(graphs)
    err = _scaled_err(out, ref)
    print("25k synthetic, H=64 T=8: max scaled error %.3g" % err)
    assert err <= TOL


def test_routenet_512_synth50_batch():
    if device_count() == 0:
        pytest.fail("no GPU visible")
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "synth50", 512)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(1, bias_scale=0.05)
    eng = Engine(plan, 0)
    eng.set_params(prm)
    b = Batch(eng, graphs)
    assert b.edges_per_forward == workloads.edges_per_forward(mi, graphs)
    o1 = b.forward().reshape(-1)
    o2 = b.forward().reshape(-1)
    b.close()
    np.testing.assert_array_equal(o1, o2)
    assert np.all(np.isfinite(o1))
    P = [int(g["num_path"]) for g in graphs]
    off = np.cumsum([0] + P)
    assert o1.size == off[-1]
    for gi in (0, 255, 511):
        alone = Batch(eng, [graphs[gi]])
        np.testing.assert_array_equal(o1[off[gi]:off[gi + 1]], alone.forward().reshape(-1))
        alone.close()
    ora = DenseOracle(desc, dims, prm)
    for gi in (7, 400):
        err = _scaled_err(o1[off[gi]:off[gi + 1]], ora.forward([graphs[gi]]))
        assert err <= TOL, (gi, err)
    eng.close()


IEEE_VARIANTS = {"default": {}, "bf16x6": {"IGN_SEQ_VARIANT": "4", "IGN_READOUT_VARIANT": "2", "IGN_SUM_VARIANT": "7"},
                 "f32mfma": {"IGN_SEQ_VARIANT": "2", "IGN_READOUT_VARIANT": "1", "IGN_SUM_VARIANT": "3"}}


def _tails(e):
    return {"max": float(e.max()), "p9999": float(np.quantile(e, 0.9999)), "mean": float(e.mean())}


@pytest.mark.parametrize("model,topology", [("routenet", "synth50"), ("qsize", "synth50"), ("routenet", "geant2")])
def test_full_batch_precision_vs_ieee_float32(monkeypatch, model, topology):
    """512 graphs: the default's 99.99th percentile and mean within 1.25x of IEEE float32's, its
    maximum within 1.5x.  Why not 1.25x for the maximum: the worst of 1.25 M predictions after
    8 GRU iterations is one chaotic outlier, and float32 evaluations of EQUAL accuracy move it by
    ~1.3x (libm tanhf vs a 1.2-ulp polynomial: 1.74e-4 vs 1.97e-4 on RouteNet synth50;
    tools/probes/gate_precision_emulation.py), while the 99.99th percentile moves by < 10 %.
    Measured round 3 (max / p99.99 vs IEEE): RouteNet synth50 1.25x / 1.22x, Q-size 1.11x / 1.19x,
    GEANT2 1.10x / 0.75x.  The round-2 kernels' exp-form tanh gave 1.84x / 2.42x on RouteNet."""
    if device_count() == 0:
        pytest.fail("no GPU visible")
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs(model, topology, 512)
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(1, bias_scale=0.05)
    ref = cpu_oracle.cpu_forward(plan, graphs, prm, 0, float64=True)
    res = {"ieee_f32": _tails(_scaled(cpu_oracle.cpu_forward(plan, graphs, prm, 0, ieee=True), ref))}
    for name, env in IEEE_VARIANTS.items():
        for k in ("IGN_SEQ_VARIANT", "IGN_READOUT_VARIANT", "IGN_SUM_VARIANT"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        eng = Engine(plan, 0)
        eng.set_params(prm)
        b = Batch(eng, graphs)
        out = b.forward().reshape(-1)
        b.close()
        eng.close()
        assert np.all(np.isfinite(out))
        res[name] = _tails(_scaled(out, ref))
    print("%s_%s_x512 vs float64:" % (model, topology),
          "; ".join("%s max %.3g p99.99 %.3g mean %.3g" % (k, v["max"], v["p9999"], v["mean"]) for k, v in res.items()))
    d, y = res["default"], res["ieee_f32"]
    assert d["p9999"] <= 1.25 * y["p9999"], res
    assert d["mean"] <= 1.25 * y["mean"], res
    assert d["max"] <= 1.5 * y["max"], res
