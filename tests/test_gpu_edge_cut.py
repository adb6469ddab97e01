"""Edge-cut partitions on the GPU, all partitions in one process on one device
(LoopbackComm stands in for RCCL; the engine side — halo rows, stepped forward, interior /
boundary launches, HIP halo pack — is the same as under torchrun).

Expected: the concatenated partition predictions equal the unpartitioned engine's bit for bit
(each destination keeps its in-edges in order, so every sum associates identically), and the
oracle's within the §8c tolerance."""
import copy

import numpy as np
import pytest
import torch

from ignnition_amd import partition, workloads
from ignnition_amd.engine import Batch, Engine, MPPlan, device_count
from ignnition_amd.json_operations import Model_information
from oracle.dense_forward import DenseOracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def setup():
    if device_count() == 0:
        pytest.fail("no GPU visible: the gpu tests must run on the MI355X box")
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=6000, iterations=3, window=96)
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    prm = plan.init_params(5, bias_scale=0.1)
    eng = Engine(plan, 0)
    eng.set_params(prm)
    whole = Batch(eng, graphs)
    ref = whole.forward().reshape(-1)
    whole.close()
    return desc, dims, graphs[0], plan, prm, eng, ref


@pytest.mark.parametrize("world,overlap", [(1, True), (2, True), (2, False), (3, True), (4, True)])
def test_partitioned_equals_whole(setup, world, overlap):
    desc, dims, x, plan, prm, eng, ref = setup
    parts = [partition.local_part(x, plan, r, world) for r in range(world)]
    comm = partition.LoopbackComm(world)
    partition.exchange_requests(parts, comm)
    fw = partition.EdgeCutForward(eng, parts, comm, overlap=overlap)
    try:
        outs = fw.forward()
        got = np.concatenate([o.reshape(-1) for o in outs])
        np.testing.assert_array_equal(got, ref)
        assert fw.edges_per_forward == 3 * len(x["src_adj_nodes_nodes"])
        if world > 1:
            splits = [b.mp_split(0) for b in fw.batches]
            assert all(i > 0 and bd > 0 for i, bd in splits)
        # a second forward on the same partitions (buffers and halo state reused) is identical
        got2 = np.concatenate([o.reshape(-1) for o in fw.forward()])
        np.testing.assert_array_equal(got2, ref)
    finally:
        fw.close()
        torch.cuda.synchronize()


def test_partitioned_matches_oracle(setup):
    desc, dims, x, plan, prm, eng, ref = setup
    exp = DenseOracle(desc, dims, prm).forward([x]).reshape(-1)
    err = np.abs(ref.astype(np.float64) - exp) / np.maximum(1.0, np.abs(exp))
    assert err.max() <= 1e-4


def test_gather_rows(setup):
    eng = setup[5]
    src = torch.randn(1000, 64, device="cuda")
    idx = torch.randint(0, 1000, (777,), dtype=torch.int32, device="cuda")
    dst = torch.empty(777, 64, device="cuda")
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.gather_rows(src, idx, dst)
    torch.cuda.synchronize()
    assert torch.equal(dst, src[idx.long()])
