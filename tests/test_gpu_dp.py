"""Data-parallel training step: two ranks (gloo, both on GPU 0), each on its own
batch; after ``Trainer.train_step`` both hold the average of the two single-rank gradients and
identical parameters (GM:790-818 + the gradient all-reduce of training.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from ignnition_amd import workloads
    from ignnition_amd.training import Trainer
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        desc, dims, mi, graphs, labels = workloads.make_batch_inputs("routenet", "nsfnet", 2, first_id=2 * rank)
        alone = Trainer(mi, seed=3)
        alone.train_step(graphs, labels)
        g_alone = alone.grads.cpu().numpy().copy()
        dp = Trainer(mi, seed=3, dist=dist)
        dp.train_step(graphs, labels)
        p = dp.params()
        out[rank] = (g_alone, dp.grads.cpu().numpy().copy(), {k: np.asarray(v) for k, v in p.items()})
    finally:
        dist.destroy_process_group()


def test_data_parallel_step_averages_gradients():
    from ignnition_amd.engine import device_count
    if device_count() == 0:
        pytest.fail("no GPU visible")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        mp.start_processes(_worker, args=(world, port, out), nprocs=world, join=True, start_method="spawn")
        res = dict(out)
    g0, g1 = res[0][0].astype(np.float64), res[1][0].astype(np.float64)
    avg = (g0 + g1) / 2
    assert not np.allclose(g0, g1)
    for r in range(world):
        np.testing.assert_allclose(res[r][1], avg, rtol=1e-5, atol=1e-7 * np.abs(avg).max())
    np.testing.assert_array_equal(res[0][1], res[1][1])
    for k in res[0][2]:
        np.testing.assert_array_equal(res[0][2][k], res[1][2][k])


def _edge_cut_train_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import copy as _copy

    import torch
    import torch.distributed as dist
    from ignnition_amd import partition, workloads
    from ignnition_amd.engine import Engine, MPPlan
    from ignnition_amd.json_operations import Model_information
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        desc, dims, _, graphs, labels = workloads.make_synthetic_inputs(n_nodes=2000, hidden=32, iterations=2,
                                                                       window=96)
        plan = MPPlan.from_model_info(Model_information(_copy.deepcopy(desc), dims))
        eng = Engine(plan, 0)
        eng.set_params(plan.init_params(21, bias_scale=0.1))
        comm = partition.TorchComm(dist, None, host_staged=True)
        part = partition.local_part(graphs[0], plan, rank, world)
        partition.exchange_requests([part], comm)
        r = part.ranges["node"]
        lab = np.asarray(labels[0], np.float32).reshape(-1)[r[rank]:r[rank + 1]]
        tr = partition.EdgeCutTraining(eng, [part], comm)
        loss, g, preds = tr.step([lab])
        torch.cuda.synchronize()
        out[rank] = (loss, g.cpu().numpy(), preds[0].reshape(-1))
        tr.close()
    finally:
        dist.destroy_process_group()


def test_edge_cut_training_two_processes():
    """partition.EdgeCutTraining under torch.distributed (2 ranks, gloo host-staged, both on GPU 0,
    the TorchComm path the RCCL run takes): both ranks hold the same summed gradient, equal to the
    whole graph's step on one engine."""
    import copy as _copy

    import torch
    from ignnition_amd import workloads
    from ignnition_amd.engine import Batch, Engine, MPPlan, device_count
    from ignnition_amd.json_operations import Model_information
    if device_count() == 0:
        pytest.fail("no GPU visible")
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    with ctx.Manager() as m:
        out = m.dict()
        mp.start_processes(_edge_cut_train_worker, args=(world, port, out), nprocs=world, join=True,
                           start_method="spawn")
        res = dict(out)
    desc, dims, _, graphs, labels = workloads.make_synthetic_inputs(n_nodes=2000, hidden=32, iterations=2, window=96)
    plan = MPPlan.from_model_info(Model_information(_copy.deepcopy(desc), dims))
    eng = Engine(plan, 0)
    eng.set_params(plan.init_params(21, bias_scale=0.1))
    b = Batch(eng, graphs)
    b.enable_training()
    pred = b.forward_train().reshape(-1)
    y = torch.from_numpy(np.asarray(labels[0], np.float32).reshape(-1)).cuda()
    d = torch.empty_like(y)
    loss = eng.mse_loss(b.predictions_ptr(), y, d)
    g = torch.zeros(eng.n_params, dtype=torch.float32, device="cuda")
    b.backward(d, g)
    torch.cuda.synchronize()
    gw = g.cpu().numpy().astype(np.float64)
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(np.concatenate([res[0][2], res[1][2]]), pred)
    for r in range(world):
        assert res[r][0] == pytest.approx(loss, rel=1e-6)
        assert np.linalg.norm(res[r][1] - gw) <= 1e-5 * np.linalg.norm(gw)
