"""N>1 path on CPU (gloo, world_size 2): graph sharding and the step-statistics reduction used
by bench.py.  No GPU involved: each rank builds its shard's index arrays on the host."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ignnition_amd import workloads


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per_rank, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = workloads.shard_graph_ids(rank, world, per_rank)
        desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "nsfnet", len(ids), first_id=ids[0])
        edges = workloads.edges_per_forward(mi, graphs)
        elapsed = 0.5 + rank          # rank-dependent fake timing
        t, e = workloads.reduce_step_stats(dist, elapsed, edges)
        all_ids = [None] * world
        dist.all_gather_object(all_ids, ids)
        out[rank] = (t, e, edges, all_ids)
    finally:
        dist.destroy_process_group()


def test_graph_sharding_gloo_world2():
    world, per_rank = 2, 3
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, per_rank, out), nprocs=world, join=True)
        res = dict(out)
    desc, dims, mi, graphs, _ = workloads.make_batch_inputs("routenet", "nsfnet", world * per_rank)
    total = workloads.edges_per_forward(mi, graphs)
    for r in range(world):
        t, e, local, all_ids = res[r]
        assert t == pytest.approx(0.5 + (world - 1))        # MAX over ranks
        assert e == total                                  # SUM of shard edges == whole batch
        flat = [i for ids in all_ids for i in ids]
        assert sorted(flat) == list(range(world * per_rank)) and len(set(flat)) == len(flat)


def test_shard_bounds():
    assert workloads.shard_graph_ids(1, 4, 512) == list(range(512, 1024))
    with pytest.raises(ValueError):
        workloads.shard_graph_ids(4, 4, 1)
