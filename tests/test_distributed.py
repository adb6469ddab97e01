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


# ---------------------------------------------------------------------------------------------
# Edge-cut partitions of one graph: partition + request all-to-all + halo exchange.
import numpy as np

from ignnition_amd import partition
from ignnition_amd.engine import MPPlan

N_SMALL = 3000


def _synthetic_plan_and_inputs(n=N_SMALL):
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=n, iterations=2, window=64)
    return MPPlan.from_model_info(mi), graphs[0]


def _state_value(gid, H):
    """Row content a rank holds for global node id gid: distinct per id and column."""
    return np.asarray(gid, np.float32)[..., None] * 100.0 + np.arange(H, dtype=np.float32)


def _check_halo_exchange(parts, comm, H=8):
    partition.exchange_requests(parts, comm)
    sends, recvs, sc, rc, states = [], [], [], [], []
    for p in parts:
        h = p.halos["node"]
        lo = p.ranges["node"][p.rank]
        state = torch.zeros((h.n_owned + h.n_halo, H))
        state[:h.n_owned] = torch.from_numpy(_state_value(np.arange(lo, lo + h.n_owned), H))
        sends.append(state[torch.from_numpy(h.send_rows.astype(np.int64))])
        recvs.append(state[h.n_owned:])
        sc.append(h.send_counts)
        rc.append(h.recv_counts)
        states.append(state)
    comm.exchange(sends, sc, recvs, rc, async_op=False).wait()
    for p, state in zip(parts, states):
        h = p.halos["node"]
        np.testing.assert_array_equal(state[h.n_owned:].numpy(), _state_value(h.halo_ids, H))
    return states


def _check_partition_edges(parts, x):
    """The partitions' in-edges, mapped back to global ids, are the whole graph, each destination's
    in-edges in their original order (so message sums associate identically)."""
    s_all, d_all = [], []
    for p in parts:
        h = p.halos["node"]
        lo = p.ranges["node"][p.rank]
        s = p.inputs["src_adj_nodes_nodes"]
        glob = s + lo
        if h.n_halo:
            glob = np.where(s < h.n_owned, s + lo, h.halo_ids[np.clip(s - h.n_owned, 0, h.n_halo - 1)])
        s_all.append(glob)
        d_all.append(p.inputs["dst_adj_nodes_nodes"] + lo)
        assert p.inputs["num_node"] == h.n_owned
    s_all, d_all = np.concatenate(s_all), np.concatenate(d_all)
    order = np.argsort(x["dst_adj_nodes_nodes"], kind="stable")
    order2 = np.argsort(d_all, kind="stable")
    np.testing.assert_array_equal(d_all[order2], x["dst_adj_nodes_nodes"][order])
    np.testing.assert_array_equal(s_all[order2], x["src_adj_nodes_nodes"][order])


@pytest.mark.parametrize("world", [1, 2, 3])
def test_edge_cut_loopback(world):
    plan, x = _synthetic_plan_and_inputs()
    parts = [partition.local_part(x, plan, r, world) for r in range(world)]
    _check_halo_exchange(parts, partition.LoopbackComm(world))
    _check_partition_edges(parts, x)
    if world > 1:
        assert all(p.halos["node"].n_halo > 0 for p in parts)


def test_edge_cut_rejects_ordered():
    desc, dims, mi = workloads.model("routenet")
    plan = MPPlan.from_model_info(mi)
    with pytest.raises(ValueError):
        partition.local_part({}, plan, 0, 2)


def _edge_cut_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan, x = _synthetic_plan_and_inputs()
        part = partition.local_part(x, plan, rank, world)
        states = _check_halo_exchange([part], partition.TorchComm(dist))
        h = part.halos["node"]
        out[rank] = (h.n_owned, h.n_halo, list(h.send_counts), list(h.recv_counts), float(states[0].sum()))
    finally:
        dist.destroy_process_group()


def test_edge_cut_gloo_world2():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_edge_cut_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    plan, x = _synthetic_plan_and_inputs()
    parts = [partition.local_part(x, plan, r, world) for r in range(world)]
    partition.exchange_requests(parts, partition.LoopbackComm(world))
    for r in range(world):
        n_owned, n_halo, sc, rc, _ = res[r]
        h = parts[r].halos["node"]
        assert (n_owned, n_halo, sc, rc) == (h.n_owned, h.n_halo, h.send_counts, h.recv_counts)
        # what r sends to q is what q receives from r
        assert sc[1 - r] == res[1 - r][3][r]


def test_edge_cut_carries_edge_parameters():
    """A partition keeps the per-edge parameters (params_<adj>, GEN:156-163) of the in-edges it
    keeps, in their original order (message networks reading edge_params)."""
    from ignnition_amd.engine import MPPlan as _P
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=400, hidden=32, iterations=2, window=16)
    plan = _P.from_model_info(mi)
    x = dict(graphs[0])
    E = len(x["src_adj_nodes_nodes"])
    x["params_adj_nodes_nodes"] = np.arange(2 * E, dtype=np.float32).reshape(E, 2)
    world = 3
    kept = []
    for r in range(world):
        p = partition.local_part(x, plan, r, world)
        prm = p.inputs["params_adj_nodes_nodes"]
        assert prm.shape == (len(p.inputs["src_adj_nodes_nodes"]), 2)
        kept.append(prm[:, 0] / 2)
    ids = np.concatenate(kept).astype(np.int64)
    assert sorted(ids.tolist()) == list(range(E))   # every edge exactly once
    for k in kept:
        assert np.all(np.diff(k) > 0)                # original order within a partition


def _bench(args, env_extra=None, timeout=300):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=repo)
    lines = []
    for ln in r.stdout.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            lines.append(json.loads(ln))
    return r, lines


def test_bench_gpus_n_launches_n_ranks():
    """The driver runs `python bench.py --gpus N` without a launcher: bench.py must start N ranks
    itself (torch.distributed.run as a child process) and print exactly one line, from rank 0,
    with n_gpus N and the edges of every rank's shard summed."""
    r, lines = _bench(["--gpus", "2", "--dry-run", "--topology", "nsfnet", "--graphs", "2", "--steps", "3",
                       "--warmup", "1", "--edge-cut-nodes", "20000"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["scaling"] == "weak"
    _, _, mi, graphs, _ = workloads.make_batch_inputs("routenet", "nsfnet", 4)
    assert line["config"]["edges_per_step_total"] == workloads.edges_per_forward(mi, graphs)
    # the edge-cut leg (BASELINE configs[4]) in the same ranks: the two partitions' in-edges add up to
    # the whole graph's, and every halo row a rank reads is sent by exactly one owner
    ec = line["edge_cut_20000n"]
    _, _, smi, sgraphs, _ = workloads.make_synthetic_inputs(n_nodes=20000)
    whole = workloads.edges_per_forward(smi, sgraphs)
    assert ec["n_ranks"] == 2 and ec["edges_per_step"] == whole == ec["edges_per_step_whole_graph"]
    assert ec["edges_match_whole_graph"] and ec["halo_rows"]["total"] == ec["send_rows_total"] > 0
    # --no-edge-cut drops the leg
    r, lines = _bench(["--gpus", "2", "--dry-run", "--topology", "nsfnet", "--graphs", "2", "--steps", "1",
                       "--no-edge-cut"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1 and not any(k.startswith("edge_cut") for k in lines[0])


@pytest.mark.parametrize("n", [4, 8])
def test_bench_gpus_n_dry_run_partition_and_halo_symmetry(n):
    """`bench.py --gpus N --dry-run` for the driver's N = 4 and N = 8: N
    ranks, one line; the graph-sharded RouteNet edges of all N shards; the edge-cut leg's N
    partitions add up to the whole graph's in-edges, and the halo exchange is symmetric per rank
    pair (rows rank i reads from rank j = rows j sends to i), with no rank reading its own rows."""
    r, lines = _bench(["--gpus", str(n), "--dry-run", "--topology", "nsfnet", "--graphs", "2", "--steps", "2",
                       "--warmup", "1", "--edge-cut-nodes", "20000"], timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == n
    _, _, mi, graphs, _ = workloads.make_batch_inputs("routenet", "nsfnet", 2 * n)
    assert line["config"]["edges_per_step_total"] == workloads.edges_per_forward(mi, graphs)
    ec = line["edge_cut_20000n"]
    assert ec["n_ranks"] == n and ec["edges_match_whole_graph"]
    assert ec["halo_symmetric"], (ec["halo_recv_by_pair"], ec["halo_send_by_pair"])
    recv = np.asarray(ec["halo_recv_by_pair"])
    assert recv.shape == (n, n) and np.all(np.diag(recv) == 0) and recv.sum() == ec["halo_rows"]["total"] > 0
    assert (recv > 0).sum() >= n * (n - 1) // 2   # the 10 % uniform sources reach beyond the neighbouring ranges


def test_bench_single_rank_dry_run_and_world_mismatch():
    r, lines = _bench(["--dry-run", "--topology", "nsfnet", "--graphs", "2", "--steps", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 1
    # launched by torchrun with a world that differs from --gpus: refuse instead of mislabeling
    r, lines = _bench(["--gpus", "4", "--dry-run", "--topology", "nsfnet", "--graphs", "2"],
                      {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and not lines
    assert "WORLD_SIZE" in r.stderr
