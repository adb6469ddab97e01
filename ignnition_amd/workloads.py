"""Synthetic workloads for tests and bench: samples -> GEN index dicts -> normalised inputs.

The normalisation functions restate the examples' ``main.py`` (RNM:26-38, QSM:27-39) on
numpy (the reference's use ``tf.math.log``).
"""

from __future__ import annotations

import numpy as np

from . import model_examples, synthetic
from .framework_operations import dimensions_of_sample
from .generator import sample_to_data
from .json_operations import Model_information


def normalization_routenet(feature, feature_name):
    """RNM:26-31."""
    if feature_name == "traffic":
        feature = (feature - 170) / 130
    if feature_name == "link_capacity":
        feature = (feature - 25000) / 40000
    return feature


def normalization_queue_size(feature, feature_name):
    """QSM:27-39 / MAIN:26-38."""
    if feature_name == "delay":
        feature = (np.log(feature) + 1.78) / 0.93
    if feature_name == "traffic":
        feature = (feature - 0.28) / 0.15
    if feature_name == "jitter":
        feature = (feature - 1.5) / 1.5
    if feature_name == "link_capacity":
        feature = (feature - 27.0) / 14.86
    if feature_name == "queue_sizes":
        feature = (feature - 16.5) / 15.5
    return feature


def log(feature, feature_name):
    return np.log(feature)


def exp(feature, feature_name):
    return np.exp(feature)


USER_FUNCTIONS = {"normalization_routenet": normalization_routenet,
                  "normalization_queue_size": normalization_queue_size, "log": log, "exp": exp}


def model(kind: str):
    """(description dict, Model_information) for 'routenet' or 'qsize'."""
    desc = model_examples.routenet() if kind == "routenet" else model_examples.qsize()
    sample = synthetic.routenet_sample("nsfnet", 0, qsize=(kind == "qsize"))
    dims = dimensions_of_sample(sample)
    return desc, dims, Model_information(desc, dims)


def graph_inputs(mi, samples, normalize: bool = True):
    """GEN + normalisation (GM:46-86) for a list of samples -> (inputs, labels)."""
    feature_list = mi.get_all_features()
    names = [f.name for f in feature_list]
    out_name, out_norm, _ = mi.get_output_info()
    graphs, labels = [], []
    for s in samples:
        data, y = sample_to_data(s, names, out_name, mi.get_adjecency_info(), mi.get_interleave_tensors(), [], True)
        if normalize:
            for f in feature_list:
                if str(f.normalization) != "None":
                    data[f.name] = USER_FUNCTIONS[f.normalization](np.asarray(data[f.name], np.float32), f.name)
            if out_norm is not None and str(out_norm) != "None":
                y = USER_FUNCTIONS[out_norm](np.asarray(y, np.float32), out_name)
        graphs.append(data)
        labels.append(np.asarray(y, np.float32))
    return graphs, labels


def make_batch_inputs(kind: str, topology: str, n_graphs: int, first_id: int = 0):
    desc, dims, mi = model(kind)
    samples = [synthetic.routenet_sample(topology, first_id + g, qsize=(kind == "qsize")) for g in range(n_graphs)]
    graphs, labels = graph_inputs(mi, samples)
    return desc, dims, mi, graphs, labels


def edges_per_forward(mi, graphs) -> int:
    """B x T x sum over MPs and sources of |adj|."""
    T = mi.get_mp_iterations()
    tot = 0
    for _, mps in mi.get_mp_instances():
        for mp in mps:
            for s in mp.source_entities:
                tot += sum(len(g["src_" + s.adj_vector]) for g in graphs)
    return T * tot


# ----------------------------------------------------------------------------------------------
# Multi-GPU sharding (one process per GPU).  RouteNet / Q-size batches shard by graph: graphs are
# independent, so each rank owns a disjoint range of graph ids and the forward needs no
# collective (weak scaling: every rank processes `per_rank` graphs).  Timing is reduced with a
# MAX over ranks; edge counts with a SUM.

def shard_graph_ids(rank: int, world: int, per_rank: int) -> list:
    """Graph ids owned by ``rank``: [rank*per_rank, (rank+1)*per_rank)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def reduce_step_stats(dist, elapsed_s: float, edges: int, device=None):
    """(max elapsed over ranks, total edges over ranks).  ``dist`` is torch.distributed or None."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed_s, edges
    import torch
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=device)
    e = torch.tensor([edges], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(e, op=dist.ReduceOp.SUM)
    return float(t.item()), int(e.item())


def make_synthetic_inputs(n_nodes: int = 1_000_000, hidden: int = 64, iterations: int = 8, graph_id: int = 0,
                          **kw):
    """The large synthetic graph: (description, dims, Model_information, [inputs], [labels])."""
    desc = model_examples.synthetic_graph(hidden=hidden, iterations=iterations)
    dims = {"node_feature": 1, "target": 1, "entities": 0, "adj_nodes_nodes": 0}
    mi = Model_information(desc, dims)
    arr = synthetic.synthetic_graph_arrays(n_nodes=n_nodes, graph_id=graph_id, **kw)
    label = arr.pop("target")
    return desc, dims, mi, [arr], [label]
