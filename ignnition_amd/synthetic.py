"""Synthetic IGNNITION samples in the reference dataset layout.

The real NSFNET / GEANT2 / synth50 datasets are not available (the reference lists
them as missing blobs and they need a download).  This module fabricates samples
with the exact JSON layout the reference's migration script writes
(examples/Routenet/migrate.py:54-109): an ``entities`` dict (links first, named
``l<k>`` in ``G.edges`` order, then paths ``p<k>`` for every ordered (i, j), i != j,
lexicographic), ``adj_paths_links`` keyed in first-traversal order and
``adj_links_paths`` keyed by path.  The Q-size variant adds ``node`` entities,
``adj_nodes_paths`` / ``adj_paths_nodes`` and a per-sample ``path_interleave``
pattern (examples/Q-size/model_description.json:72-76).

Every generator is seeded with numpy PCG64, seed = 20261015 + graph_id.
Feature/label values are synthetic (uniform / log-normal), not simulator output.
"""

from __future__ import annotations

import numpy as np
import networkx as nx

BASE_SEED = 20261015

# (nodes, undirected links) of the random stand-in topologies.
TOPOLOGIES = {
    "nsfnet": (14, 21),
    "geant2": (24, 37),
    "synth50": (50, 100),
}


def _connected_gnm(n: int, m: int, rng: np.random.Generator) -> nx.Graph:
    for _ in range(1000):
        g = nx.gnm_random_graph(n, m, seed=int(rng.integers(0, 2**31 - 1)))
        if nx.is_connected(g):
            return g
    raise RuntimeError("could not draw a connected topology")


def _topology(n: int, m: int, rng: np.random.Generator):
    """Directed topology (both directions of every undirected link) + shortest-path routing."""
    g = _connected_gnm(n, m, rng)
    dg = nx.DiGraph()
    dg.add_nodes_from(range(n))
    for (a, b) in sorted(g.edges()):
        dg.add_edge(a, b)
        dg.add_edge(b, a)
    routing = dict(nx.all_pairs_shortest_path(dg))
    return dg, routing


def routenet_sample(topology: str = "nsfnet", graph_id: int = 0, qsize: bool = False,
                    n_nodes: int | None = None, n_links: int | None = None) -> dict:
    """One sample dict in the migrate.py layout (MIG:54-109); ``qsize`` adds node entities."""
    if n_nodes is None:
        n_nodes, n_links = TOPOLOGIES[topology]
    rng = np.random.Generator(np.random.PCG64(BASE_SEED + graph_id))
    dg, routing = _topology(n_nodes, n_links, rng)

    n_paths = n_nodes * (n_nodes - 1)
    n_dlinks = dg.number_of_edges()
    data: dict = {}
    if qsize:   # value ranges centred on the Q-size normalisation (QSM:27-39)
        data["traffic"] = [float(x) for x in rng.uniform(0.05, 0.5, n_paths)]
        data["link_capacity"] = [float(x) for x in rng.choice([10.0, 25.0, 40.0], n_dlinks)]
    else:       # centred on normalization_routenet (RNM:26-31)
        data["traffic"] = [float(x) for x in rng.uniform(20.0, 320.0, n_paths)]
        data["link_capacity"] = [float(x) for x in rng.choice([10000.0, 40000.0], n_dlinks)]
    data["delay"] = [float(x) for x in rng.lognormal(-1.0, 0.5, n_paths)]
    data["jitter"] = [float(x) for x in rng.lognormal(-2.0, 0.5, n_paths)]

    data["entities"] = {}
    link_of = {}
    for k, (a, b) in enumerate(dg.edges):
        name = "l" + str(k)
        data["entities"][name] = "link"
        link_of[(a, b)] = name

    data["adj_paths_links"] = {}
    data["adj_links_paths"] = {}
    if qsize:
        data["adj_paths_nodes"] = {}
        data["adj_nodes_paths"] = {}

    p = 0
    for i in range(n_nodes):
        for j in range(n_nodes):
            if i == j:
                continue
            pname = "p" + str(p)
            data["entities"][pname] = "path"
            route = routing[i][j]
            for h in range(1, len(route)):
                lname = link_of[(route[h - 1], route[h])]
                data["adj_paths_links"].setdefault(lname, []).append(pname)
                data["adj_links_paths"].setdefault(pname, []).append(lname)
                if qsize:
                    nname = "n" + str(route[h - 1])
                    data["adj_paths_nodes"].setdefault(nname, []).append(pname)
                    data["adj_nodes_paths"].setdefault(pname, []).append(nname)
            p += 1

    if qsize:
        for v in range(n_nodes):
            data["entities"]["n" + str(v)] = "node"
        data["queue_sizes"] = [float(x) for x in rng.integers(1, 33, n_nodes)]
        data["path_interleave"] = ["node", "link"]
    return data


def dataset(topology: str, n_graphs: int, qsize: bool = False, first_id: int = 0) -> list:
    return [routenet_sample(topology, first_id + g, qsize=qsize) for g in range(n_graphs)]


def write_tar_dataset(samples: list, directory: str, per_file: int = 100) -> list:
    """Write samples as ``sample_<k>.tar.gz`` archives holding ``data.json`` (MIG:112-127)."""
    import io
    import json
    import os
    import tarfile

    os.makedirs(directory, exist_ok=True)
    paths = []
    for k in range(0, len(samples), per_file):
        blob = json.dumps(samples[k:k + per_file]).encode()
        path = os.path.join(directory, "sample_%d.tar.gz" % (k // per_file))
        with tarfile.open(path, "w:gz") as tar:
            info = tarfile.TarInfo("data.json")
            info.size = len(blob)
            tar.addfile(info, io.BytesIO(blob))
        paths.append(path)
    return paths


# ----------------------------------------------------------------------------------------------
# Large synthetic graph (BASELINE configs[4]): one entity ``node``, one scalar feature
# ``node_feature``, adjacency ``adj_nodes_nodes`` (sum + GRU), label ``target``.  In-degree
# ~ Poisson(mean_deg) capped at max_deg; 90 % of the sources are drawn within +-window ids of
# the destination (locality -> contiguous-range edge-cut), 10 % uniformly.  The arrays are built
# vectorised in the exact layout the generator emits for the equivalent dict sample (destination
# keys in increasing id order, nodes without in-edges are not keys): see synthetic_sample().

def synthetic_graph_arrays(n_nodes: int = 1_000_000, mean_deg: float = 10.0, max_deg: int = 30,
                           window: int = 4096, p_local: float = 0.9, graph_id: int = 0) -> dict:
    rng = np.random.Generator(np.random.PCG64(BASE_SEED + graph_id))
    deg = np.minimum(rng.poisson(mean_deg, n_nodes), max_deg).astype(np.int64)
    E = int(deg.sum())
    dst = np.repeat(np.arange(n_nodes, dtype=np.int64), deg)
    starts = np.cumsum(deg) - deg
    seq = np.arange(E, dtype=np.int64) - np.repeat(starts, deg)
    local = rng.random(E) < p_local
    off = rng.integers(-window, window + 1, E)
    src = np.where(local, np.clip(dst + off, 0, n_nodes - 1), rng.integers(0, n_nodes, E)).astype(np.int64)
    feat = rng.random(n_nodes).astype(np.float32)
    target = rng.random(n_nodes).astype(np.float32)
    return {"node_feature": feat, "target": target, "src_adj_nodes_nodes": src, "dst_adj_nodes_nodes": dst,
            "seq_node_node": seq, "num_node": n_nodes}


def synthetic_sample(arrays: dict) -> dict:
    """The dict sample (migrate-style layout) equivalent to ``synthetic_graph_arrays`` output
    (small instances only: used to pin the vectorised arrays against the generator)."""
    n = int(arrays["num_node"])
    names = ["n%d" % i for i in range(n)]
    adj: dict = {}
    for s, d in zip(arrays["src_adj_nodes_nodes"].tolist(), arrays["dst_adj_nodes_nodes"].tolist()):
        adj.setdefault(names[d], []).append(names[s])
    return {"entities": {nm: "node" for nm in names}, "adj_nodes_nodes": adj,
            "node_feature": [float(x) for x in arrays["node_feature"]],
            "target": [float(x) for x in arrays["target"]]}
