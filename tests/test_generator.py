"""Index contract: ignnition_amd.generator vs the reference generator's own outputs.

Fixtures: tests/golden/gen_fixtures.json, produced by tests/golden/make_golden.py from
/root/reference/code/utils/generator_std_to_framework.py (GEN:53-224).  Bit-exact.
"""
import json

import numpy as np

import numpy as np
import pytest

from ignnition_amd import generator as G
from ignnition_amd import synthetic


def _norm(v):
    if isinstance(v, np.ndarray):
        return v.tolist()
    return v


@pytest.mark.parametrize("idx", range(8))
def test_generator_matches_reference(gen_fixtures, idx, tmp_path):
    case = gen_fixtures[idx]
    synthetic.write_tar_dataset(case["samples"], str(tmp_path), per_file=len(case["samples"]))
    out = list(G.generator(str(tmp_path), case["feature_names"], case["output_name"], case["adj_names"],
                           case["interleave_names"], [], case["training"], False))
    assert len(out) == len(case["expected"])
    for got, exp in zip(out, case["expected"]):
        data = got[0] if case["training"] else got
        assert set(data) == set(exp["data"]), case["name"]
        for k, v in exp["data"].items():
            assert _norm(data[k]) == v, (case["name"], k)
        if case["training"]:
            assert got[1] == exp["output"]


def test_generator_bytes_arguments(gen_fixtures, tmp_path):
    """The reference receives its arguments as bytes from tf.data (GEN:75-80)."""
    case = gen_fixtures[0]
    synthetic.write_tar_dataset(case["samples"], str(tmp_path))
    enc = lambda s: s.encode()
    out = list(G.generator(enc(str(tmp_path)), [enc(f) for f in case["feature_names"]], enc(case["output_name"]),
                           [[enc(x) for x in a] for a in case["adj_names"]], [], [], True))
    assert out[0][0]["src_adj_links_paths"] == case["expected"][0]["data"]["src_adj_links_paths"]


def test_make_indices_order():
    counter, idx = G.make_indices({"b": "x", "a": "y", "c": "x"})
    assert list(counter.items()) == [("x", 2), ("y", 1)]
    assert idx == {"b": 0, "a": 0, "c": 1}


def test_wrong_destination_type_skips_file(tmp_path, caplog):
    """GEN:147-151 raise -> GEN:229-230 log and abandon the file."""
    s = {"traffic": [1.0], "link_capacity": [1.0], "delay": [1.0],
         "entities": {"l0": "link", "p0": "path"},
         "adj_links_paths": {"l0": ["l0"]}, "adj_paths_links": {"l0": ["p0"]}}
    synthetic.write_tar_dataset([s], str(tmp_path))
    out = list(G.generator(str(tmp_path), ["traffic"], "delay",
                           [["adj_links_paths", "link", "path", "False"]], [], [], True))
    assert out == []
    assert any("was expected to be from" in r.message for r in caplog.records)


def test_missing_feature_raises_message():
    with pytest.raises(Exception, match="feature named"):
        G.sample_to_data({"entities": {}}, ["traffic"], "delay", [], [], [], True)


def test_synthetic_layout_matches_migrate():
    """Synthetic samples follow migrate.py's layout (MIG:54-109): links first in entity order,
    paths for every ordered pair, adj_links_paths keyed by path in path order."""
    s = synthetic.routenet_sample("nsfnet", 3)
    ents = list(s["entities"].items())
    n_links = sum(1 for _, t in ents if t == "link")
    assert all(t == "link" for _, t in ents[:n_links])
    assert sum(1 for _, t in ents if t == "path") == 14 * 13
    assert list(s["adj_links_paths"]) == ["p%d" % i for i in range(182)]
    assert len(s["traffic"]) == 182 and len(s["link_capacity"]) == n_links == 42
    again = synthetic.routenet_sample("nsfnet", 3)
    assert json.dumps(again) == json.dumps(s)


def test_synthetic_large_graph_arrays_match_generator():
    """The vectorised 1M-node generator emits exactly what the generator (GEN:134-190) makes of
    the equivalent dict sample (checked on a small instance)."""
    arr = synthetic.synthetic_graph_arrays(n_nodes=500, window=20, graph_id=3)
    sample = synthetic.synthetic_sample(arr)
    data, y = G.sample_to_data(sample, ["node_feature"], "target", [["adj_nodes_nodes", "node", "node", "False"]],
                               [], [], True)
    for k in ("src_adj_nodes_nodes", "dst_adj_nodes_nodes", "seq_node_node"):
        assert data[k] == arr[k].tolist(), k
    assert data["num_node"] == 500
    assert y == [float(v) for v in arr["target"]]
    deg = np.bincount(arr["dst_adj_nodes_nodes"], minlength=500)
    assert deg.max() <= 30 and abs(deg.mean() - 10) < 1.0
