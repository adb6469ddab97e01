"""Generate the golden fixtures from the REFERENCE's own pure-Python code.

Run in the build container only (it reads /root/reference, which does not exist on
the GPU box):   python tests/golden/make_golden.py

* ``gen_fixtures.json``  — inputs (sample dicts in the reference dataset layout) and the
  outputs of the reference generator ``code/utils/generator_std_to_framework.py``
  (GEN:53-224), run on tar.gz archives exactly as the reference reads them.
* ``plan_fixtures.json`` — the plan that the reference ``Model_information``
  (code/utils/json_operations.py:128-149) builds from the reference's two example
  ``model_description.json`` files, dumped through its public getters.

The reference imports TensorFlow / Keras / jsonschema at module top level; none is
installed, so minimal stand-in modules are registered in ``sys.modules`` that provide
only what these two code paths touch at import/run time (``tf.compat.v1.logging`` and
``tf.keras.regularizers.l2``; ``jsonschema.validate`` as a no-op — the schema itself is
restated in ignnition_amd/schema.py).  No numeric TF code runs.  Bytecode writing is
disabled so nothing is written into the read-only reference tree.
"""

import json
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from ignnition_amd import synthetic  # noqa: E402


def _install_stubs():
    logged = []

    class _Log:
        def error(self, *a):
            logged.append(("error", " ".join(str(x) for x in a)))

        def warn(self, *a):
            logged.append(("warn", " ".join(str(x) for x in a)))

        info = warn
        warning = warn

        def set_verbosity(self, *a):
            pass

        INFO = 20

    tf = types.ModuleType("tensorflow")
    tf.compat = types.SimpleNamespace(v1=types.SimpleNamespace(logging=_Log()))
    keras_ns = types.SimpleNamespace(
        regularizers=types.SimpleNamespace(l2=lambda c: {"l2": float(c)}),
        layers=types.SimpleNamespace(),
        activations=types.SimpleNamespace(),
    )
    tf.keras = keras_ns
    tfk = types.ModuleType("tensorflow.keras")
    tfk_act = types.ModuleType("tensorflow.keras.activations")
    keras = types.ModuleType("keras")
    keras_backend = types.ModuleType("keras.backend")
    keras.backend = keras_backend
    jsonschema = types.ModuleType("jsonschema")
    jsonschema.validate = lambda instance, schema: None
    sys.modules.update({
        "tensorflow": tf, "tensorflow.keras": tfk, "tensorflow.keras.activations": tfk_act,
        "keras": keras, "keras.backend": keras_backend, "jsonschema": jsonschema,
    })
    sys.path.insert(0, os.path.join(REF, "code", "utils"))
    return logged


def _gen_case(GEN, name, samples, feature_names, output_name, adj_names, interleave_names, training=True):
    with tempfile.TemporaryDirectory() as d:
        synthetic.write_tar_dataset(samples, d, per_file=len(samples))
        enc = lambda s: s.encode("ascii")
        out = list(GEN.generator(enc(d), [enc(f) for f in feature_names], enc(output_name),
                                 [[enc(x) for x in a] for a in adj_names],
                                 [[enc(x) for x in i] for i in interleave_names], [], training, False))
    expected = []
    for item in out:
        if training:
            data, output = item
            expected.append({"data": data, "output": output})
        else:
            expected.append({"data": item})
    return {"name": name, "samples": samples, "feature_names": feature_names, "output_name": output_name,
            "adj_names": adj_names, "interleave_names": interleave_names, "training": training,
            "expected": expected}


def make_gen_fixtures(GEN):
    cases = []
    rn_adj = [["adj_links_paths", "link", "path", "False"], ["adj_paths_links", "path", "link", "False"]]
    qs_adj = [["adj_links_paths", "link", "path", "False"], ["adj_nodes_paths", "node", "path", "False"],
              ["adj_paths_links", "path", "link", "False"], ["adj_paths_nodes", "path", "node", "False"]]

    # 1) the survey's 2-link / 3-path hand sample — destination groups unsorted.
    tiny = {"traffic": [1.0, 2.0, 3.0], "delay": [0.5, 0.25, 0.125], "link_capacity": [10.0, 40.0],
            "entities": {"l0": "link", "l1": "link", "p0": "path", "p1": "path", "p2": "path"},
            "adj_links_paths": {"p0": ["l0", "l1"], "p1": ["l1"], "p2": ["l1", "l0"]},
            "adj_paths_links": {"l0": ["p0", "p2"], "l1": ["p1", "p0", "p2"]}}
    cases.append(_gen_case(GEN, "tiny_routenet", [tiny], ["link_capacity", "traffic"], "delay", rn_adj, []))

    # 2) entities listed interleaved by type + out-of-order destination keys.
    mixed = {"traffic": [5.0, 6.0], "delay": [1.0, 2.0], "link_capacity": [1.0, 2.0, 3.0],
             "entities": {"p1": "path", "l2": "link", "l0": "link", "p0": "path", "l1": "link"},
             "adj_links_paths": {"p0": ["l1", "l2", "l0"], "p1": ["l2"]},
             "adj_paths_links": {"l1": ["p0"], "l2": ["p1", "p0"], "l0": ["p0"]}}
    cases.append(_gen_case(GEN, "mixed_order", [mixed], ["link_capacity", "traffic"], "delay", rn_adj, []))

    # 3) edge parameters ([[src, params], ...]) on one adjacency (GEN:156-163).
    params = {"traffic": [1.0, 2.0], "delay": [0.1, 0.2], "link_capacity": [3.0, 4.0],
              "entities": {"l0": "link", "l1": "link", "p0": "path", "p1": "path"},
              "adj_links_paths": {"p0": [["l0", [1, 2]], ["l1", [3, 4]]], "p1": [["l1", [5, 6]]]},
              "adj_paths_links": {"l1": ["p0", "p1"], "l0": ["p0"]}}
    cases.append(_gen_case(GEN, "edge_params", [params], ["link_capacity", "traffic"], "delay",
                           [["adj_links_paths", "link", "path", "True"], rn_adj[1]], []))

    # 4) Q-size-style hand sample with a ["node","link"] interleave.
    qs = {"traffic": [1.0, 2.0], "delay": [0.3, 0.4], "link_capacity": [1.0, 2.0], "queue_sizes": [4.0, 8.0, 16.0],
          "entities": {"l0": "link", "l1": "link", "p0": "path", "p1": "path", "n0": "node", "n1": "node",
                       "n2": "node"},
          "adj_links_paths": {"p0": ["l0", "l1"], "p1": ["l1"]},
          "adj_nodes_paths": {"p0": ["n0", "n1"], "p1": ["n1"]},
          "adj_paths_links": {"l0": ["p0"], "l1": ["p0", "p1"]},
          "adj_paths_nodes": {"n0": ["p0"], "n1": ["p0", "p1"]},
          "path_interleave": ["node", "link"]}
    cases.append(_gen_case(GEN, "tiny_qsize", [qs], ["link_capacity", "traffic", "queue_sizes"], "delay", qs_adj,
                           [["path_interleave", "path"]]))

    # 5) unequal source lengths in an interleave pattern of length 3.
    qs2 = json.loads(json.dumps(qs))
    qs2["adj_nodes_paths"] = {"p0": ["n0"], "p1": ["n1"]}
    qs2["path_interleave"] = ["link", "node", "link"]
    cases.append(_gen_case(GEN, "interleave_ragged", [qs2], ["link_capacity", "traffic", "queue_sizes"], "delay",
                           qs_adj, [["path_interleave", "path"]]))

    # 6) synthetic NSFNET-size RouteNet samples (migrate.py layout), two graphs in one archive.
    rn = [synthetic.routenet_sample("nsfnet", g) for g in range(2)]
    cases.append(_gen_case(GEN, "nsfnet_routenet", rn, ["link_capacity", "traffic"], "delay", rn_adj, []))

    # 7) synthetic NSFNET-size Q-size sample.
    q = [synthetic.routenet_sample("nsfnet", 7, qsize=True)]
    cases.append(_gen_case(GEN, "nsfnet_qsize", q, ["link_capacity", "traffic", "queue_sizes"], "delay", qs_adj,
                           [["path_interleave", "path"]]))

    # 8) predict mode (training=False): no label read.
    cases.append(_gen_case(GEN, "tiny_predict", [tiny], ["link_capacity", "traffic"], "delay", rn_adj, [],
                           training=False))
    return cases


def dump_plan(JO, path, dims):
    mi = JO.Model_information(path, dict(dims))
    stages = []
    for name, mps in mi.get_mp_instances():
        out = []
        for mp in mps:
            upd = mp.update
            out.append({
                "destination_entity": mp.destination_entity,
                "sources": [{"name": s.name, "adj_vector": s.adj_vector, "extra_parameters": s.extra_parameters,
                             "message": [o.type for o in s.message_formation]} for s in mp.source_entities],
                "aggregation": mp.aggregation.type,
                "interleave_definition": getattr(mp.aggregation, "combination_definition", None),
                "concat_axis": getattr(mp.aggregation, "concat_axis", None),
                "update_type": upd.type,
                "recurrent_type": getattr(upd.model, "type", None) if upd.type == "recurrent_nn" else None,
                "recurrent_params": dict(getattr(upd.model, "parameters", {})) if upd.type == "recurrent_nn" else None,
            })
        stages.append([name, out])
    readout = []
    for op in mi.get_readout_operations():
        d = {"type": op.type, "input": list(op.input)}
        if op.type == "predict":
            d["label"] = op.label
            d["label_normalization"] = op.label_normalization
            d["label_denormalization"] = op.label_denormalization
            d["layers"] = [{"type": l.type, "parameters": {k: v for k, v in l.parameters.items()}}
                           for l in op.architecture.layers]
        readout.append(d)
    return {
        "entities": [{"name": e.name, "hidden_state_dimension": e.hidden_state_dimension,
                      "features": [{"name": f.name, "size": f.size, "normalization": f.normalization}
                                   for f in e.features]} for e in mi.get_entities()],
        "iterations": mi.get_mp_iterations(),
        "stages": stages,
        "readout": readout,
        "adjacency_info": mi.get_adjecency_info(),
        "interleave_tensors": mi.get_interleave_tensors(),
        "interleave_sources": mi.get_interleave_sources(),
        "input_dimensions": mi.get_input_dimensions(),
        "all_features": [f.name for f in mi.get_all_features()],
        "output_info": list(mi.get_output_info()),
        "loss": mi.get_loss(),
        "optimizer": mi.get_optimizer(),
        "additional_input_names": sorted(mi.get_additional_input_names()),
        "dims": dims,
    }


def main():
    _install_stubs()
    import generator_std_to_framework as GEN  # noqa: E402
    cwd = os.getcwd()
    os.chdir(os.path.join(REF, "code"))  # JO opens './utils/schema.json' relative to cwd (JO:139)
    try:
        import json_operations as JO  # noqa: E402
        rn_dims = {"traffic": 1, "delay": 1, "jitter": 1, "link_capacity": 1, "entities": 0,
                   "adj_paths_links": 0, "adj_links_paths": 0}
        qs_dims = dict(rn_dims, queue_sizes=1, adj_paths_nodes=0, adj_nodes_paths=0, path_interleave=1)
        plans = {
            "routenet": dump_plan(JO, os.path.join(REF, "examples/Routenet/model_description.json"), rn_dims),
            "qsize": dump_plan(JO, os.path.join(REF, "examples/Q-size/model_description.json"), qs_dims),
        }
    finally:
        os.chdir(cwd)
    with open(os.path.join(HERE, "plan_fixtures.json"), "w") as fh:
        json.dump(plans, fh, indent=1, sort_keys=True)
    cases = make_gen_fixtures(GEN)
    with open(os.path.join(HERE, "gen_fixtures.json"), "w") as fh:
        json.dump(cases, fh, separators=(",", ":"))
    print("wrote", len(cases), "generator cases and", len(plans), "plans")


if __name__ == "__main__":
    main()
