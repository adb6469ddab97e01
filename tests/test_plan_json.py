"""ign_plan_create_json (CPU, no GPU): the C++ lowering of model_description.json + dimensions
gives the same plan as the Python path (Model_information -> MPPlan.to_desc -> ign_plan_create):
the same parameter tensors (kind, owner, offset, shape), the same Keras-style names, adjacency /
interleave input keys and entity order, and the same errors for models the engine or the
reference rejects (JO:184-245, GM:338, AUX:764)."""
import copy
import ctypes as C
import json

import pytest

from ignnition_amd import _lib, model_examples, workloads
from ignnition_amd.engine import MPPlan
from ignnition_amd.json_operations import Model_information
from tests.readout_cases import READOUT_CASES

ROUTENET_DIMS = workloads.model("routenet")[1]
QSIZE_DIMS = workloads.model("qsize")[1]
SYNTH_DIMS = {"node_feature": 1, "target": 1, "entities": 0, "adj_nodes_nodes": 0}


def _cases():
    c = {"routenet": (model_examples.routenet(), ROUTENET_DIMS),
         "routenet_h16_t3": (model_examples.routenet(hidden=16, iterations=3), ROUTENET_DIMS),
         "qsize": (model_examples.qsize(), QSIZE_DIMS),
         "synthetic": (model_examples.synthetic_graph(), SYNTH_DIMS)}
    for a in ({"type": "attention"}, {"type": "convolution", "activation_function": "tanh"}, {"type": "ordered"}):
        c["routenet_" + a["type"]] = (model_examples.routenet_aggregation(a), ROUTENET_DIMS)
    for a in ({"type": "attention"}, {"type": "convolution"}, {"type": "concat", "concat_axis": 1},
              {"type": "concat", "concat_axis": 2}):
        c["qsize_%s%s" % (a["type"], a.get("concat_axis", ""))] = (model_examples.qsize_aggregation(a), QSIZE_DIMS)
    c["routenet_msgnet"] = (model_examples.routenet_message_net(inputs=("hs_source", "hs_dest"), units=(24, 32),
                                                                activation="selu"), ROUTENET_DIMS)
    for name, (ops, pin, nets) in READOUT_CASES.items():
        c["readout_" + name] = (model_examples.routenet_readout(ops, pin, nets), ROUTENET_DIMS)
    return c


CASES = _cases()


def _tensors(h):
    n = C.c_int32()
    _lib.check(_lib.lib.ign_plan_num_param_tensors(h, C.byref(n)))
    out = []
    for i in range(n.value):
        k, o, off, r, c = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32(), C.c_int32()
        _lib.check(_lib.lib.ign_plan_param_tensor(h, i, C.byref(k), C.byref(o), C.byref(off), C.byref(r), C.byref(c)))
        out.append((k.value, o.value, off.value, r.value, c.value))
    total = C.c_int64()
    _lib.check(_lib.lib.ign_plan_num_params(h, C.byref(total)))
    return out, total.value


def _create_json(desc, dims):
    h = C.c_void_p()
    rc = _lib.lib.ign_plan_create_json(json.dumps(desc).encode(), json.dumps(dims).encode(), 0, C.byref(h))
    return rc, h


def _describe(h):
    need = C.c_int64()
    _lib.check(_lib.lib.ign_plan_describe_json(h, None, 0, C.byref(need)))
    buf = C.create_string_buffer(need.value)
    _lib.check(_lib.lib.ign_plan_describe_json(h, buf, need.value, C.byref(need)))
    return json.loads(buf.value.decode())


@pytest.mark.parametrize("case", sorted(CASES))
def test_json_plan_equals_python_lowering(case):
    desc, dims = CASES[case]
    plan = MPPlan.from_model_info(Model_information(copy.deepcopy(desc), dims))
    d, keep = plan.to_desc()
    hp = C.c_void_p()
    _lib.check(_lib.lib.ign_plan_create(C.byref(d), 0, C.byref(hp)))
    rc, hj = _create_json(desc, dims)
    try:
        assert rc == 0, _lib.lib.ign_last_error()
        assert _tensors(hj) == _tensors(hp)
        info = _describe(hj)
        specs = plan.param_specs()
        assert [p["name"] for p in info["params"]] == [n for n, _ in specs]
        assert [tuple(p["shape"]) for p in info["params"]] == [tuple(s) for _, s in specs]
        assert [e["name"] for e in info["entities"]] == plan.entities
        assert [e["hidden"] for e in info["entities"]] == plan.hidden
        assert [[tuple(f) for f in e["features"]] for e in info["entities"]] == [list(f) for f in plan.features]
        assert [tuple(a["keys"]) for a in info["adjacencies"]] == [s.keys for s in plan.adj_slots]
        assert info["interleave"] == plan.il_slots
        assert info["label"] == plan.readout_label and info["iterations"] == plan.iterations
    finally:
        _lib.lib.ign_plan_destroy(hp)
        if hj:
            _lib.lib.ign_plan_destroy(hj)


def test_describe_needs_a_json_plan():
    plan = MPPlan.from_model_info(Model_information(model_examples.routenet(), ROUTENET_DIMS))
    d, keep = plan.to_desc()
    h = C.c_void_p()
    _lib.check(_lib.lib.ign_plan_create(C.byref(d), 0, C.byref(h)))
    try:
        assert _lib.lib.ign_plan_describe_json(h, None, 0, None) == -1
    finally:
        _lib.lib.ign_plan_destroy(h)


def _rejected(desc, dims, code, text):
    rc, h = _create_json(desc, dims)
    if h:
        _lib.lib.ign_plan_destroy(h)
    assert rc == code
    assert text in _lib.lib.ign_last_error().decode()


def test_unsupported_models_rejected_like_python():
    d = model_examples.routenet()
    d["message_passing"]["stages"][0]["stage_mp"][0]["update"] = {"type": "neural_network", "nn_name": "readout_model"}
    _rejected(d, ROUTENET_DIMS, -2, "GM:338")
    d = model_examples.routenet()
    for n in d["neural_networks"]:
        if n["nn_name"] == "recurrent1":
            n["recurrent_type"] = "LSTM"
    _rejected(d, ROUTENET_DIMS, -2, "AUX:764")
    d = model_examples.routenet()
    d["readout"][0]["input"] = ["link_capacity"]
    _rejected(d, ROUTENET_DIMS, -2, "raw input features")
    d = model_examples.routenet()
    d["readout"] = [{"type": "product", "type_product": "dot_product", "input": ["path", "path"], "output_name": "p"}] \
        + d["readout"]
    _rejected(d, ROUTENET_DIMS, -2, "tensordot")


def test_reference_validation_errors():
    d = model_examples.routenet()
    d["message_passing"]["stages"][0]["stage_mp"][0]["source_entities"][0]["name"] = "router"
    _rejected(d, ROUTENET_DIMS, -1, "The source entity router was used in a message passing")
    d = model_examples.routenet()
    d["readout"][0]["nn_name"] = "nope"
    _rejected(d, ROUTENET_DIMS, -1, "The name nope is used as a reference to a neural network")
    dims = dict(ROUTENET_DIMS)
    dims.pop("traffic")
    _rejected(model_examples.routenet(), dims, -1, "no entry for 'traffic'")
    _rejected(model_examples.routenet(), {"a": 1}, -1, "no entry")
    rc, h = C.c_int(0), C.c_void_p()
    assert _lib.lib.ign_plan_create_json(b"{not json", b"{}", 0, C.byref(h)) == -1
    assert b"malformed model_description.json" in _lib.lib.ign_last_error()
