"""The two example GNNs of the reference as Python dicts.

Semantically identical to the reference's ``examples/Routenet/model_description.json``
(RNJ:1-165) and ``examples/Q-size/model_description.json`` (QSJ:1-209): same entities,
stages, aggregations, GRU update, readout network and learning options.  Kept as
data here so the tests, bench and ``examples/*/main.py`` can write them out to a
``model_description.json`` that the engine then parses exactly like a user's file.
"""

from __future__ import annotations

import copy
import json

_READOUT = [
    {"type_layer": "Dense", "units": 256, "kernel_regularizer": 0.1, "activation": "selu"},
    {"type_layer": "Dense", "units": 256, "kernel_regularizer": 0.1, "activation": "selu"},
    {"type_layer": "Dense", "units": 1, "kernel_regularizer": 0.01, "activation": "None"},
]


def _entity(name, feature, norm, hidden=32):
    return {"name": name, "hidden_state_dimension": hidden,
            "features": [{"name": feature, "normalization": norm}]}


def _src(name, adj):
    return {"name": name, "adj_vector": adj, "message": [{"type": "direct_assignation"}]}


def _gru_update():
    return {"type": "recurrent_neural_network", "nn_name": "recurrent1"}


def routenet_aggregation(aggregation: dict, hidden: int = 32, iterations: int = 8) -> dict:
    """RouteNet with the path -> link stage aggregated by ``aggregation`` (e.g. {"type":
    "attention"} or {"type": "convolution", "activation_function": "relu"}): schema-legal
    aggregations outside the example configs (AUX:264-401)."""
    d = routenet(hidden, iterations)
    d["message_passing"]["stages"][1]["stage_mp"][0]["aggregation"] = dict(aggregation)
    return d


def qsize_aggregation(aggregation: dict, iterations: int = 8) -> dict:
    """Q-size with the {link, node} -> path stage aggregated by ``aggregation`` instead of
    interleave: a two-source attention / convolution (AUX:264-401 with GM:523-541)."""
    d = qsize(iterations=iterations)
    mp = d["message_passing"]["stages"][0]["stage_mp"][0]
    mp["aggregation"] = dict(aggregation)
    if aggregation.get("type") == "concat":
        d["message_passing"]["stages"][0]["stage_mp"][0].pop("interleave_definition", None)
    return d


def routenet_message_net(inputs=("hs_source", "hs_dest"), units=(32,), activation="relu", hidden: int = 32,
                         iterations: int = 8) -> dict:
    """RouteNet whose path -> link messages come from a message-creation network (GM:440-475)
    on ``inputs`` (hs_source, hs_dest, edge_params) instead of direct assignation."""
    d = routenet(hidden, iterations)
    src = d["message_passing"]["stages"][1]["stage_mp"][0]["source_entities"][0]
    src["message"] = [{"type": "neural_network", "nn_name": "message_nn", "input": list(inputs)}]
    d["neural_networks"].append({"nn_name": "message_nn", "nn_type": "feed_forward", "nn_architecture": [
        {"type_layer": "Dense", "units": u, "activation": activation} for u in units]})
    return d


def routenet_readout(ops: list, predict_input: list, nets: dict = None, hidden: int = 32,
                     iterations: int = 8) -> dict:
    """RouteNet with readout operations before predict (GM:605-655, AUX:1033-1265): ``ops`` is
    the readout list without the predict, ``predict_input`` the predict op's inputs, ``nets``
    extra neural networks {nn_name: [(units, activation), ...]} used by neural_network ops."""
    d = routenet(hidden, iterations)
    pred = d["readout"][0]
    pred["input"] = list(predict_input)
    d["readout"] = [copy.deepcopy(o) for o in ops] + [pred]
    for name, layers in (nets or {}).items():
        d["neural_networks"].append({"nn_name": name, "nn_type": "feed_forward", "nn_architecture": [
            {"type_layer": "Dense", "units": u, "activation": a} for u, a in layers]})
    return d


def routenet(hidden: int = 32, iterations: int = 8) -> dict:
    """RNJ:1-165."""
    layer_names = ["1st_dense_layer", "2nd_dense_layer", "Output_layer"]
    readout = [dict(l, name=n) for l, n in zip(copy.deepcopy(_READOUT), layer_names)]
    return {
        "entities": [_entity("link", "link_capacity", "normalization_routenet", hidden),
                     _entity("path", "traffic", "normalization_routenet", hidden)],
        "message_passing": {
            "num_iterations": iterations,
            "stages": [
                {"stage_name": "stage1", "stage_mp": [
                    {"destination_entity": "path",
                     "source_entities": [_src("link", "adj_links_paths")],
                     "aggregation": {"type": "ordered"},
                     "update": _gru_update()}]},
                {"stage_name": "stage2", "stage_mp": [
                    {"source_entity": "path", "destination_entity": "link",
                     "source_entities": [_src("path", "adj_paths_links")],
                     "aggregation": {"type": "sum"},
                     "update": _gru_update()}]},
            ]},
        "readout": [{"type": "predict", "input": ["path"], "label": "delay",
                     "label_normalization": "log", "nn_name": "readout_model"}],
        "neural_networks": [
            {"nn_name": "readout_model", "nn_type": "feed_forward", "nn_architecture": readout},
            {"nn_name": "recurrent1", "nn_type": "recurrent_neural_network", "recurrent_type": "GRU"}],
        "learning_options": {"loss": "MeanSquaredError",
                             "optimizer": {"type": "Adam",
                                           "schedule": {"type": "ExponentialDecay",
                                                        "initial_learning_rate": 0.001,
                                                        "decay_steps": 80000, "decay_rate": 0.6}}},
    }


def qsize(hidden: int = 32, iterations: int = 8) -> dict:
    """QSJ:1-209."""
    layer_names = ["First_dense_layer", "Second_dense_layer", "Output_layer"]
    readout = [dict(l, name=n) for l, n in zip(copy.deepcopy(_READOUT), layer_names)]
    norm = "normalization_queue_size"
    return {
        "entities": [_entity("link", "link_capacity", norm, hidden),
                     _entity("path", "traffic", norm, hidden),
                     _entity("node", "queue_sizes", norm, hidden)],
        "message_passing": {
            "num_iterations": iterations,
            "stages": [
                {"stage_name": "step1", "stage_mp": [
                    {"destination_entity": "path",
                     "source_entities": [_src("link", "adj_links_paths"), _src("node", "adj_nodes_paths")],
                     "aggregation": {"type": "interleave", "interleave_definition": "path_interleave"},
                     "update": _gru_update()}]},
                {"stage_name": "step2", "stage_mp": [
                    {"destination_entity": "link",
                     "source_entities": [_src("path", "adj_paths_links")],
                     "aggregation": {"type": "sum"}, "update": _gru_update()},
                    {"destination_entity": "node",
                     "source_entities": [_src("path", "adj_paths_nodes")],
                     "aggregation": {"type": "sum"}, "update": _gru_update()}]},
            ]},
        "readout": [{"type": "predict", "input": ["path"], "label": "delay",
                     "label_normalization": norm, "nn_name": "readout_model"}],
        "neural_networks": [
            {"nn_name": "readout_model", "nn_type": "feed_forward", "nn_architecture": readout},
            {"nn_name": "recurrent1", "nn_type": "recurrent_neural_network", "recurrent_type": "GRU"}],
        "learning_options": {"loss": "MeanSquaredError",
                             "optimizer": {"type": "Adam",
                                           "schedule": {"type": "ExponentialDecay",
                                                        "initial_learning_rate": 0.001, "decay_steps": 82000,
                                                        "decay_rate": 0.8, "staircase": "True"}}},
    }


def synthetic_graph(hidden: int = 64, iterations: int = 8) -> dict:
    """The 1M-node / 10M-edge synthetic config: one entity, sum + GRU, predict."""
    return {
        "entities": [_entity("node", "node_feature", "None", hidden)],
        "message_passing": {"num_iterations": iterations, "stages": [
            {"stage_name": "stage1", "stage_mp": [
                {"destination_entity": "node", "source_entities": [_src("node", "adj_nodes_nodes")],
                 "aggregation": {"type": "sum"}, "update": _gru_update()}]}]},
        "readout": [{"type": "predict", "input": ["node"], "label": "target", "nn_name": "readout_model"}],
        "neural_networks": [
            {"nn_name": "readout_model", "nn_type": "feed_forward", "nn_architecture": copy.deepcopy(_READOUT)},
            {"nn_name": "recurrent1", "nn_type": "recurrent_neural_network", "recurrent_type": "GRU"}],
        "learning_options": {"loss": "MeanSquaredError", "optimizer": {"type": "Adam"}},
    }


def write(desc: dict, path: str) -> str:
    with open(path, "w") as fh:
        json.dump(desc, fh, indent=1)
    return path
