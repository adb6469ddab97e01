"""User API: ``create_model``, ``find_dataset_dimensions``, ``predict``, ``debug``, ``train_and_evaluate``.

Mirrors ``code/utils/framework_operations.py`` (FO): same names, the same
``./train_options.ini`` (ConfigParser with ExtendedInterpolation, FO:34-36) and the same
``model_description.json``.  The compute underneath is the HIP engine (libignmp.so).
"""

from __future__ import annotations

import configparser
import datetime
import glob
import json
import logging
import os
import sys
import tarfile

import numpy as np

from . import generate_model as gm
from .json_operations import Model_information

log = logging.getLogger("ignnition_amd")

CONFIG = configparser.ConfigParser()
CONFIG._interpolation = configparser.ExtendedInterpolation()
CONFIG.read("./train_options.ini")


def load_config(path: str):
    CONFIG.read(path)
    return CONFIG


def create_model():
    """FO:42-47."""
    json_path = CONFIG["PATHS"]["json_path"]
    dimensions = find_dataset_dimensions(CONFIG["PATHS"]["train_dataset"])
    return Model_information(json_path, dimensions)


def dimensions_of_sample(sample_data: dict) -> dict:
    """FO:68-87 for one sample: list-of-lists -> len of the inner list, other non-dict -> 1,
    dict whose first value's first element is a [node, params] list -> len(params), else 0."""
    dimensions = {}
    for k, v in sample_data.items():
        if not isinstance(v, dict):
            if isinstance(v, list) and isinstance(v[0], list):
                dimensions[k] = len(v[0])
            else:
                dimensions[k] = 1
        elif v:
            first_key = list(v.keys())[0]
            element = v[first_key]
            if (not isinstance(element[0], str)) and isinstance(element[0], list):
                dimensions[k] = len(element[0][1])
            else:
                dimensions[k] = 0
    return dimensions


def find_dataset_dimensions(path):
    """FO:50-91."""
    files = glob.glob(str(path) + "/*.tar.gz")
    if not files:
        log.error("IGNNITION: no *.tar.gz dataset found in " + str(path))
        sys.exit(1)
    sample = files[0]
    try:
        with tarfile.open(sample, "r:gz") as tar:
            sample_data = json.load(tar.extractfile("data.json"))[0]
    except Exception:
        log.error("IGNNITION: Failed to read the data file " + sample)
        sys.exit(1)
    return dimensions_of_sample(sample_data)


def str_to_bool(a):
    return a == "True"


def predict(model_info, params=None, batch_size: int = 1):
    """FO:169-236: run the model over ``predict_dataset`` and return the per-sample flattened,
    denormalised predictions.  ``params`` (dict or a safetensors path) replaces the TF
    Saver restore of ``warm_start_path`` (FO:218-221)."""
    log.warning("IGNNITION: Starting to make the predictions...")
    gm.set_model_info(model_info)
    data_path = CONFIG["PATHS"]["predict_dataset"]
    if params is None:
        params = CONFIG["PATHS"].get("warm_start_path", None)
    if isinstance(params, str):
        from .checkpoint import load_params
        params = load_params(params)
    model = gm.ComnetModel(model_info, params=params)
    output_name, _, output_denorm = model_info.get_output_info()
    all_predictions = []
    for batch in gm.input_fn(data_path, training=False, batch_size=batch_size, repeat=False):
        out = model.batch(batch)
        pred = out.forward()
        start = 0
        flat = pred.reshape(-1)
        units = out.output_units
        for n in out.graph_rows[:, model.plan.readout_inputs[0]]:
            p = flat[start:start + n * units]
            start += n * units
            if output_denorm is not None:
                try:
                    p = gm._resolve(output_denorm)(p, output_name)
                except KeyError:
                    log.warning("IGNNITION: A denormalization function for output " + output_name +
                                " was not defined. The output will be normalized.")
            print(p)
            all_predictions.append(np.asarray(p))
    return all_predictions


def debug(model_description, out_dir: str = "../debug_model/"):
    """FO:239-268.  The reference dumps the TF graph for TensorBoard; here the lowered plan
    (entities, adjacency slots, MPs in execution order, cells, readout, parameter layout)
    is written as ``<out_dir>/plan.json``."""
    log.warning("IGNNITION: Generating the debug model...")
    gm.set_model_info(model_description)
    from .engine import MPPlan
    plan = MPPlan.from_model_info(model_description)
    dump = {
        "entities": [{"name": n, "hidden": h, "features": f} for n, h, f in zip(plan.entities, plan.hidden,
                                                                                plan.features)],
        "iterations": plan.iterations,
        "adjacency_slots": [s.__dict__ for s in plan.adj_slots],
        "interleave_slots": plan.il_slots,
        "message_passings": plan.mps,
        "cells": plan.cells,
        "readout_inputs": plan.readout_inputs,
        "dense": plan.dense,
        "parameters": [[n, list(s)] for n, s in plan.param_specs()],
        "created": str(datetime.datetime.now()),
    }
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "plan.json"), "w") as fh:
        json.dump(dump, fh, indent=1)
    log.warning("IGNNITION: The debug model has been generated.")
    return dump


def train_and_evaluate(model):
    """FO:108-166.  Training (backward through the packed GRU, MSE + L2, Adam) is the next
    row of the build and is not lowered yet."""
    raise NotImplementedError("train_and_evaluate: the backward pass is not implemented in this round "
                              "(forward / predict are)")
