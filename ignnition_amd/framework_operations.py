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
        for n in out.graph_predictions:
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
        "readout_ops": plan.readout_ops,
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


WARM_START_VARS = ["kernel.*", "recurrent_kernel.*", "bias.*"]   # FO:127-129


def warm_start(defaults: dict, checkpoint: dict, patterns=WARM_START_VARS, match: str = "component") -> dict:
    """tf.estimator.WarmStartSettings(vars_to_warm_start=["kernel.*", "recurrent_kernel.*",
    "bias.*"]) (FO:126-131) over the model's freshly initialised ``defaults``: a tensor is taken
    from the checkpoint when its name matches one of the regexes; every other tensor keeps its
    initial value.  A checkpoint tensor of another shape raises, as TF's warm start does; a
    checkpoint that lacks a matching tensor leaves it initialised.

    ``match`` says which name the regexes see ("warm start"):
    * ``"component"`` (default): the variable's own name, the last component of the Keras-like
      name (``kernel1`` of ``attention/kernel1``) -- the evident intent of the reference's list;
    * ``"full"``: TF's literal rule.  WarmStartSettings resolves each string through
      ``get_collection(TRAINABLE_VARIABLES, scope=regex)``, i.e. ``re.match`` anchored at the start
      of the FULL variable name.  Every variable of the reference's model is nested under a layer
      scope (``path_update/...``), so under this rule the reference's three patterns select
      nothing and warm start restores no tensor."""
    import re
    if match not in ("component", "full"):
        raise ValueError("warm start: match must be 'component' or 'full', not %r" % (match,))
    out = dict(defaults)
    for name, init in defaults.items():
        key = name if match == "full" else name.split("/")[-1]
        if name not in checkpoint or not any(re.match(p, key) for p in patterns):
            continue
        v = np.asarray(checkpoint[name], np.float32)
        if v.shape != np.shape(init):
            raise ValueError("warm start: %s has shape %s in the checkpoint, the model needs %s"
                             % (name, v.shape, np.shape(init)))
        out[name] = v
    return out


def train_and_evaluate(model, dist=None, device: int = 0, log_every: int = 10):
    """FO:108-166 on the HIP engine.

    The same INI options drive it:
    - ``[PATHS]`` train_dataset, eval_dataset, model_dir (an ``experiment_<datetime>`` subdirectory
      is created, FO:124), warm_start_path (``kernel`` / ``recurrent_kernel`` / ``bias`` tensors,
      FO:126-131);
    - ``[TRAINING_OPTIONS]`` batch_size, train_steps, eval_samples, shuffle_train_samples,
      shuffle_eval_samples, save_checkpoints_secs, keep_checkpoint_max, throttle_secs, and
      ``native_reader`` (default True: the C++ dataset reader; False: the Python generator).

    The Estimator's checkpoint/evaluate cycle becomes:
    - a safetensors checkpoint every ``save_checkpoints_secs`` and at the end;
    - an evaluation of ``eval_samples`` one-graph batches after each checkpoint, at most every
      ``throttle_secs``;
    - metrics appended to ``<model_dir>/metrics.jsonl``.

    ``execute_gpu`` is ignored: in the reference, ``True`` *hides* the GPU (FO:134-145); here
    every step runs on the HIP engine. With ``dist`` (torch.distributed, initialised), each rank
    trains on its slice of every global batch (disjoint samples, one shuffle seed broadcast from
    rank 0) and gradients are averaged by all-reduce."""
    import time

    from .checkpoint import load_params, save_params
    from .training import Trainer

    log.warning("IGNNITION: Starting the training and evaluation process...")
    gm.set_model_info(model)
    opts = CONFIG["TRAINING_OPTIONS"]
    paths = CONFIG["PATHS"]
    batch_size = int(opts.get("batch_size", "1"))
    train_steps = int(opts["train_steps"])
    eval_samples = int(opts.get("eval_samples", "100"))
    save_secs = float(opts.get("save_checkpoints_secs", "600"))
    keep = int(opts.get("keep_checkpoint_max", "5"))
    throttle = float(opts.get("throttle_secs", "600"))
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    model_dir = os.path.join(paths["model_dir"], "experiment_" + str(datetime.datetime.now()).replace(" ", "_"))
    if rank == 0:
        os.makedirs(model_dir, exist_ok=True)
    trainer = Trainer(model, device=device, dist=dist)
    if paths.get("warm_start_path", None):
        trainer.set_params(warm_start(trainer.params(), load_params(paths["warm_start_path"]),
                                      match=opts.get("warm_start_match", "component")))
    native = str_to_bool(opts.get("native_reader", "True"))   # C++ reader
    make_input = gm.input_fn_native if native else gm.input_fn
    # data parallel: one shuffle seed for every rank (rank 0's), each rank reads its slice of
    # every global batch of world * batch_size samples
    seed = int(np.random.SeedSequence().entropy % (2 ** 31))
    if world > 1:
        box = [seed]
        dist.broadcast_object_list(box, src=0)
        seed = int(box[0])
    shuffle_train = str_to_bool(opts.get("shuffle_train_samples", "False"))
    # 8 builders keep a 512-sample synth50 batch stream ahead of the GPU step (bench --train
    # --fresh-batches: 22.2 ms/step fresh vs 22.5 resident)
    workers = int(opts.get("input_workers", str(min(8, len(os.sched_getaffinity(0))))))
    depth = int(opts.get("prefetch_batches", str(workers + 1)))
    if native:   # the gathers, normalisation and host CSR builds of `workers` batches run in parallel
        source = gm.NativeInput(paths["train_dataset"], shuffle=shuffle_train, batch_size=batch_size, seed=seed,
                                rank=rank, world=world)
        prepared = trainer.prefetch(source.ids(), depth=depth, workers=workers, load=source.load)
    else:
        # the training stream shuffles with its own random.Random(seed): the same order on every
        # rank, whatever the eval generator (rank 0, main thread) draws from the global random
        prepared = trainer.prefetch(gm.input_fn(paths["train_dataset"], shuffle=shuffle_train, batch_size=batch_size,
                                                rank=rank, world=world, seed=seed), depth=depth)

    def eval_batches():
        it = make_input(paths["eval_dataset"], shuffle=str_to_bool(opts.get("shuffle_eval_samples", "False")),
                        batch_size=1)
        for _ in range(eval_samples):
            yield next(it)

    ckpts, history = [], []
    last_save = last_eval = time.time()
    metrics = None

    def checkpoint_and_eval(step, force=False):
        nonlocal last_save, last_eval, metrics
        if rank != 0:
            return
        path = os.path.join(model_dir, "ckpt-%d.safetensors" % step)
        save_params(trainer.params(), path, {"step": str(step)})
        ckpts.append(path)
        while len(ckpts) > keep:
            os.remove(ckpts.pop(0))
        last_save = time.time()
        if force or time.time() - last_eval >= throttle:
            metrics = dict(trainer.evaluate(eval_batches()), step=step)
            history.append(metrics)
            with open(os.path.join(model_dir, "metrics.jsonl"), "a") as fh:
                fh.write(json.dumps(metrics) + "\n")
            log.warning("IGNNITION: eval at step %d: %s", step, metrics)
            last_eval = time.time()

    # the next batches are read and built on worker threads while the GPU runs the current step
    try:
        for step in range(1, train_steps + 1):
            logged = step % log_every == 0 or step == 1
            # the loss reaches the host only on the logged steps: the others are enqueued without a
            # wait, so the next batch's host work overlaps this step on the GPU
            out = trainer.train_prepared(*next(prepared), want_loss=logged)
            if rank == 0 and logged:
                log.warning("IGNNITION: step %d  Loss %.6g  Regularization loss %.6g  Total loss %.6g", step,
                            out["loss"], out["regularization_loss"], out["total_loss"])
            if time.time() - last_save >= save_secs:
                checkpoint_and_eval(step)
    finally:
        prepared.close()
    checkpoint_and_eval(train_steps, force=True)
    return {"model_dir": model_dir, "final_metrics": metrics, "history": history, "checkpoints": list(ckpts),
            "trainer": trainer}
