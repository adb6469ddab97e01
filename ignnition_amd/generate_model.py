"""Host half of ``code/utils/generate_model.py`` (GM) on top of the HIP engine.

* ``set_model_info``      GM:34-43
* ``normalization``       GM:46-86  user functions resolved *by name* from the user's
                                    namespace (the reference uses ``eval`` on ``from main import *``)
* ``batching_func`` / ``input_fn``  GM:89-198 (a host iterator instead of tf.data)
* ``r_squared``           GM:201-216 (numpy)
* ``ComnetModel``         GM:219-694: construction lowers the plan to ``libignmp.so``;
                          ``__call__`` runs one graph, ``predict_batch`` a disjoint-union
                          batch of graphs (what ``model_fn`` does graph by graph, GM:712-724).
"""

from __future__ import annotations

import logging
import sys

import numpy as np

from .engine import Batch, Engine, MPPlan
from .generator import generator

log = logging.getLogger("ignnition_amd")

model_info = None
user_namespace: dict = {}


def set_model_info(model_description):
    """GM:34-43."""
    global model_info
    model_info = model_description


def register_user_functions(namespace: dict):
    """The reference reaches the user's normalization functions through ``from main import *``
    (GM:24) and ``eval(name)``; here the caller hands its namespace over explicitly."""
    user_namespace.update(namespace)


def _resolve(name):
    if name in user_namespace:
        return user_namespace[name]
    main = sys.modules.get("__main__")
    if main is not None and hasattr(main, name):
        return getattr(main, name)
    raise KeyError(name)


def normalization(x, feature_list, output_name, output_normalization, y=None):
    """GM:46-86."""
    for f in feature_list:
        norm_type = f.normalization
        if str(norm_type) != "None":
            try:
                x[f.name] = _resolve(norm_type)(np.asarray(x[f.name], np.float32), f.name)
            except KeyError:
                log.error("IGNNITION: The normalization function " + str(norm_type) + " is not defined in the main file.")
                sys.exit(1)
    if str(output_normalization) != "None" and y is not None:
        try:
            y = _resolve(output_normalization)(np.asarray(y, np.float32), output_name)
        except KeyError:
            log.error("IGNNITION: The normalization function " + str(output_normalization) +
                      " is not defined in the main file.")
            sys.exit(1)
        return x, y
    return x


def _global_batches(stream, batch_size: int, rank: int, world: int):
    """Batches of a sample stream for rank ``rank`` of ``world`` data-parallel ranks: the stream is
    cut into global batches of ``world * batch_size`` consecutive samples and rank r keeps the r-th
    ``batch_size`` of each, so the ranks of a step train on disjoint samples and every sample of an
    epoch is used once.  Batches run across epoch boundaries, as the reference's
    ``ds.repeat()`` followed by ``batching_func`` (GM:185-194) makes them."""
    import itertools
    while True:
        chunk = list(itertools.islice(stream, world * batch_size))
        mine = chunk[rank * batch_size:(rank + 1) * batch_size]
        if not mine:
            return
        yield mine


def input_fn(data_dir, shuffle=False, training=True, batch_size=1, repeat=True, rank=0, world=1, seed=None):
    """GM:102-198: generator -> normalization -> repeat -> batches of ``batch_size`` graphs.
    ``rank`` / ``world``: data-parallel slice of every global batch (``_global_batches``); the
    ranks must draw the same stream: pass the same ``seed`` on every rank, which gives the stream
    its own ``random.Random`` (reshuffled every epoch from it, untouched by any other draw of the
    process).  ``seed=None`` shuffles with the global ``random``, as the reference does."""
    mi = model_info
    feature_list = mi.get_all_features()
    adjacency_info = mi.get_adjecency_info()
    interleave_list = mi.get_interleave_tensors()
    output_name, output_normalization, _ = mi.get_output_info()
    additional_input = mi.get_additional_input_names()
    unique_additional_input = [a for a in additional_input if a not in [f.name for f in feature_list]]
    feature_names = [f.name for f in feature_list]

    import random
    rng = random.Random(seed) if seed is not None else None

    def stream():
        while True:
            n = 0
            for item in generator(data_dir, feature_names, output_name, adjacency_info, interleave_list,
                                  unique_additional_input, training, shuffle, rng):
                n += 1
                if training:
                    xs, ys = item
                    yield normalization(xs, feature_list, output_name, output_normalization, ys)
                else:
                    yield normalization(item, feature_list, output_name, output_normalization)
            if not repeat or n == 0:
                return

    for batch in _global_batches(stream(), batch_size, rank, world):
        if training:
            yield [b[0] for b in batch], [b[1] for b in batch]
        else:
            yield batch


class NativeInput:
    """input_fn on the native reader (ignnition_amd.dataset), in two halves so that an input
    pipeline can run the second on worker threads:

    * ``ids()``: the sample-id stream (one repeated stream, reshuffled every epoch with ``seed``,
      the same on every data-parallel rank) cut into this rank's batches (``_global_batches``);
    * ``load(ids)``: the native reader's gather (thread safe) and the normalisation functions,
      applied by name to each feature's graph-concatenated array and to the labels (the same
      values as the per-sample call for elementwise functions, those of the examples).  Returns
      a ``BatchedGraphs`` with ``sample_ids``, and the batch's label array when training.

    Iterating yields ``load(ids)`` for every batch of ``ids()``."""

    def __init__(self, data_dir, shuffle=False, training=True, batch_size=1, repeat=True, threads=16, seed=None,
                 rank=0, world=1):
        from .dataset import NativeDataset, plan_keys
        mi = model_info
        self.ds = NativeDataset.for_model(data_dir, mi, training=training, threads=threads)
        self.keys = plan_keys(MPPlan.from_model_info(mi))
        self.feature_list = mi.get_all_features()
        self.output_name, self.output_normalization, _ = mi.get_output_info()
        self.shuffle, self.training, self.batch_size, self.repeat = shuffle, training, batch_size, repeat
        self.rng = np.random.default_rng(seed)
        self.rank, self.world = rank, world

    def ids(self):
        n = len(self.ds)
        if n == 0:
            return

        def id_stream():
            while True:
                yield from (self.rng.permutation(n) if self.shuffle else np.arange(n)).tolist()
                if not self.repeat:
                    return

        yield from _global_batches(id_stream(), self.batch_size, self.rank, self.world)

    def load(self, ids):
        # integer keys as int32 (the batch build reads them at that width: half the gather's bytes)
        bg, labels = self.ds.batch(ids, self.keys, narrow=True)
        bg.sample_ids = list(ids)
        for f in self.feature_list:
            if str(f.normalization) != "None" and f.name in bg:
                v, lens = bg.get(f.name)
                try:
                    fn = _resolve(f.normalization)
                except KeyError:
                    log.error("IGNNITION: The normalization function " + str(f.normalization) +
                              " is not defined in the main file.")
                    sys.exit(1)
                bg.arrays[f.name] = (np.asarray(fn(v, f.name), np.float32), lens)
        if not self.training:
            return bg
        y = labels[0]
        if str(self.output_normalization) != "None":
            y = np.asarray(_resolve(self.output_normalization)(y, self.output_name), np.float32)
        return bg, [y]

    def __iter__(self):
        for ids in self.ids():
            yield self.load(ids)


def input_fn_native(data_dir, shuffle=False, training=True, batch_size=1, repeat=True, threads=16, seed=None,
                    rank=0, world=1):
    """input_fn on the native reader: an iterator over ``NativeInput(...)`` (BatchedGraphs, and
    the label arrays when training)."""
    return iter(NativeInput(data_dir, shuffle, training, batch_size, repeat, threads, seed, rank, world))


def r_squared(labels, predictions):
    """GM:201-216 (value of the streaming mean for one batch)."""
    labels = np.asarray(labels, np.float64)
    predictions = np.asarray(predictions, np.float64)
    total_error = np.sum(np.square(labels - labels.mean()))
    unexplained_error = np.sum(np.square(labels - predictions))
    return 1.0 - unexplained_error / total_error


class ComnetModel:
    """GM:219-694, executed by the HIP engine."""

    def __init__(self, model_description=None, device: int = 0, params: dict | None = None, seed: int = 0):
        mi = model_description if model_description is not None else model_info
        if mi is None:
            raise RuntimeError("set_model_info() first (GM:34)")
        self.model_info = mi
        self.plan = MPPlan.from_model_info(mi)
        self.engine = Engine(self.plan, device)
        self.params = params if params is not None else self.plan.init_params(seed)
        self.engine.set_params(self.params)

    def set_params(self, params: dict):
        self.params = params
        self.engine.set_params(params)

    @property
    def trainable_variables(self):
        return self.params

    @property
    def losses(self):
        """Keras ``model.losses``: l2 terms of the readout kernel_regularizers (AUX:833-834)."""
        out = []
        for (name, _, _, _, l2), (pname, _) in zip(self.plan.dense, [s for s in self.plan.param_specs()
                                                                      if s[0].startswith("readout_model_%d/" % self.plan.predict_counter)
                                                                      and s[0].endswith("/kernel")]):
            if l2:
                w = np.asarray(self.params[pname], np.float64)
                out.append(l2 * float((w * w).sum()))
        return out

    def batch(self, graphs) -> Batch:
        """``graphs``: a list of feature dicts or a ``BatchedGraphs`` (native reader)."""
        return Batch(self.engine, graphs)

    def predict_batch(self, graphs: list) -> np.ndarray:
        """Flattened predictions of every graph, concatenated in batch order (GM:716-724)."""
        return self.batch(graphs).forward().reshape(-1)

    def __call__(self, input: dict, training: bool = False) -> np.ndarray:
        """``ComnetModel.call`` (GM:384) for one graph: [P, units] predictions."""
        return self.batch([input]).forward()
