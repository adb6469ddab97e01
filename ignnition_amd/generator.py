"""Index builder: samples -> the reference's feature-dict contract.

Restates ``code/utils/generator_std_to_framework.py`` (GEN) on plain Python/numpy:

* ``make_indices``          GEN:32-50   rank of each node within its entity type, in
                                        ``entities`` dict order (JSON key order).
* ``sample_to_data``        GEN:97-219  one sample -> ``src_<adj>``, ``dst_<adj>``,
                                        ``seq_<srcEnt>_<dstEnt>``, ``params_<adj>``,
                                        ``num_<entity>``, ``indices_<src>_to_<dst>``.
* ``generator``             GEN:53-230  walks ``<dir>/*.tar.gz`` -> ``data.json``.

The arrays it emits are the bit-exact index contract the HIP engine consumes
(tests/test_generator.py pins them against fixtures produced by the reference itself).
Quirks kept on purpose: destination groups follow JSON key order (GEN:145), the
``seq_`` key is per entity pair so two adjacencies between the same entities collide
(GEN:181), the params branch skips the source-type check (GEN:156-163), and a file
whose sample raises is abandoned after logging (GEN:229-230).
"""

from __future__ import annotations

import glob
import json
import logging
import math
import random
import tarfile

import numpy as np

log = logging.getLogger("ignnition_amd")


def make_indices(entities: dict):
    """GEN:32-50 — per-type counters and the per-node rank within its type."""
    counter: dict = {}
    indices: dict = {}
    for node, entity in entities.items():
        if entity not in counter:
            counter[entity] = 0
        indices[node] = counter[entity]
        counter[entity] += 1
    return counter, indices


def _s(x):
    return x.decode("ascii") if isinstance(x, (bytes, bytearray)) else x


def sample_to_data(sample: dict, feature_names, output_name, adj_names, interleave_names,
                   additional_input, training: bool):
    """GEN:97-224 for one sample.  Returns ``data`` (and ``output`` when training)."""
    data: dict = {}
    output: list = []

    for f in feature_names:                                   # GEN:102-107
        if f not in sample:
            raise Exception('A list for feature named "' + str(f) + '" was not found although being expected.')
        data[f] = sample[f]

    for a in additional_input:                                # GEN:110-114
        if a not in sample:
            raise Exception('The input name "' + str(a) + '" was not found although being expected.')
        data[a] = sample[a]

    if training:                                              # GEN:117-126
        if output_name not in sample:
            raise Exception('A list for the output named "' + str(output_name) +
                            '" was not found although being expected.')
        value = sample[output_name]
        if not isinstance(value, list):
            value = [value]
        output += value

    seq_by_pair: dict = {}
    entities = sample["entities"]
    num_nodes, indices = make_indices(entities)

    for a in adj_names:                                       # GEN:134-185
        name, src_entity, dst_entity, uses_parameters = a
        if name not in sample:
            raise Exception('A list for the adjecency vector named "' + name +
                            '" was not found although being expected.')
        adjacency_lists = sample[name]
        src_idx, dst_idx, seq, parameters = [], [], [], []
        for destination, sources in adjacency_lists.items():
            if entities[destination] != dst_entity:
                raise Exception('The adjecency list "' + name + '" was expected to be from ' + src_entity +
                                ' to ' + dst_entity + '.\n However, "' + destination +
                                '" was found which is of type "' + entities[destination] +
                                '" instead of ' + dst_entity)
            seq += range(0, len(sources))
            if isinstance(sources[0], list):                  # edge parameters present
                for s in sources:
                    src_idx.append(indices[s[0]])
                    dst_idx.append(indices[destination])
                    if uses_parameters == "True":
                        parameters.append(s[1])
            else:
                for s in sources:
                    if entities[s] != src_entity:
                        raise Exception('The adjecency list "' + name + '" was expected to be from "' +
                                        src_entity + '" to "' + dst_entity + '.\n However, "' + destination +
                                        '" was found which is of type "' + entities[destination] +
                                        '" instead of "' + src_entity)
                    src_idx.append(indices[s])
                    dst_idx.append(indices[destination])
        data["src_" + name] = src_idx
        data["dst_" + name] = dst_idx
        data["seq_" + src_entity + "_" + dst_entity] = seq
        seq_by_pair["seq_" + src_entity + "_" + dst_entity] = seq
        if parameters != []:
            data["params_" + name] = parameters

    for entity, n_nodes in num_nodes.items():                 # GEN:188-190
        data["num_" + entity] = n_nodes

    for name, dst_entity in interleave_names:                 # GEN:193-219
        interleave_definition = sample[name]
        involved: dict = {}
        total_sequence = []
        total_size, n_total, counter = 0, 0, 0
        for entity in interleave_definition:
            total_size += 1
            if entity not in involved:
                involved[entity] = counter
                s = seq_by_pair["seq_" + entity + "_" + dst_entity]
                n_total += max(s) + 1
                counter += 1
            total_sequence.append(involved[entity])
        repetitions = math.ceil(float(n_total) / total_size)
        result = np.array((total_sequence * repetitions)[:n_total])
        for entity, ident in involved.items():
            data["indices_" + entity + "_to_" + dst_entity] = np.where(result == ident)[0].tolist()

    if training:
        return data, output
    return data


def generator(dir, feature_names, output_name, adj_names, interleave_names, additional_input,
              training, shuffle=False, rng=None):
    """GEN:53-230.  Accepts str or bytes arguments (the reference receives bytes from tf.data).
    ``rng``: a ``random.Random`` for the shuffle (default: the process-global ``random``, as GEN);
    a data-parallel input stream passes its own so that no other thread or rank's draws move it."""
    dir = _s(dir)
    feature_names = [_s(x) for x in feature_names]
    output_name = _s(output_name)
    adj_names = [[_s(x[0]), _s(x[1]), _s(x[2]), _s(x[3])] for x in adj_names]
    interleave_names = [[_s(i[0]), _s(i[1])] for i in interleave_names]
    additional_input = [_s(x) for x in additional_input]
    # glob order is filesystem order in the reference; sorted here so runs are reproducible.
    samples = sorted(glob.glob(str(dir) + "/*.tar.gz"))
    if shuffle:
        (rng or random).shuffle(samples)
    for sample_file in samples:
        try:
            with tarfile.open(sample_file, "r:gz") as tar:
                try:
                    fh = tar.extractfile("data.json")
                except KeyError:
                    raise SystemExit("IGNNITION: The file data.json was not found in " + sample_file)
                file_samples = json.load(fh)
            for sample in file_samples:
                yield sample_to_data(sample, feature_names, output_name, adj_names, interleave_names,
                                     additional_input, training)
        except KeyboardInterrupt:
            raise SystemExit(1)
        except SystemExit:
            raise
        except Exception as inf:                              # GEN:229-230: log, skip rest of file
            log.error("IGNNITION: " + str(inf))


def read_first_sample(path: str) -> dict:
    """First sample of the first archive (used by find_dataset_dimensions, FO:58-67)."""
    sample = sorted(glob.glob(str(path) + "/*.tar.gz"))[0]
    with tarfile.open(sample, "r:gz") as tar:
        return json.load(tar.extractfile("data.json"))[0]
