"""``Model_information``: the model plan parsed from ``model_description.json``.

Restates ``code/utils/json_operations.py`` (JO) with identical getters so the rest
of the host code (and users' scripts) read it the same way:

* construction order JO:128-149 (read -> schema validate -> semantic validate ->
  inject dimensions -> nn mapping -> entities -> iterations -> mp instances ->
  readout -> training options -> input dims),
* ``__validate_model_description`` JO:184-245 (including its quirk at JO:214 where
  ``op['type'] == ('predict' or 'neural_network')`` only matches ``predict``),
* ``__add_nn_architecture`` JO:270-300 (nn_name resolved into the op, recurrent
  extras copied into the update dict),
* getters JO:384-475.

Schema validation uses :mod:`ignnition_amd.schema` (a restatement of SCH, since
``jsonschema`` is absent).  Errors log and exit like the reference (JO:243-245).
"""

from __future__ import annotations

import copy
import json
import logging
import sys
from functools import reduce

from . import schema
from .auxilary_classes import (Entity, Extend_adjacencies, Interleave_aggr, Message_Passing,
                               Pooling_operation, Predicting_operation, Product_operation, Readout_nn)

log = logging.getLogger("ignnition_amd")


class Model_information:
    def __init__(self, path, dimensions):
        data = self._read_json(path)
        schema.validate(data)
        self._validate_model_description(data)
        self._add_dimensions(data, dimensions)

        self.nn_architectures = self._get_nn_mapping(data["neural_networks"])
        self.entities = self._get_entities(data["entities"])
        self.iterations_mp = int(data["message_passing"]["num_iterations"])
        self.mp_instances = self._get_mp_instances(data["message_passing"]["stages"])
        self.readout_op = self._get_readout_op(data["readout"])
        self.training_op = self._get_training_op(data)
        self.input_dim = self._get_input_dims(dimensions)

    # ---------------------------------------------------------------- private
    @staticmethod
    def _read_json(path):
        if isinstance(path, dict):
            return copy.deepcopy(path)
        with open(path) as fh:
            return json.load(fh)

    @staticmethod
    def _add_dimensions(data, dimensions):
        """JO:162-180."""
        for e in data["entities"]:
            for f in e["features"]:
                f["size"] = dimensions[f["name"]]
        for stage in data["message_passing"]["stages"]:
            for mp in stage["stage_mp"]:
                for src in mp["source_entities"]:
                    src["extra_parameters"] = dimensions[src["adj_vector"]]

    @staticmethod
    def _validate_model_description(data):
        """JO:184-245."""
        stages = data["message_passing"]["stages"]
        src_names, dst_names, called_nn_names, input_names = [], [], [], []
        output_names = ["hs_source", "hs_dest", "edge_params"]
        for stage in stages:
            for mp in stage["stage_mp"]:
                dst_names.append(mp["destination_entity"])
                for src in mp["source_entities"]:
                    src_names.append(src["name"])
                    for op in src["message"]:
                        if op["type"] == "neural_network":
                            called_nn_names.append(op["nn_name"])
                            input_names += op["input"]
                        if "output_name" in op:
                            output_names.append(op["output_name"])
        readout_op = data["readout"]
        # JO:214 quirk: ('predict' or 'neural_network') == 'predict'.
        called_nn_names += [op["nn_name"] for op in readout_op if op["type"] == "predict"]
        entity_names = [a["name"] for a in data["entities"]]
        nn_names = [n["nn_name"] for n in data["neural_networks"]]
        try:
            for a in src_names:
                if a not in entity_names:
                    raise Exception("The source entity " + a + " was used in a message passing. However, there is"
                                    " no such entity. \n Please check the spelling or define a new entity.")
            for d in dst_names:
                if d not in entity_names:
                    raise Exception("The destination entity " + d + " was used in a message passing. However, there"
                                    " is no such entity. \n Please check the spelling or define a new entity.")
            for name in called_nn_names:
                if name not in nn_names:
                    raise Exception("The name " + name + " is used as a reference to a neural network (nn_name), even"
                                    " though the neural network was not defined. \n Please make sure the name is"
                                    " correctly spelled or define a neural network named " + name)
            for i in input_names:
                if i not in output_names:
                    raise Exception("The name " + i + " was used as input of a message creation operation even"
                                    " though it wasn't the output of one.")
        except Exception as inf:
            log.error("IGNNITION: " + str(inf) + "\n")
            sys.exit(1)

    @staticmethod
    def _get_nn_mapping(models):
        return {m["nn_name"]: m for m in models}

    @staticmethod
    def _get_entities(entities):
        return [Entity(e) for e in entities]

    def _add_nn_architecture(self, m):
        """JO:270-300."""
        for s in m["source_entities"]:
            for op in s["message"]:
                if op["type"] == "neural_network":
                    info = copy.deepcopy(self.nn_architectures[op["nn_name"]])
                    del op["nn_name"]
                    op["architecture"] = info["nn_architecture"]
        if "update" in m:
            if m["update"]["type"] == "neural_network":
                info = copy.deepcopy(self.nn_architectures[m["update"]["nn_name"]])
                del m["update"]["nn_name"]
                m["update"]["architecture"] = info["nn_architecture"]
            if m["update"]["type"] == "recurrent_neural_network":
                arch = copy.deepcopy(self.nn_architectures[m["update"]["nn_name"]])
                del m["update"]["nn_name"]
                for k, v in arch.items():
                    if k != "nn_name" and k != "nn_type":
                        m["update"][k] = v
        return m

    def _get_mp_instances(self, inst):
        return [[step["stage_name"], [Message_Passing(self._add_nn_architecture(m)) for m in step["stage_mp"]]]
                for step in inst]

    def _add_readout_architecture(self, output):
        info = copy.deepcopy(self.nn_architectures[output["nn_name"]])
        del output["nn_name"]
        output["architecture"] = info["nn_architecture"]
        return output

    def _get_readout_op(self, output_operations):
        """JO:326-350."""
        result = []
        for op in output_operations:
            t = op["type"]
            if t == "predict":
                result.append(Predicting_operation(self._add_readout_architecture(op)))
            elif t == "pooling":
                result.append(Pooling_operation(op))
            elif t == "product":
                result.append(Product_operation(op))
            elif t == "neural_network":
                result.append(Readout_nn(self._add_readout_architecture(op)))
            elif t == "extend_adjacencies":
                result.append(Extend_adjacencies(op))
        return result

    @staticmethod
    def _get_training_op(data):
        train_hp = data["learning_options"]
        return {"loss": train_hp["loss"], "optimizer": train_hp["optimizer"]}

    def _get_input_dims(self, dimensions):
        d = {e.name: e.hidden_state_dimension for e in self.entities}
        return {**d, **dimensions}

    # ---------------------------------------------------------------- getters
    def get_input_dimensions(self):
        return self.input_dim

    def get_entities(self):
        return self.entities

    def get_interleave_sources(self):
        aux = [[[src.name, mp.destination_entity] for src in mp.source_entities]
               for _, mps in self.mp_instances for mp in mps if isinstance(mp.aggregation, Interleave_aggr)]
        return reduce(lambda accum, a: accum + a, aux, [])

    def get_mp_iterations(self):
        return self.iterations_mp

    def get_interleave_tensors(self):
        return [[mp.aggregation.combination_definition, mp.destination_entity]
                for _, mps in self.mp_instances for mp in mps if isinstance(mp.aggregation, Interleave_aggr)]

    def get_mp_instances(self):
        return self.mp_instances

    def get_optimizer(self):
        return self.training_op["optimizer"]

    def get_loss(self):
        return self.training_op["loss"]

    def get_readout_operations(self):
        return self.readout_op

    def get_output_info(self):
        preds = [o for o in self.readout_op if o.type == "predict"]
        return preds[0].label, preds[0].label_normalization, preds[0].label_denormalization

    def get_all_features(self):
        return reduce(lambda accum, e: accum + e.features, self.entities, [])

    @staticmethod
    def get_feature_size(feature):
        return feature["size"] if "size" in feature else 1

    def get_adjecency_info(self):
        aux = [instance.get_instance_info() for step in self.mp_instances for instance in step[1]]
        return reduce(lambda accum, a: accum + a, aux, [])

    def get_additional_input_names(self):
        output_names, input_names = set(), set()
        for r in self.readout_op:
            if r.type == "extend_adjacencies":
                output_names.update(r.output_name)
            elif r.type != "predict":
                output_names.add(r.output_name)
            for i in r.input:
                input_names.add(i)
        for e in self.entities:
            output_names.add(e.name)
        return list(input_names.difference(output_names))
