"""Model-description descriptor objects (no TensorFlow).

Mirrors the *descriptor* half of ``code/utils/auxilary_classes.py`` (AUX): the same
class names, attributes and parsing rules, so a ``Model_information`` built here
answers the same getters as the reference's.  The TF/Keras *execution* half
(``calculate_hs``, ``calculate_input``, ``perform_*_update``, ``construct_tf_model``)
is not restated here: the HIP engine (``ignnition_amd/csrc``) executes it.

Cited reference lines: Feature AUX:28-59, Entity AUX:62-125, Operation/Apply_nn/Apply_rnn
AUX:163-226, aggregations AUX:229-456, Message_Passing AUX:458-561, Source_Entity
AUX:641-698, Recurrent_Cell AUX:702-750, Feed_forward_Layer/model AUX:799-1003,
readout operations AUX:1033-1234.
"""

from __future__ import annotations


class Feature:
    """AUX:28-59."""

    def __init__(self, f):
        self.name = f["name"]
        self.size = 1
        self.normalization = "None"
        if "size" in f:
            self.size = f["size"]
        if "normalization" in f:
            self.normalization = f["normalization"]


class Entity:
    """AUX:62-125.  ``calculate_hs`` (AUX:128-160) runs on the GPU (init_state kernel)."""

    def __init__(self, d):
        self.name = d["name"]
        self.hidden_state_dimension = d["hidden_state_dimension"]
        self.features = []
        if "features" in d:
            self.features = [Feature(f) for f in d["features"]]

    def get_entity_total_feature_size(self):
        # AUX:107-112 calls a non-existent Feature.get_size(); fixed here.
        return sum(int(f.size) for f in self.features)

    def get_features_names(self):
        return [f.name for f in self.features]

    def add_feature(self, f):
        self.features.append(f)


class Operation:
    """AUX:163-174."""

    def __init__(self, type):
        self.type = type


class Apply_nn(Operation):
    """AUX:177-205 — message-creation / feed-forward update network."""

    def __init__(self, op, counter=0):
        super().__init__(type="feed_forward_nn")
        if "input" in op:
            self.input = op["input"]
        self.output_name = op["output_name"] if "output_name" in op else "None"
        self.model = Feed_forward_message_creation(op["architecture"], counter, 0)


class Apply_rnn(Operation):
    """AUX:208-226."""

    def __init__(self, op):
        super().__init__(type="recurrent_nn")
        del op["type"]
        recurrent_type = op["recurrent_type"]
        del op["recurrent_type"]
        self.model = Recurrent_Cell(recurrent_type, op)


class Aggregation:
    """AUX:229-239 (also the plain ``ordered`` aggregation, AUX:561)."""

    def __init__(self, d):
        self.type = d["type"]


class Sum_aggr(Aggregation):
    """AUX:241-262."""


class Attention_aggr(Aggregation):
    """AUX:264-344."""


class Conv_aggr(Aggregation):
    """AUX:347-401."""

    def __init__(self, d):
        super().__init__(d)
        self.activation_function = d.get("activation_function", "relu")


class Interleave_aggr(Aggregation):
    """AUX:406-440."""

    def __init__(self, d):
        super().__init__(d)
        self.combination_definition = d["interleave_definition"]


class Concat_aggr(Aggregation):
    """AUX:443-456."""

    def __init__(self, d):
        super().__init__(d)
        self.concat_axis = int(d["concat_axis"])


class Source_Entity:
    """AUX:641-698."""

    def __init__(self, d):
        self.name = d["name"]
        self.adj_vector = d["adj_vector"]
        self.message_formation = (self.create_message_formation(d["message"]) if "message" in d
                                  else [Operation("direct_assignation")])
        self.extra_parameters = d["extra_parameters"]

    def create_message_formation(self, operations):
        result = []
        counter = 0
        for op in operations:
            if op["type"] == "neural_network":
                result.append(Apply_nn(op, counter))
            if op["type"] == "direct_assignation":
                result.append(Operation("direct_assignation"))
            counter += 1
        return result

    def get_instance_info(self, dst_name):
        """AUX:690-698: [adj_vector, src, dst, 'True'|'False' (has edge params)]."""
        return [self.adj_vector, self.name, dst_name, str(self.extra_parameters > 0)]


class Message_Passing:
    """AUX:458-561."""

    def __init__(self, m):
        self.destination_entity = m["destination_entity"]
        self.source_entities = [Source_Entity(s) for s in m["source_entities"]]
        self.aggregation = self.create_aggregation(m["aggregation"])
        self.update = self.create_update(m["update"])

    def create_update(self, u):
        if u["type"] == "neural_network":
            return Apply_nn({"architecture": u["architecture"]})
        if u["type"] == "recurrent_neural_network":
            return Apply_rnn(u)

    def create_aggregation(self, d):
        t = d["type"]
        if t == "interleave":
            return Interleave_aggr(d)
        if t == "concat":
            return Concat_aggr(d)
        if t == "sum":
            return Sum_aggr(d)
        if t == "attention":
            return Attention_aggr(d)
        if t == "convolution":
            return Conv_aggr(d)
        return Aggregation(d)

    def get_instance_info(self):
        return [src.get_instance_info(self.destination_entity) for src in self.source_entities]


class Recurrent_Cell:
    """AUX:702-750.  ``type`` is the Keras cell family (GRU); ``parameters`` the extra kwargs."""

    def __init__(self, type, parameters):
        self.type = type
        self.parameters = parameters

    def get_cell_spec(self, destination_dimension):
        """Counterpart of ``get_tensorflow_object`` (AUX:740-750): units = dst hidden dim."""
        self.parameters["units"] = destination_dimension
        return {"type": self.type, **self.parameters}


class Feed_forward_Layer:
    """AUX:799-865.  Keeps the raw layer kwargs; ``kernel_regularizer`` becomes an l2 float."""

    def __init__(self, type, parameters):
        self.type = type
        self.parameters = parameters
        if "kernel_regularizer" in parameters:
            self.parameters["kernel_regularizer"] = float(parameters["kernel_regularizer"])
        if "activation" in parameters and parameters["activation"] == "None":
            self.parameters["activation"] = None


class Feed_forward_model:
    """AUX:869-1003 (layer list only; ``construct_tf_model`` is the engine's job)."""

    def __init__(self, model, model_role):
        self.layers = []
        self.counter = 0
        if "architecture" in model:
            for l in model["architecture"]:
                type_layer = l["type_layer"]
                if "name" not in l:
                    l["name"] = "layer_" + str(self.counter) + "_" + type_layer + "_" + str(model_role)
                del l["type_layer"]
                self.layers.append(Feed_forward_Layer(type_layer, l))
                self.counter += 1

    def add_layer_aux(self, l):
        type_layer = l["type_layer"]
        del l["type_layer"]
        self.layers.append(Feed_forward_Layer(type_layer, l))


class Feed_forward_message_creation(Feed_forward_model):
    """AUX:1006-1030."""

    def __init__(self, architecture, counter, num_parameter):
        super().__init__({"architecture": architecture}, model_role="message_creation_" + str(counter))
        self.num_extra_parameters = num_parameter


class Readout_operation:
    """AUX:1033-1051."""

    def __init__(self, op):
        self.type = op["type"]
        self.input = op["input"]
        self.output_name = None


class Product_operation(Readout_operation):
    """AUX:1054-1094."""

    def __init__(self, op):
        super().__init__(op)
        self.type_product = op["type_product"]
        self.output_name = op["output_name"]


class Predicting_operation(Readout_operation):
    """AUX:1097-1133."""

    def __init__(self, operation):
        super().__init__(operation)
        self.architecture = Feed_forward_model({"architecture": operation["architecture"]},
                                               model_role="readout")
        self.label = operation["label"]
        self.label_normalization = operation.get("label_normalization", None)
        self.label_denormalization = operation.get("label_denormalization", None)


class Pooling_operation(Readout_operation):
    """AUX:1136-1185."""

    def __init__(self, operation):
        super().__init__(operation)
        self.type_pooling = operation["type_pooling"]
        self.output_name = operation["output_name"]


class Readout_nn(Readout_operation):
    """AUX:1188-1211."""

    def __init__(self, op):
        super().__init__(op)
        if "input" in op:
            self.input = op["input"]
        self.output_name = op["output_name"] if "output_name" in op else "None"
        self.architecture = Feed_forward_model({"architecture": op["architecture"]}, model_role="readout")


class Extend_adjacencies(Readout_operation):
    """AUX:1214-1234."""

    def __init__(self, op):
        super().__init__({"type": op["type"], "input": op["input"]})
        self.adj_list = op["adj_list"]
        self.output_name = [op["output_name_src"], op["output_name_dst"]]
