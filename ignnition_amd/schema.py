"""Structural validation of ``model_description.json``.

Restates the constraints of ``code/utils/schema.json`` (SCH, JSON-Schema draft-07,
applied at JO:138-139) as plain Python checks, because ``jsonschema`` is not
available in this image.  Only the constraints SCH actually states are checked:
types, enums, ``required`` lists and the if/then conditionals (including the
reference's own ``extend_adjecencies`` spelling at SCH:367, which makes that
conditional dead — kept as-is).
"""

from __future__ import annotations


class SchemaError(ValueError):
    pass


def _req(obj, keys, where):
    for k in keys:
        if k not in obj:
            raise SchemaError("%s: '%s' is a required property" % (where, k))


def _type(v, t, where):
    ok = {
        "object": isinstance(v, dict),
        "array": isinstance(v, list),
        "string": isinstance(v, str),
        "number": isinstance(v, (int, float)) and not isinstance(v, bool),
        "integer": isinstance(v, int) and not isinstance(v, bool),
    }[t]
    if not ok:
        raise SchemaError("%s: %r is not of type '%s'" % (where, v, t))


def _enum(v, values, where):
    if v not in values:
        raise SchemaError("%s: %r is not one of %r" % (where, v, values))


def _opt(obj, key, t, where):
    if key in obj:
        _type(obj[key], t, where + "." + key)


def validate(instance: dict) -> None:
    _type(instance, "object", "$")

    if "entities" in instance:                                        # SCH:8-50
        ents = instance["entities"]
        _type(ents, "array", "entities")
        seen = []
        for i, e in enumerate(ents):
            w = "entities[%d]" % i
            _type(e, "object", w)
            if e in seen:
                raise SchemaError("entities: items are not unique")
            seen.append(e)
            _opt(e, "name", "string", w)
            if "hidden_state_dimension" in e:
                _type(e["hidden_state_dimension"], "number", w + ".hidden_state_dimension")
                if not e["hidden_state_dimension"] > 0:
                    raise SchemaError(w + ".hidden_state_dimension must be > 0")
            if "features" in e:
                _type(e["features"], "array", w + ".features")
                for j, f in enumerate(e["features"]):
                    wf = w + ".features[%d]" % j
                    _type(f, "object", wf)
                    _opt(f, "name", "string", wf)
                    _opt(f, "normalization", "string", wf)
                    _req(f, ["name"], wf)
            _req(e, ["name", "hidden_state_dimension", "features"], w)

    if "message_passing" in instance:                                 # SCH:51-230
        mp = instance["message_passing"]
        _type(mp, "object", "message_passing")
        if "num_iterations" in mp:
            _type(mp["num_iterations"], "number", "message_passing.num_iterations")
            if not mp["num_iterations"] > 0:
                raise SchemaError("message_passing.num_iterations must be > 0")
        if "stages" in mp:
            _type(mp["stages"], "array", "message_passing.stages")
            for si, st in enumerate(mp["stages"]):
                w = "stages[%d]" % si
                _type(st, "object", w)
                _opt(st, "stage_name", "string", w)
                if "stage_mp" in st:
                    _type(st["stage_mp"], "array", w + ".stage_mp")
                    for mi, m in enumerate(st["stage_mp"]):
                        _validate_mp(m, w + ".stage_mp[%d]" % mi)
                _req(st, ["stage_name", "stage_mp"], w)
        _req(mp, ["num_iterations", "stages"], "message_passing")

    if "readout" in instance:                                         # SCH:231-352
        ro = instance["readout"]
        _type(ro, "array", "readout")
        for i, op in enumerate(ro):
            w = "readout[%d]" % i
            _type(op, "object", w)
            if "type" in op:
                _type(op["type"], "string", w + ".type")
                _enum(op["type"], ["predict", "pooling", "product", "neural_network", "extend_adjacencies"],
                      w + ".type")
            if "type_pooling" in op:
                _enum(op["type_pooling"], ["sum", "max", "mean"], w + ".type_pooling")
            if "type_product" in op:
                _enum(op["type_product"], ["dot_product", "element_wise"], w + ".type_product")
            if "input" in op:
                _type(op["input"], "array", w + ".input")
                for x in op["input"]:
                    _type(x, "string", w + ".input[]")
            for k in ("label", "label_normalization", "label_denormalization", "nn_name", "output_name",
                      "output_name_src", "output_name_dst", "adj_list"):
                _opt(op, k, "string", w)
            t = op.get("type")
            if t == "predict":
                _req(op, ["nn_name", "label"], w)
            elif t == "pooling":
                _req(op, ["type_pooling", "output_name"], w)
            elif t == "product":
                _req(op, ["type_product", "output_name"], w)
            elif t == "neural_network":
                _req(op, ["nn_name", "output_name"], w)
            # SCH:367 tests the misspelt const "extend_adjecencies": never triggers.
            _req(op, ["input"], w)

    if "neural_networks" in instance:                                 # SCH:353-423
        nns = instance["neural_networks"]
        _type(nns, "array", "neural_networks")
        for i, nn in enumerate(nns):
            w = "neural_networks[%d]" % i
            _type(nn, "object", w)
            _opt(nn, "nn_name", "string", w)
            if "nn_type" in nn:
                _enum(nn["nn_type"], ["feed_forward", "recurrent_neural_network"], w + ".nn_type")
            if "recurrent_type" in nn:
                _enum(nn["recurrent_type"], ["GRU", "LSTM"], w + ".recurrent_type")
            if "nn_architecture" in nn:
                _type(nn["nn_architecture"], "array", w + ".nn_architecture")
                for j, l in enumerate(nn["nn_architecture"]):
                    _type(l, "object", w + ".nn_architecture[%d]" % j)
                    _opt(l, "type_layer", "string", w)
                    _opt(l, "name", "string", w)
            if nn.get("nn_type") == "feed_forward":
                _req(nn, ["nn_architecture"], w)
            else:
                _req(nn, ["recurrent_type"], w)
            _req(nn, ["nn_name", "nn_type"], w)

    if "learning_options" in instance:                                # SCH:424-488
        lo = instance["learning_options"]
        _type(lo, "object", "learning_options")
        _opt(lo, "loss", "string", "learning_options")
        if "optimizer" in lo:
            _type(lo["optimizer"], "object", "learning_options.optimizer")
            _opt(lo["optimizer"], "type", "string", "learning_options.optimizer")
            if "schedule" in lo["optimizer"]:
                _type(lo["optimizer"]["schedule"], "object", "learning_options.optimizer.schedule")
                _opt(lo["optimizer"]["schedule"], "type", "string", "learning_options.optimizer.schedule")
        _req(lo, ["loss", "optimizer"], "learning_options")


def _validate_mp(m, w):
    _type(m, "object", w)
    _opt(m, "destination_entity", "string", w)
    if "source_entities" in m:
        _type(m["source_entities"], "array", w + ".source_entities")
        for i, s in enumerate(m["source_entities"]):
            ws = w + ".source_entities[%d]" % i
            _type(s, "object", ws)
            _opt(s, "name", "string", ws)
            _opt(s, "adj_vector", "string", ws)
            if "message" in s:
                _type(s["message"], "array", ws + ".message")
                for j, op in enumerate(s["message"]):
                    wo = ws + ".message[%d]" % j
                    _type(op, "object", wo)
                    if "type" in op:
                        _enum(op["type"], ["neural_network", "direct_assignation"], wo + ".type")
                    _opt(op, "nn_name", "string", wo)
                    _opt(op, "input", "array", wo)
                    _opt(op, "output_name", "string", wo)
                    if op.get("type") == "neural_network":
                        _req(op, ["nn_name", "input"], wo)
                    _req(op, ["type"], wo)
            _req(s, ["name", "adj_vector", "message"], ws)
    if "aggregation" in m:
        a = m["aggregation"]
        _type(a, "object", w + ".aggregation")
        if "type" in a:
            _enum(a["type"], ["sum", "ordered", "attention", "concat", "interleave", "convolution"],
                  w + ".aggregation.type")
        if "concat_axis" in a:
            _type(a["concat_axis"], "integer", w + ".aggregation.concat_axis")
            _enum(a["concat_axis"], [1, 2], w + ".aggregation.concat_axis")
        _opt(a, "interleave_definition", "string", w + ".aggregation")
        _opt(a, "activation_function", "string", w + ".aggregation")
        if a.get("type") == "interleave":
            _req(a, ["interleave_definition"], w + ".aggregation")
        if a.get("type") == "concat":
            _req(a, ["concat_axis"], w + ".aggregation")
    if "update" in m:
        u = m["update"]
        _type(u, "object", w + ".update")
        if "type" in u:
            _enum(u["type"], ["neural_network", "recurrent_neural_network"], w + ".update.type")
        _opt(u, "nn_name", "string", w + ".update")
        if u.get("type") in ("neural_network", "recurrent_neural_network"):
            _req(u, ["nn_name"], w + ".update")
    _req(m, ["source_entities", "destination_entity", "aggregation", "update"], w)
