"""Readout-operation cases (GM:605-655, AUX:1033-1265) shared by the forward parity and the
gradient tests: {name: (operations before predict, predict inputs, extra networks)}."""

_POOL = lambda kind, inp, out: {"type": "pooling", "type_pooling": kind, "input": [inp], "output_name": out}
_NN = lambda net, ins, out: {"type": "neural_network", "nn_name": net, "input": list(ins), "output_name": out}
_PROD = lambda a, b, out: {"type": "product", "type_product": "element_wise", "input": [a, b], "output_name": out}
_EXT = {"type": "extend_adjacencies", "adj_list": "adj_paths_links", "input": ["path", "link"],
        "output_name_src": "ep", "output_name_dst": "el"}
READOUT_CASES = {
    "pool_sum": ([_POOL("sum", "path", "g")], ["g"], None),
    "pool_mean": ([_POOL("mean", "link", "g")], ["g"], None),
    "pool_max": ([_POOL("max", "path", "g")], ["g"], None),
    "nn_pool_product": ([_NN("emb", ["path", "path"], "pe"), _POOL("max", "pe", "gmax"), _PROD("gmax", "pe", "prod")],
                        ["prod", "path"], {"emb": [(32, "relu")]}),
    "product_width1": ([_NN("gate", ["path"], "w"), _PROD("path", "w", "gated")], ["gated"], {"gate": [(1, "sigmoid")]}),
    "extend_nn": ([_EXT, _NN("emb", ["ep", "el"], "edge")], ["edge"], {"emb": [(16, "tanh"), (32, "selu")]}),
    "extend_pool": ([_EXT, _PROD("ep", "el", "pl"), _POOL("sum", "pl", "g"), _POOL("mean", "path", "gp")],
                    ["g", "gp"], None),
    "shadow_entity_name": ([_NN("emb", ["path"], "path")], ["path"], {"emb": [(48, "tanh")]}),
}
