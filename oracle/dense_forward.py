"""ORACLE (test infrastructure only) — dense-padded CPU restatement of ComnetModel.call.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / the timed CPU baseline.  The product path
(ignnition_amd/) never imports it and has no CPU execution path.

It follows the reference's TensorFlow op sequence literally, one graph at a time
(model_fn calls the model per graph, code/utils/generate_model.py:712-724 = GM):

  hidden states        AUX:146-159   concat(features reshaped [num, size]) | zeros
  message passing      GM:404-603    for T iterations, stages, MPs, sources:
    gather               GM:432      msgs = state_src[src_idx]
    combine              GM:479-490  lens = unsorted_segment_sum(1, dst); Lmax = max(seq)+1;
                                     s = scatter_nd([dst, seq], msgs, [N, Lmax, H]) (adds duplicates)
    multi-source         GM:496-543  concat on axis 1 (sum/ordered, concat), or stack of the
                                     interleave index lists (interleave); final_len = sum(lens)
    aggregation          AUX:254-262 sum over axis 1;  AUX:421-440 interleave = transpose,
                                     scatter_nd by the flattened index list, transpose
    update               AUX:752-765 GRUCell on every destination (sum);
                         AUX:767-796 RNN(GRUCell) with sequence_mask(final_len), then
                                     gather_nd(outputs, [d, final_len-1])
  readout              GM:605-655   neural_network / pooling / element-wise product /
                                     extend_adjacencies, then predict: concat inputs on axis 1,
                                     Dense stack (AUX:833-837)

TF / Keras math (not in the reference repo, restated from their published definitions):
GRUCell v2 defaults (tanh / sigmoid, reset_after=True, gate order z, r, h); Dense
y = act(x W + b); selu with lambda=1.0507009873554805, alpha=1.6732632423543772.

Parity status: INDEX contract pinned bit-exact against the reference generator
(tests/golden/gen_fixtures.json) and the plan against the reference parser
(tests/golden/plan_fixtures.json).  NUMERIC parity vs TensorFlow 2.1 is UNPINNED:
TensorFlow is not installed and the reference ships no outputs; the numerics are pinned
only by known-answer tests (tests/test_oracle.py) and by agreement with the engine.
"""

from __future__ import annotations

import numpy as np

SELU_LAMBDA = 1.0507009873554805
SELU_ALPHA = 1.6732632423543772


class OracleError(ValueError):
    """Raised where TensorFlow raises at run time (bad gather/scatter indices, etc.)."""


def _act(x, name):
    if name in (None, "None", "linear"):
        return x
    if name == "relu":
        return np.maximum(x, 0)
    if name == "selu":
        return SELU_LAMBDA * np.where(x > 0, x, SELU_ALPHA * (np.exp(np.minimum(x, 0)) - 1))
    if name == "sigmoid":
        return 1 / (1 + np.exp(-x))
    if name == "tanh":
        return np.tanh(x)
    raise OracleError("activation %r not restated" % name)


def gru_cell(x, h, kernel, recurrent_kernel, bias):
    """Keras GRUCell v2 (reset_after=True) one step; x [N, Din], h [N, H]."""
    H = h.shape[1]
    with np.errstate(over="ignore"):
        return _gru_cell(x, h, kernel, recurrent_kernel, bias, H)


def _gru_cell(x, h, kernel, recurrent_kernel, bias, H):
    mx = x @ kernel + bias[0]
    mh = h @ recurrent_kernel + bias[1]
    z = 1 / (1 + np.exp(-(mx[:, :H] + mh[:, :H])))
    r = 1 / (1 + np.exp(-(mx[:, H:2 * H] + mh[:, H:2 * H])))
    hh = np.tanh(mx[:, 2 * H:] + r * mh[:, 2 * H:])
    return z * h + (1 - z) * hh


def _gather(table, idx, what):
    idx = np.asarray(idx, np.int64)
    if idx.size and (idx.min() < 0 or idx.max() >= table.shape[0]):
        raise OracleError("%s: index out of range [0, %d)" % (what, table.shape[0]))
    return table[idx]


def _scatter_nd(idx_rows, idx_cols, updates, shape):
    out = np.zeros(shape, updates.dtype)
    if np.any(idx_rows < 0) or np.any(idx_rows >= shape[0]) or np.any(idx_cols < 0) or np.any(idx_cols >= shape[1]):
        raise OracleError("scatter_nd index out of range")
    np.add.at(out, (idx_rows, idx_cols), updates)
    return out


class DenseOracle:
    """Interprets a model_description dict directly (independent of ignnition_amd's lowering)."""

    def __init__(self, description: dict, dims: dict, params: dict, dtype=np.float64):
        self.d = description
        self.dims = dims
        self.dtype = dtype
        self.p = {k: np.asarray(v, dtype) for k, v in params.items()}
        self.nn = {n["nn_name"]: n for n in description["neural_networks"]}

    # ------------------------------------------------------------------------------------
    def forward_graph(self, x: dict) -> np.ndarray:
        dt = self.dtype
        state = {}
        for ent in self.d["entities"]:                                   # AUX:140-159
            n = int(np.asarray(x["num_" + ent["name"]]))
            cols, total = [], 0
            for f in ent["features"]:
                size = int(self.dims.get(f["name"], 1))
                total += size
                cols.append(np.asarray(x[f["name"]], dt).reshape(n, size))
            H = int(ent["hidden_state_dimension"])
            if H - total < 0:
                raise OracleError("features exceed hidden_state_dimension")
            cols.append(np.zeros((n, H - total), dt))
            state[ent["name"]] = np.concatenate(cols, axis=1)

        mp_cfg = self.d["message_passing"]
        for _ in range(int(mp_cfg["num_iterations"])):                    # GM:406
            for stage in mp_cfg["stages"]:                                # GM:410
                for mp in stage["stage_mp"]:                              # GM:414
                    self._message_passing(mp, state, x)
        return self._readout(state, x)

    def forward(self, graphs: list) -> np.ndarray:
        """model_fn's per-graph loop + reshape(-1) + concat (GM:712-724)."""
        return np.concatenate([self.forward_graph(g).reshape(-1) for g in graphs])

    # ------------------------------------------------------------------------------------
    def _message_passing(self, mp, state, x):
        dt = self.dtype
        dst = mp["destination_entity"]
        dst_states = state[dst]
        num_dst = int(np.asarray(x["num_" + dst]))
        aggr = mp["aggregation"]["type"]
        first = True
        src_input = final_len = indices = None
        for src in mp["source_entities"]:                                 # GM:423
            sname, adj = src["name"], src["adj_vector"]
            src_idx = np.asarray(x["src_" + adj], np.int64)
            dst_idx = np.asarray(x["dst_" + adj], np.int64)
            seq = np.asarray(x["seq_" + sname + "_" + dst], np.int64)
            msgs = _gather(state[sname], src_idx, "gather " + sname)      # GM:432
            dst_msgs = _gather(dst_states, dst_idx, "gather " + dst)      # GM:433
            src_messages = msgs
            for k, op in enumerate(src["message"]):                        # GM:440-475
                if op["type"] == "direct_assignation":
                    continue
                if op["type"] != "neural_network":
                    raise OracleError("message operation %r not restated" % op["type"])
                parts = []
                for name in op["input"]:
                    if name == "hs_source":
                        parts.append(src_messages)
                    elif name == "hs_dest":
                        parts.append(dst_msgs)
                    elif name == "edge_params":
                        parts.append(np.asarray(x["params_" + adj], dt).reshape(len(src_idx), -1))
                    else:   # other ops' outputs: stored as name+'var', read as name+'_var' (GM:458/470)
                        raise OracleError("message input %r is not readable in the reference" % name)
                h = np.concatenate(parts, axis=1)
                pre = "%s_to_%s_message_creation_0/" % (sname, dst)   # the counter is per source (GM:251, 281)
                for li, layer in enumerate(self.nn[op["nn_name"]]["nn_architecture"]):
                    lname = layer.get("name", "layer_%d_%s_message_creation_%d" % (li, layer["type_layer"], k))
                    b = self.p.get(pre + lname + "/bias")
                    h = h @ self.p[pre + lname + "/kernel"] + (b if b is not None else 0)
                    h = _act(h, layer.get("activation"))
                msgs = h                                                  # the last operation's result
            lens = np.bincount(dst_idx, minlength=num_dst)[:num_dst].astype(np.int64)   # GM:481
            if seq.size == 0:
                raise OracleError("empty adjacency: reduce_max of an empty seq")   # GM:484
            max_len = int(seq.max()) + 1
            s = _scatter_nd(dst_idx, seq, msgs, (num_dst, max_len, msgs.shape[1]))   # GM:490
            if aggr == "concat":                                          # GM:496-505
                axis = int(mp["aggregation"]["concat_axis"])
                if first:
                    src_input, final_len, first = s, lens, False
                else:
                    src_input = np.concatenate([src_input, s], axis=axis)
                    if axis == 1:
                        final_len = final_len + lens
            elif aggr == "interleave":                                    # GM:507-519
                ind = np.asarray(x["indices_" + sname + "_to_" + dst], np.int64)
                if first:
                    src_input, indices, final_len, first = s, ind, lens, False
                else:
                    src_input = np.concatenate([src_input, s], axis=1)
                    if ind.shape != indices.shape:
                        raise OracleError("tf.stack of interleave indices with different lengths")
                    indices = np.stack([indices, ind], axis=0)
                    final_len = final_len + lens
            else:                                                         # GM:523-543
                if first:
                    src_input, final_len, first = s, lens, False
                    comb_src, comb_dst, comb_seq = msgs, dst_idx, seq      # GM:528
                else:
                    src_input = np.concatenate([src_input, s], axis=1)
                    comb_src = np.concatenate([comb_src, msgs], axis=0)   # GM:533-541
                    comb_dst = np.concatenate([comb_dst, dst_idx], axis=0)
                    # quirk: the offset is this source's own lens (GM:539-540)
                    comb_seq = np.concatenate([comb_seq, seq + lens[dst_idx]], axis=0)
                    final_len = final_len + lens

        if aggr == "sum":                                                 # AUX:261
            src_input = src_input.sum(axis=1)
        elif aggr == "interleave":                                        # AUX:432-439
            t = np.transpose(src_input, (1, 0, 2))
            flat = np.asarray(indices, np.int64).reshape(-1)
            if flat.shape[0] != t.shape[0]:
                raise OracleError("interleave: %d indices for %d slots" % (flat.shape[0], t.shape[0]))
            if flat.size and (flat.min() < 0 or flat.max() >= t.shape[0]):
                raise OracleError("interleave index out of range")
            out = np.zeros_like(t)
            np.add.at(out, flat, t)
            src_input = np.transpose(out, (1, 0, 2))
        elif aggr == "attention":                                         # AUX:287-343
            K1, K2, A = (self.p["attention/kernel1"], self.p["attention/kernel2"], self.p["attention/attn_kernel"])
            t_src = comb_src @ K1
            t_dst = dst_states[comb_dst] @ K2
            ai = np.concatenate([t_src, t_dst], axis=1) @ A               # [E, 1]
            ai = np.where(ai > 0, ai, 0.2 * ai)                           # LeakyReLU(alpha=0.2)
            max_len = int(comb_seq.max()) + 1
            aux = _scatter_nd(comb_dst, comb_seq, ai, (num_dst, max_len, 1))
            aux = aux - aux.max(axis=0, keepdims=True)                    # softmax over axis 0 (AUX:336)
            coef = np.exp(aux) / np.exp(aux).sum(axis=0, keepdims=True)
            fc = coef[comb_dst, comb_seq]                                 # gather_nd, [E, 1]
            src_input = np.zeros((num_dst, comb_src.shape[1]), dt)
            np.add.at(src_input, comb_dst, comb_src * fc)                 # unsorted_segment_sum
        elif aggr == "convolution":                                       # AUX:384-401
            Kc = self.p["convolution/kernel"]
            ns = np.zeros((num_dst, Kc.shape[1]), dt)
            np.add.at(ns, comb_dst, comb_src @ Kc)
            deg = np.bincount(comb_dst, minlength=num_dst)[:num_dst].astype(dt)
            with np.errstate(divide="ignore", invalid="ignore"):
                src_input = (ns + dst_states) / deg[:, None]
            src_input = _act(src_input, mp["aggregation"].get("activation_function", "relu"))

        upd = mp["update"]
        if upd["type"] != "recurrent_neural_network":
            raise OracleError("feed-forward update is broken in the reference (GM:338)")
        cell = self._cell(dst)
        old = state[dst]
        if aggr in ("sum", "attention", "convolution"):                   # AUX:752-765
            new = gru_cell(src_input, old, *cell)
        else:                                                             # AUX:767-796
            if np.any(final_len == 0):
                raise OracleError("gather_nd with index -1 (a destination receives no message)")
            if np.any(final_len > src_input.shape[1]):
                raise OracleError("gather_nd index final_len-1 beyond the padded length")
            L = src_input.shape[1]
            # mask = tf.sequence_mask(final_len) is max(final_len) steps wide (AUX:790).  Keras
            # K.rnn (TF 2.1, control flow v2) unstacks it into a TensorList of that length and its
            # while loop runs time_steps = L iterations, reading mask_ta[t] at each: a narrower mask
            # fails with InvalidArgument ("Trying to access element t in a list with t elements").
            if num_dst and final_len.max() < L:
                raise OracleError("sequence_mask(final_len) is %d steps wide, the padded input %d: "
                                  "K.rnn reads the mask TensorList past its end" % (final_len.max(), L))
            h = old
            outputs = np.zeros((num_dst, L, old.shape[1]), dt)
            for t in range(L):
                hn = gru_cell(src_input[:, t, :], h, *cell)
                m = (t < final_len)[:, None]
                h = np.where(m, hn, h)
                outputs[:, t, :] = h
            new = outputs[np.arange(num_dst), final_len - 1]
        state[dst] = new

    def _cell(self, dst):
        pre = dst + "_update/"
        return self.p[pre + "kernel"], self.p[pre + "recurrent_kernel"], self.p[pre + "bias"]

    def _dense_stack(self, h, op, counter):
        """readout_model_<counter> (GM:352-358): Dense layers as named by Feed_forward_model."""
        for li, layer in enumerate(self.nn[op["nn_name"]]["nn_architecture"]):
            name = layer.get("name", "layer_%d_%s_readout" % (li, layer["type_layer"]))  # AUX:909-910
            pre = "readout_model_%d/%s/" % (counter, name)
            h = h @ self.p[pre + "kernel"]
            if pre + "bias" in self.p:
                h = h + self.p[pre + "bias"]
            h = _act(h, layer.get("activation"))
        return h

    def _readout(self, state, x):
        """GM:605-655; names resolve as get_global_var_or_input (GM:660-675): <name>_state first."""
        var = {k: v for k, v in state.items()}

        def get(name):
            return var[name] if name in var else np.asarray(x[name], self.dtype)

        for counter, op in enumerate(self.d["readout"]):
            t = op["type"]
            if t in ("predict", "neural_network"):                         # GM:612-628
                h = np.concatenate([get(i) for i in op["input"]], axis=1)
                h = self._dense_stack(h, op, counter)
                if t == "predict":
                    return h
                var[op.get("output_name", "None")] = h
            elif t == "pooling":                                           # AUX:1165-1185
                v = get(op["input"][0])
                kind = op["type_pooling"]
                if kind == "sum":
                    r = v.sum(0)
                elif kind == "mean":
                    with np.errstate(invalid="ignore", divide="ignore"):
                        r = v.sum(0) / np.asarray(v.shape[0], v.dtype)      # empty: 0/0 = NaN
                elif kind == "max":
                    r = v.max(0) if v.shape[0] else np.full(v.shape[1], -np.inf, v.dtype)
                else:
                    raise OracleError("pooling %r not restated" % kind)
                var[op["output_name"]] = r.reshape(1, -1)
            elif t == "product":                                           # AUX:1072-1088
                if op["type_product"] != "element_wise":
                    raise OracleError("dot_product (rank-4 tensordot) not restated")
                var[op["output_name"]] = get(op["input"][0]) * get(op["input"][1])
            elif t == "extend_adjacencies":                                # AUX:1236-1265
                src = _gather(get(op["input"][0]), x["src_" + op["adj_list"]], "extend_adjacencies src")
                dst = _gather(get(op["input"][1]), x["dst_" + op["adj_list"]], "extend_adjacencies dst")
                var[op["output_name_src"]] = src
                var[op["output_name_dst"]] = dst
            else:
                raise OracleError("readout op %s not restated" % t)
        raise OracleError("no predict operation")


def l2_regularization(description: dict, params: dict) -> float:
    """sum(model.losses) for the Dense kernel_regularizers (AUX:833-834, GM:749)."""
    nn = {n["nn_name"]: n for n in description["neural_networks"]}
    total = 0.0
    for counter, op in enumerate(description["readout"]):
        if op["type"] not in ("predict", "neural_network"):
            continue
        for li, layer in enumerate(nn[op["nn_name"]]["nn_architecture"]):
            if "kernel_regularizer" in layer:
                name = layer.get("name", "layer_%d_%s_readout" % (li, layer["type_layer"]))
                W = np.asarray(params["readout_model_%d/%s/kernel" % (counter, name)], np.float64)
                total += float(layer["kernel_regularizer"]) * float((W * W).sum())
    return total
