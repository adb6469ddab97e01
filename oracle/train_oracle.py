"""ORACLE (test infrastructure only) — the training step, restated with torch autograd (float64).

Same forward as dense_forward.py (the TF op sequence of ComnetModel.call, GM:384-658), written
with torch ops so autograd gives the gradients the reference's `tf.gradients(total_loss,
model.trainable_variables)` (GM:790) computes.  Plus the rest of model_fn's TRAIN branch:

  loss            GM:749-753   MeanSquaredError(labels, predictions) over the concatenated flat
                               predictions of the batch + sum(model.losses) (Dense l2 kernel
                               regularizers, AUX:833-834: c * sum(W^2))
  optimizer       GM:797-818   Keras Adam (beta1 0.9, beta2 0.999, epsilon 1e-7), iterations =
                               global step, learning rate from ExponentialDecay(step)
  eval metrics    GM:755-785   label/prediction mean, MAE, MRE (|l - p| / |l|), r-squared (GM:201-216)

Keras / TF 2.1 optimizer math (not in the reference repo; restated from the published
definitions of training_ops.ApplyAdam and learning_rate_schedule.ExponentialDecay):
  t = iterations + 1
  lr_t = lr(iterations) * sqrt(1 - b2^t) / (1 - b1^t)
  m = b1 m + (1 - b1) g ;  v = b2 v + (1 - b2) g^2 ;  w -= lr_t m / (sqrt(v) + eps)
  lr(step) = lr0 * rate^(step / decay_steps), exponent floored when `staircase` is truthy (any
  non-empty string is, including the "True" the Q-size example passes, QSJ:204).

Only tests/ import this module.  Parity status: gradients pinned by autograd of this
restatement; agreement of its forward with dense_forward.py is a test; NUMERIC parity vs
TensorFlow is UNPINNED (TF is not installed).
"""

from __future__ import annotations

import math

import numpy as np
import torch

from .dense_forward import SELU_ALPHA, SELU_LAMBDA, OracleError

_T = torch.float64


def _act(x, name):
    if name in (None, "None", "linear"):
        return x
    if name == "relu":
        return torch.relu(x)
    if name == "selu":
        return SELU_LAMBDA * torch.where(x > 0, x, SELU_ALPHA * (torch.exp(torch.clamp(x, max=0)) - 1))
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "tanh":
        return torch.tanh(x)
    raise OracleError("activation %r not restated" % name)


def gru_cell(x, h, kernel, recurrent_kernel, bias):
    """Keras GRUCell v2, reset_after=True, gates z, r, h."""
    H = h.shape[1]
    mx = x @ kernel + bias[0]
    mh = h @ recurrent_kernel + bias[1]
    z = torch.sigmoid(mx[:, :H] + mh[:, :H])
    r = torch.sigmoid(mx[:, H:2 * H] + mh[:, H:2 * H])
    hh = torch.tanh(mx[:, 2 * H:] + r * mh[:, 2 * H:])
    return z * h + (1 - z) * hh


class TorchOracle:
    def __init__(self, description: dict, dims: dict, params: dict):
        self.d = description
        self.dims = dims
        self.p = {k: torch.tensor(np.asarray(v, np.float64), dtype=_T, requires_grad=True) for k, v in params.items()}
        self.nn = {n["nn_name"]: n for n in description["neural_networks"]}

    # ---------------------------------------------------------------- forward (GM:384-658)
    def forward_graph(self, x: dict):
        state = {}
        for ent in self.d["entities"]:
            n = int(np.asarray(x["num_" + ent["name"]]))
            cols, total = [], 0
            for f in ent["features"]:
                size = int(self.dims.get(f["name"], 1))
                total += size
                cols.append(torch.tensor(np.asarray(x[f["name"]], np.float64).reshape(n, size), dtype=_T))
            H = int(ent["hidden_state_dimension"])
            cols.append(torch.zeros((n, H - total), dtype=_T))
            state[ent["name"]] = torch.cat(cols, 1)
        mp_cfg = self.d["message_passing"]
        for _ in range(int(mp_cfg["num_iterations"])):
            for stage in mp_cfg["stages"]:
                for mp in stage["stage_mp"]:
                    self._message_passing(mp, state, x)
        return self._readout(state, x)

    def forward(self, graphs):
        return torch.cat([self.forward_graph(g).reshape(-1) for g in graphs])

    def _message_passing(self, mp, state, x):
        dst = mp["destination_entity"]
        num_dst = int(np.asarray(x["num_" + dst]))
        aggr = mp["aggregation"]["type"]
        first = True
        src_input = final_len = indices = None
        for src in mp["source_entities"]:
            sname, adj = src["name"], src["adj_vector"]
            src_idx = torch.as_tensor(np.asarray(x["src_" + adj], np.int64))
            dst_idx = torch.as_tensor(np.asarray(x["dst_" + adj], np.int64))
            seq = torch.as_tensor(np.asarray(x["seq_" + sname + "_" + dst], np.int64))
            msgs = state[sname][src_idx]                                  # GM:432
            for k, op in enumerate(src.get("message", [])):                # GM:440-475
                if op["type"] == "direct_assignation":
                    continue
                if op["type"] != "neural_network":
                    raise OracleError("message operation %r not restated" % op["type"])
                parts = []
                for name in op["input"]:
                    if name == "hs_source":
                        parts.append(state[sname][src_idx])
                    elif name == "hs_dest":
                        parts.append(state[dst][dst_idx])                 # GM:433
                    elif name == "edge_params":
                        parts.append(torch.tensor(np.asarray(x["params_" + adj], np.float64).reshape(len(src_idx), -1),
                                                  dtype=_T))
                    else:
                        raise OracleError("message input %r is not readable in the reference" % name)
                h = torch.cat(parts, 1)
                for layer, pre in self._msg_layers(sname, dst, op, k):
                    b = self.p.get(pre + "/bias")
                    h = h @ self.p[pre + "/kernel"] + (b if b is not None else 0)
                    h = _act(h, layer.get("activation"))
                msgs = h
            lens = torch.bincount(dst_idx, minlength=num_dst)[:num_dst]   # GM:481
            L = int(seq.max()) + 1
            s = torch.zeros((num_dst, L, msgs.shape[1]), dtype=_T).index_put((dst_idx, seq), msgs, accumulate=True)
            if aggr == "interleave":
                ind = torch.as_tensor(np.asarray(x["indices_" + sname + "_to_" + dst], np.int64))
                if first:
                    src_input, indices, final_len, first = s, ind, lens, False
                else:
                    src_input = torch.cat([src_input, s], 1)
                    indices = torch.stack([indices, ind], 0)
                    final_len = final_len + lens
            elif aggr == "concat" and int(mp["aggregation"]["concat_axis"]) != 1:   # GM:496-505
                if first:
                    src_input, final_len, first = s, lens, False            # the first source's lens
                else:
                    if s.shape[1] != src_input.shape[1]:
                        raise OracleError("ConcatOp: sources with different Lmax")
                    src_input = torch.cat([src_input, s], 2)
            else:
                if first:
                    src_input, final_len, first = s, lens, False
                    comb_src, comb_dst, comb_seq = msgs, dst_idx, seq      # GM:528
                else:
                    src_input = torch.cat([src_input, s], 1)
                    final_len = final_len + lens
                    comb_src = torch.cat([comb_src, msgs], 0)              # GM:533-541
                    comb_dst = torch.cat([comb_dst, dst_idx], 0)
                    comb_seq = torch.cat([comb_seq, seq + lens[dst_idx]], 0)   # quirk: own lens (GM:539-540)
        if aggr == "sum":
            src_input = src_input.sum(1)
        elif aggr == "attention":                                         # AUX:287-343
            K1, K2, A = self.p["attention/kernel1"], self.p["attention/kernel2"], self.p["attention/attn_kernel"]
            ai = torch.cat([comb_src @ K1, state[dst][comb_dst] @ K2], 1) @ A
            ai = torch.where(ai > 0, ai, 0.2 * ai)                         # LeakyReLU(alpha=0.2)
            max_len = int(comb_seq.max()) + 1
            aux = torch.zeros((num_dst, max_len, 1), dtype=_T).index_put((comb_dst, comb_seq), ai, accumulate=True)
            aux = aux - aux.max(0, keepdim=True).values                    # softmax over axis 0 (AUX:336)
            coef = torch.exp(aux) / torch.exp(aux).sum(0, keepdim=True)
            fc = coef[comb_dst, comb_seq]
            src_input = torch.zeros((num_dst, comb_src.shape[1]), dtype=_T).index_add(0, comb_dst, comb_src * fc)
        elif aggr == "convolution":                                       # AUX:384-401
            Kc = self.p["convolution/kernel"]
            ns = torch.zeros((num_dst, Kc.shape[1]), dtype=_T).index_add(0, comb_dst, comb_src @ Kc)
            deg = torch.bincount(comb_dst, minlength=num_dst)[:num_dst].to(_T)
            src_input = _act((ns + state[dst]) / deg[:, None], mp["aggregation"].get("activation_function", "relu"))
        elif aggr == "interleave":
            t = src_input.transpose(0, 1)
            flat = indices.reshape(-1)
            t = torch.zeros_like(t).index_add(0, flat, t)
            src_input = t.transpose(0, 1)
        cell = self._cell(dst)
        old = state[dst]
        if aggr in ("sum", "attention", "convolution"):
            new = gru_cell(src_input, old, *cell)
        else:
            if bool((final_len == 0).any()):
                raise OracleError("gather_nd with index -1")
            if num_dst and int(final_len.max()) != src_input.shape[1]:   # dense_forward.py, AUX:785-795
                raise OracleError("sequence_mask(final_len) width %d vs padded length %d"
                                  % (int(final_len.max()), src_input.shape[1]))
            h = old
            outs = []
            for t in range(src_input.shape[1]):
                hn = gru_cell(src_input[:, t, :], h, *cell)
                h = torch.where((t < final_len)[:, None], hn, h)
                outs.append(h)
            outputs = torch.stack(outs, 1)
            new = outputs[torch.arange(num_dst), final_len - 1]
        state[dst] = new

    def _cell(self, dst):
        pre = dst + "_update/"
        return self.p[pre + "kernel"], self.p[pre + "recurrent_kernel"], self.p[pre + "bias"]

    def _msg_layers(self, sname, dst, op, k):
        # one network name per source (the reference's counter counts sources, GM:251/281)
        for li, layer in enumerate(self.nn[op["nn_name"]]["nn_architecture"]):
            lname = layer.get("name", "layer_%d_%s_message_creation_%d" % (li, layer["type_layer"], k))
            yield layer, "%s_to_%s_message_creation_0/%s" % (sname, dst, lname)

    def _layers(self, op, counter):
        """readout_model_<index of the op in the readout list> (GM:352-358), Feed_forward_model names."""
        for li, layer in enumerate(self.nn[op["nn_name"]]["nn_architecture"]):
            name = layer.get("name", "layer_%d_%s_readout" % (li, layer["type_layer"]))
            yield layer, "readout_model_%d/%s" % (counter, name)

    def _readout(self, state, x):
        """GM:605-655: operations before predict write named tensors (get_global_var_or_input,
        GM:660-675), then predict.  As the dense oracle, with torch ops."""
        var = dict(state)

        def get(name):
            return var[name] if name in var else torch.tensor(np.asarray(x[name], np.float64), dtype=_T)

        for counter, op in enumerate(self.d["readout"]):
            t = op["type"]
            if t in ("predict", "neural_network"):                         # GM:612-628
                h = torch.cat([get(i) for i in op["input"]], 1)
                for layer, pre in self._layers(op, counter):
                    h = h @ self.p[pre + "/kernel"]
                    if pre + "/bias" in self.p:
                        h = h + self.p[pre + "/bias"]
                    h = _act(h, layer.get("activation"))
                if t == "predict":
                    return h
                var[op.get("output_name", "None")] = h
            elif t == "pooling":                                           # AUX:1165-1185
                v = get(op["input"][0])
                kind = op["type_pooling"]
                if kind == "sum":
                    r = v.sum(0)
                elif kind == "mean":
                    r = v.sum(0) / v.shape[0]
                elif kind == "max":
                    # tf.reduce_max: the gradient is split equally among the maximal rows
                    ind = (v == v.max(0).values).to(_T)
                    r = (v * ind).sum(0) / ind.sum(0)
                else:
                    raise OracleError("pooling %r not restated" % kind)
                var[op["output_name"]] = r.reshape(1, -1)
            elif t == "product":                                           # AUX:1072-1088
                if op["type_product"] != "element_wise":
                    raise OracleError("dot_product (rank-4 tensordot) not restated")
                var[op["output_name"]] = get(op["input"][0]) * get(op["input"][1])
            elif t == "extend_adjacencies":                                # AUX:1236-1265
                var[op["output_name_src"]] = get(op["input"][0])[torch.as_tensor(np.asarray(x["src_" + op["adj_list"]], np.int64))]
                var[op["output_name_dst"]] = get(op["input"][1])[torch.as_tensor(np.asarray(x["dst_" + op["adj_list"]], np.int64))]
            else:
                raise OracleError("readout op %s not restated" % t)
        raise OracleError("no predict operation")

    # ---------------------------------------------------------------- loss (GM:745-753)
    def regularization(self):
        """sum(model.losses): kernel_regularizer of every Dense layer the model owns (AUX:833-834),
        the readout's and the message-creation networks'."""
        total = torch.zeros((), dtype=_T)
        for stage in self.d["message_passing"]["stages"]:
            for mp in stage["stage_mp"]:
                for src in mp["source_entities"]:
                    for k, op in enumerate(src.get("message", [])):
                        if op["type"] != "neural_network":
                            continue
                        for layer, pre in self._msg_layers(src["name"], mp["destination_entity"], op, k):
                            if "kernel_regularizer" in layer:
                                W = self.p[pre + "/kernel"]
                                total = total + float(layer["kernel_regularizer"]) * (W * W).sum()
        for counter, op in enumerate(self.d["readout"]):
            if op["type"] not in ("predict", "neural_network"):
                continue
            for layer, pre in self._layers(op, counter):
                if "kernel_regularizer" in layer:
                    W = self.p[pre + "/kernel"]
                    total = total + float(layer["kernel_regularizer"]) * (W * W).sum()
        return total

    def loss_and_grads(self, graphs, labels):
        """(loss, regularization loss, {name: grad ndarray}, predictions)."""
        for v in self.p.values():
            v.grad = None
        pred = self.forward(graphs)
        y = torch.tensor(np.concatenate([np.asarray(l, np.float64).reshape(-1) for l in labels]), dtype=_T)
        loss = ((y - pred) ** 2).mean()
        reg = self.regularization()
        (loss + reg).backward()
        grads = {k: v.grad.detach().numpy().copy() if v.grad is not None else np.zeros(v.shape) for k, v in self.p.items()}
        return float(loss.detach()), float(reg.detach()), grads, pred.detach().numpy()


# -------------------------------------------------------------------- optimizer (GM:797-818)
def exponential_decay(step, initial_learning_rate, decay_steps, decay_rate, staircase=False):
    p = step / float(decay_steps)
    if staircase:            # truthy test, as Keras does (a "False" string is truthy too)
        p = math.floor(p)
    return initial_learning_rate * decay_rate ** p


def adam_step(params: dict, grads: dict, m: dict, v: dict, iterations: int, lr: float,
              beta_1=0.9, beta_2=0.999, epsilon=1e-7):
    """One Keras Adam update in float64 (in place on params / m / v)."""
    t = iterations + 1
    lr_t = lr * math.sqrt(1 - beta_2 ** t) / (1 - beta_1 ** t)
    for k in params:
        g = np.asarray(grads[k], np.float64)
        m[k] = beta_1 * m[k] + (1 - beta_1) * g
        v[k] = beta_2 * v[k] + (1 - beta_2) * g * g
        params[k] = params[k] - lr_t * m[k] / (np.sqrt(v[k]) + epsilon)


def eval_metrics(labels, predictions):
    """GM:755-785 and r_squared (GM:201-216), on one evaluation batch."""
    l = np.asarray(labels, np.float64).reshape(-1)
    p = np.asarray(predictions, np.float64).reshape(-1)
    tot = ((l - l.mean()) ** 2).sum()
    return {"label/mean": l.mean(), "prediction/mean": p.mean(), "mae": np.abs(l - p).mean(),
            "mre": (np.abs(l - p) / np.abs(l)).mean(), "r-squared": 1.0 - ((l - p) ** 2).sum() / tot}
