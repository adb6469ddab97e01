"""Lowering of a ``Model_information`` plan to the C ABI, parameters and batches.

``MPPlan`` is the counterpart of ``ComnetModel.__init__`` (GM:235-382): it walks the MP
stages in order and decides, per message passing, the aggregation, the GRU cell of the
destination (one per destination entity name, GM:309-313) and the adjacency arrays each
source reads (``src_/dst_<adj>``, ``seq_<src>_<dst>``, ``indices_<src>_to_<dst>``, exactly
the keys of input_fn, GM:127-158).  ``Batch`` turns a list of per-graph feature dicts
into one disjoint-union batch on the device.

Parameters use Keras-style names so checkpoints read like the reference's variables:
``<dst>_update/kernel`` [in, 3H], ``<dst>_update/recurrent_kernel`` [H, 3H],
``<dst>_update/bias`` [2, 3H], ``readout_model_0/<layer>/kernel`` / ``bias``.
"""

from __future__ import annotations

import atexit
import ctypes as C
import weakref
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check, lib

SUPPORTED_GRU_KEYS = {"units", "name"}

# Live handles, released explicitly at interpreter exit (batches before plans) while the HIP
# runtime is still up; relying on __del__ during module teardown can run after it is gone.
_LIVE_BATCHES: "weakref.WeakSet" = weakref.WeakSet()
_LIVE_ENGINES: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _release_all():
    for b in list(_LIVE_BATCHES):
        b.close()
    for e in list(_LIVE_ENGINES):
        e.close()


class UnsupportedModel(ValueError):
    pass


@dataclass
class AdjSlot:
    adj: str
    src: str
    dst: str

    @property
    def keys(self):
        return "src_" + self.adj, "dst_" + self.adj, "seq_" + self.src + "_" + self.dst


def _message_net(s, dst, plan, eidx):
    """The message-creation network of one MP source (GM:440-475), or None (direct_assignation).
    The reference builds every network of a source under one name (its counter counts sources,
    GM:251/281) and reads chained outputs under another (GM:458 vs 470), so exactly one network
    per source reading hs_source / hs_dest / edge_params is what it can run."""
    nets = [op for op in s.message_formation if op.type != "direct_assignation"]
    if not nets:
        return None
    if len(nets) > 1:
        raise UnsupportedModel("more than one message network per source (the reference cannot chain them, GM:458/470)")
    op = nets[0]
    inputs = list(getattr(op, "input", []))
    for name in inputs:
        if name not in _lib.MSG_INPUT:
            raise UnsupportedModel("message input %r is not readable in the reference (GM:458/470)" % name)
    layers = []
    for l in op.model.layers:
        if l.type != "Dense":
            raise UnsupportedModel("message layer type %s is not lowered (Dense only)" % l.type)
        prm = dict(l.parameters)
        act = prm.get("activation", None)
        if act not in _lib.ACT:
            raise UnsupportedModel("activation %r not supported" % act)
        known = {"units", "activation", "kernel_regularizer", "name", "use_bias"}
        if set(prm) - known:
            raise UnsupportedModel("Dense options %s are not lowered" % sorted(set(prm) - known))
        layers.append((prm.get("name"), int(prm["units"]), _lib.ACT[act], int(bool(prm.get("use_bias", True))),
                       float(prm.get("kernel_regularizer", 0.0) or 0.0)))
    widths = {"hs_source": plan.hidden[eidx[s.name]], "hs_dest": plan.hidden[eidx[dst]],
              "edge_params": int(s.extra_parameters)}
    return {"prefix": "%s_to_%s_message_creation_0/" % (s.name, dst), "inputs": inputs,
            "param_dim": int(s.extra_parameters), "din": sum(widths[i] for i in inputs), "layers": layers}


@dataclass
class MPPlan:
    """The lowered plan (entities, adjacency slots, MPs, cells, readout)."""
    model_info: object
    entities: list = field(default_factory=list)       # names
    hidden: list = field(default_factory=list)
    features: list = field(default_factory=list)       # [(name, size)] per entity
    adj_slots: list = field(default_factory=list)
    il_slots: list = field(default_factory=list)       # indices_<src>_to_<dst> keys
    mps: list = field(default_factory=list)            # dicts
    cells: list = field(default_factory=list)          # [(dst_name, din, H)]
    readout_inputs: list = field(default_factory=list)  # predict inputs: readout tensor ids
    readout_ops: list = field(default_factory=list)     # operations before predict (dicts)
    ro_widths: list = field(default_factory=list)       # readout tensor widths (entity states first)
    ro_spaces: list = field(default_factory=list)       # row space per tensor: ("entity", e) / ("graph",) / ("adj", slot)
    predict_counter: int = 0                           # readout_model_<index of predict in the readout list>
    dense: list = field(default_factory=list)          # [(name, units, act, use_bias, l2)]
    iterations: int = 0
    readout_label: str = ""
    convolution_dim: int = 0                           # F of convolution/kernel [F, F] (0: none)
    attention_dim: int = 0                             # F of the attention weights (0: none)

    @classmethod
    def from_model_info(cls, mi) -> "MPPlan":
        p = cls(model_info=mi)
        p.iterations = mi.get_mp_iterations()
        for e in mi.get_entities():
            p.entities.append(e.name)
            h = int(e.hidden_state_dimension)
            if h != e.hidden_state_dimension:
                raise UnsupportedModel("non-integer hidden_state_dimension")
            p.hidden.append(h)
            p.features.append([(f.name, int(f.size)) for f in e.features])
        eidx = {n: i for i, n in enumerate(p.entities)}
        cell_of = {}
        for stage_name, mps in mi.get_mp_instances():
            for mp in mps:
                dst = mp.destination_entity
                upd = mp.update
                if upd.type != "recurrent_nn":
                    # GM:324-346 references an undefined `mp` (NameError): the reference cannot build it.
                    raise UnsupportedModel("feed-forward update is not executable in the reference (GM:338)")
                cell = upd.model
                if cell.type != "GRU":
                    raise UnsupportedModel("recurrent_type %s is not lowered (only GRU; LSTM passes one state, "
                                           "AUX:764)" % cell.type)
                extra = set(cell.parameters) - SUPPORTED_GRU_KEYS
                if extra:
                    raise UnsupportedModel("GRU options %s are not lowered (Keras defaults only)" % sorted(extra))
                aggr = mp.aggregation.type
                if aggr not in ("sum", "ordered", "interleave", "concat", "attention", "convolution"):
                    raise UnsupportedModel("aggregation %r is not lowered yet" % aggr)
                act = 0
                if aggr == "convolution":       # AUX:370-374: activation_function, default relu
                    fn = getattr(mp.aggregation, "activation_function", "relu")
                    if fn not in _lib.ACT:
                        raise UnsupportedModel("convolution activation %r is not lowered" % fn)
                    act = _lib.ACT[fn]
                feature_concat = aggr == "concat" and mp.aggregation.concat_axis == 2
                srcs = []
                nets = []
                din = None
                for s in mp.source_entities:
                    net = _message_net(s, dst, p, eidx)
                    nets.append(net)
                    slot = AdjSlot(s.adj_vector, s.name, dst)
                    if slot not in p.adj_slots:
                        p.adj_slots.append(slot)
                    il = -1
                    if aggr == "interleave":
                        key = "indices_" + s.name + "_to_" + dst
                        if key not in p.il_slots:
                            p.il_slots.append(key)
                        il = p.il_slots.index(key)
                    srcs.append((eidx[s.name], p.adj_slots.index(slot), il))
                    msg_dim = net["layers"][-1][1] if net else p.hidden[eidx[s.name]]
                    # axis-2 concat feeds the GRU the sources' concatenated messages (AUX:443-456)
                    din = (din or 0) + msg_dim if feature_concat else msg_dim
                if dst not in cell_of:
                    cell_of[dst] = len(p.cells)
                    p.cells.append((dst, din, p.hidden[eidx[dst]]))
                p.mps.append({"dst": eidx[dst], "aggr": aggr, "axis": getattr(mp.aggregation, "concat_axis", 0),
                              "cell": cell_of[dst], "sources": srcs, "stage": stage_name, "act": act,
                              "nets": nets})
                if aggr in ("attention", "convolution"):
                    # one weight set per model: the reference overwrites self.kernel1 / conv_kernel per
                    # MP and every MP uses the last one (GM:288-300)
                    setattr(p, aggr + "_dim", p.hidden[eidx[dst]])
        p._lower_readout(mi)
        return p

    @staticmethod
    def _dense_layers(arch, what):
        out = []
        for l in arch.layers:
            if l.type != "Dense":
                raise UnsupportedModel("%s layer type %s is not lowered (Dense only)" % (what, l.type))
            prm = dict(l.parameters)
            act = prm.get("activation", None)
            if act not in _lib.ACT:
                raise UnsupportedModel("activation %r not supported" % act)
            known = {"units", "activation", "kernel_regularizer", "name", "use_bias"}
            if set(prm) - known:
                raise UnsupportedModel("Dense options %s are not lowered" % sorted(set(prm) - known))
            out.append((prm.get("name"), int(prm["units"]), _lib.ACT[act], int(bool(prm.get("use_bias", True))),
                        float(prm.get("kernel_regularizer", 0.0) or 0.0)))
        return out

    def _lower_readout(self, mi):
        """The readout list (GM:605-655) up to the first predict, which returns (GM:629); names
        resolve like get_global_var_or_input (GM:660-675): entity states, then op outputs, later
        outputs shadowing earlier names."""
        names = {n: i for i, n in enumerate(self.entities)}
        self.ro_widths = list(self.hidden)
        self.ro_spaces = [("entity", i) for i in range(len(self.entities))]

        def resolve(name):
            if name not in names:
                raise UnsupportedModel("readout input %r is not an entity state or a readout output (raw input "
                                       "features are not lowered as readout inputs)" % name)
            return names[name]

        def add(name, width, space):
            names[name] = len(self.ro_widths)
            self.ro_widths.append(width)
            self.ro_spaces.append(space)

        pred = None
        for counter, op in enumerate(mi.get_readout_operations()):
            if op.type == "predict":
                pred = (counter, op)
                break
            ids = [resolve(n) for n in op.input]
            first = self.ro_spaces[ids[0]]
            d = {"type": op.type, "inputs": ids, "mode": 0, "adj": -1, "layers": [], "counter": counter}
            if op.type == "neural_network":
                d["layers"] = self._dense_layers(op.architecture, "readout")
                d["in_width"] = sum(self.ro_widths[i] for i in ids)
                add(op.output_name, d["layers"][-1][1], first)
            elif op.type == "pooling":
                if op.type_pooling not in _lib.POOLING:
                    raise UnsupportedModel("pooling type %r is not lowered" % op.type_pooling)
                d["mode"] = _lib.POOLING[op.type_pooling]
                add(op.output_name, self.ro_widths[ids[0]], ("graph",))
            elif op.type == "product":
                if op.type_product != "element_wise":
                    raise UnsupportedModel("product %r is not lowered: tf.tensordot(axes=0) is a rank-4 outer product "
                                           "that the reference records as width 1 (GM:374-375)" % op.type_product)
                if len(ids) < 2:
                    raise UnsupportedModel("product needs two inputs")
                space = first if first != ("graph",) else self.ro_spaces[ids[1]]
                add(op.output_name, self.ro_widths[ids[0]], space)
            elif op.type == "extend_adjacencies":
                slots = [k for k, sl in enumerate(self.adj_slots) if sl.adj == op.adj_list]
                if not slots:
                    raise UnsupportedModel("extend_adjacencies: adjacency %r is not read by any message passing "
                                           "(the reference's input has no src_/dst_ for it)" % op.adj_list)
                d["adj"] = slots[0]
                add(op.output_name[0], self.ro_widths[ids[0]], ("adj", slots[0]))
                add(op.output_name[1], self.ro_widths[ids[1]], ("adj", slots[0]))
            else:
                raise UnsupportedModel("readout operation %r is not lowered" % op.type)
            self.readout_ops.append(d)
        if pred is None:
            raise UnsupportedModel("the readout has no predict operation")
        self.predict_counter, op = pred
        self.readout_label = op.label
        self.readout_inputs = [resolve(n) for n in op.input]
        self.dense = self._dense_layers(op.architecture, "readout")

    @property
    def predict_space(self):
        return self.ro_spaces[self.readout_inputs[0]]

    # ------------------------------------------------------------------ C structures
    def to_desc(self):
        keep = []
        ents = (_lib.EntityDesc * len(self.entities))(
            *[_lib.EntityDesc(h, sum(s for _, s in f)) for h, f in zip(self.hidden, self.features)])
        mps = (_lib.MPDesc * len(self.mps))()
        for i, m in enumerate(self.mps):
            srcs = (_lib.SourceDesc * len(m["sources"]))()
            for k, src in enumerate(m["sources"]):
                net = m.get("nets", [None] * len(m["sources"]))[k]
                if net:
                    ins = (C.c_int32 * len(net["inputs"]))(*[_lib.MSG_INPUT[x] for x in net["inputs"]])
                    lay = (_lib.DenseDesc * len(net["layers"]))(*[_lib.DenseDesc(u, a, b, l2)
                                                                  for _, u, a, b, l2 in net["layers"]])
                    keep += [ins, lay]
                    srcs[k] = _lib.SourceDesc(*src, len(net["inputs"]), ins, net["param_dim"], len(net["layers"]), lay)
                else:
                    srcs[k] = _lib.SourceDesc(*src)
            keep.append(srcs)
            mps[i] = _lib.MPDesc(m["dst"], _lib.AGGR[m["aggr"]], int(m["axis"] or 0), m["cell"], len(m["sources"]),
                                 C.cast(srcs, C.POINTER(_lib.SourceDesc)), int(m.get("act", 0)))
        cells = (_lib.CellDesc * len(self.cells))(*[_lib.CellDesc(din, h) for _, din, h in self.cells])
        ro = (C.c_int32 * len(self.readout_inputs))(*self.readout_inputs)
        dense = (_lib.DenseDesc * len(self.dense))(*[_lib.DenseDesc(u, a, b, l2) for _, u, a, b, l2 in self.dense])
        rops = (_lib.ReadoutOpDesc * max(1, len(self.readout_ops)))()
        for k, op in enumerate(self.readout_ops):
            ins = (C.c_int32 * len(op["inputs"]))(*op["inputs"])
            lay = (_lib.DenseDesc * max(1, len(op["layers"])))(*[_lib.DenseDesc(u, a, b, l2)
                                                                 for _, u, a, b, l2 in op["layers"]])
            keep += [ins, lay]
            rops[k] = _lib.ReadoutOpDesc(_lib.READOUT_OP[op["type"]], len(op["inputs"]), ins, op["mode"], op["adj"],
                                         len(op["layers"]), lay)
        keep += [ents, mps, cells, ro, dense, rops]
        d = _lib.PlanDesc(self.iterations, len(self.entities), ents, len(self.adj_slots), len(self.il_slots),
                          len(self.mps), mps, len(self.cells), cells, len(self.readout_inputs), ro,
                          len(self.dense), dense, len(self.readout_ops), rops)
        return d, keep

    # ------------------------------------------------------------------ parameters
    def param_specs(self):
        """[(name, shape)] in the engine's tensor order (ign_plan_param_tensor)."""
        specs = []
        for dst, din, h in self.cells:
            specs += [(dst + "_update/kernel", (din, 3 * h)), (dst + "_update/recurrent_kernel", (h, 3 * h)),
                      (dst + "_update/bias", (2, 3 * h))]
        for m in self.mps:
            for net in m.get("nets", []):
                if not net:
                    continue
                fan = net["din"]
                for name, units, _, use_bias, _ in net["layers"]:
                    specs.append((net["prefix"] + name + "/kernel", (fan, units)))
                    if use_bias:
                        specs.append((net["prefix"] + name + "/bias", (units,)))
                    fan = units
        if self.convolution_dim:
            F = self.convolution_dim
            specs.append(("convolution/kernel", (F, F)))
        if self.attention_dim:
            F = self.attention_dim
            specs += [("attention/kernel1", (F, F)), ("attention/kernel2", (F, F)), ("attention/attn_kernel", (2 * F, 1))]
        for op in self.readout_ops:
            fan_in = op.get("in_width", 0)
            for li, (name, units, _, use_bias, _) in enumerate(op["layers"]):
                pre = "readout_model_%d/%s" % (op["counter"], name or ("layer_%d" % li))
                specs.append((pre + "/kernel", (fan_in, units)))
                if use_bias:
                    specs.append((pre + "/bias", (units,)))
                fan_in = units
        fan_in = sum(self.ro_widths[i] for i in self.readout_inputs)
        for li, (name, units, _, use_bias, _) in enumerate(self.dense):
            pre = "readout_model_%d/%s" % (self.predict_counter, name or ("layer_%d" % li))
            specs += [(pre + "/kernel", (fan_in, units)), (pre + "/bias", (units,))]
            fan_in = units
        return specs

    def init_params(self, seed: int = 0, bias_scale: float = 0.0) -> dict:
        """Keras default initialisers: glorot_uniform kernels, orthogonal recurrent kernels, zero
        biases (``bias_scale`` > 0 draws biases uniformly instead, for tests)."""
        rng = np.random.default_rng(seed)
        out = {}
        for name, shape in self.param_specs():
            if name.endswith("recurrent_kernel"):
                a = rng.standard_normal((shape[1], shape[0]))
                q, r = np.linalg.qr(a)
                q = q * np.sign(np.diag(r))
                out[name] = q.T.astype(np.float32)
            elif name.endswith("kernel") or name.endswith("kernel1") or name.endswith("kernel2"):
                lim = np.sqrt(6.0 / (shape[0] + shape[1]))
                out[name] = rng.uniform(-lim, lim, shape).astype(np.float32)
            else:
                out[name] = (rng.uniform(-bias_scale, bias_scale, shape).astype(np.float32) if bias_scale
                             else np.zeros(shape, np.float32))
        return out


class Engine:
    """A plan on one device (``ign_plan``)."""

    def __init__(self, plan: MPPlan, device: int = 0):
        self.plan = plan
        self.device = device
        desc, self._keep = plan.to_desc()
        h = C.c_void_p()
        check(lib.ign_plan_create(C.byref(desc), device, C.byref(h)))
        self.handle = h
        self.params_version = 0   # bumped by every parameter update (SplitBatch re-syncs its replicas)
        self._replicas = []
        _LIVE_ENGINES.add(self)
        n = C.c_int64()
        check(lib.ign_plan_num_params(h, C.byref(n)))
        self.n_params = n.value
        nt = C.c_int32()
        check(lib.ign_plan_num_param_tensors(h, C.byref(nt)))
        self.layout = []
        specs = plan.param_specs()
        if nt.value != len(specs):
            raise RuntimeError("parameter layout mismatch between host and engine")
        for i in range(nt.value):
            kind, owner, off, rows, cols = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32(), C.c_int32()
            check(lib.ign_plan_param_tensor(h, i, C.byref(kind), C.byref(owner), C.byref(off), C.byref(rows),
                                            C.byref(cols)))
            name, shape = specs[i]
            if int(np.prod(shape)) != rows.value * cols.value:
                raise RuntimeError("parameter %s: engine shape %dx%d vs host %s" % (name, rows.value, cols.value, shape))
            self.layout.append((name, shape, off.value))

    def set_params(self, params: dict):
        """Every tensor of the layout, by its Keras-like name and with its exact shape (the
        reference's Saver.restore also refuses a missing variable or a shape mismatch)."""
        flat = np.zeros(self.n_params, np.float32)
        missing = [name for name, _, _ in self.layout if name not in params]
        if missing:
            raise ValueError("set_params: missing parameter tensor(s) %s" % ", ".join(missing))
        for name, shape, off in self.layout:
            v = np.asarray(params[name], dtype=np.float32)
            if v.size != int(np.prod(shape)) or (v.ndim > 1 and tuple(v.shape) != tuple(shape)):
                raise ValueError("set_params: %s has shape %s, the model needs %s" % (name, tuple(v.shape), tuple(shape)))
            v = np.ascontiguousarray(v).reshape(-1)
            flat[off:off + v.size] = v
        check(lib.ign_plan_set_params(self.handle, flat.ctypes.data_as(C.c_void_p), 0))
        self.params_version += 1

    def set_timing(self, on: bool, kinds=None):
        """Per-launch HIP event timing (resets the statistics); ``kinds``: kernel kind names to
        instrument (default all)."""
        check(lib.ign_plan_set_timing(self.handle, int(on)))
        mask = 0xFFFFFFFF if kinds is None else sum(1 << _lib.KERNEL_KINDS.index(k) for k in kinds)
        check(lib.ign_plan_set_timing_kinds(self.handle, mask))

    def stats(self) -> dict:
        s = _lib.Stats()
        check(lib.ign_stats(self.handle, C.byref(s)))
        return {k: {"launches": s.launches[i], "ms": s.ms[i], "flops": s.flops[i], "bytes": s.bytes[i],
                    "mfma_bf16": s.mfma_bf16[i], "mfma_f32": s.mfma_f32[i]}
                for i, k in enumerate(_lib.KERNEL_KINDS)}

    def synchronize(self):
        check(lib.ign_synchronize(self.handle))

    def trim_cache(self):
        """Release the idle cached device blocks of this plan and the idle pinned host blocks
        (ign_plan_trim_cache), e.g. when torch or RCCL run short of memory."""
        check(lib.ign_plan_trim_cache(self.handle))

    def set_stream(self, hip_stream: int):
        """Run on an external HIP stream (e.g. ``torch.cuda.current_stream().cuda_stream``)."""
        check(lib.ign_plan_set_stream(self.handle, C.c_void_p(hip_stream)))

    # ---- training (ignnition_amd.training drives these) --------------------------
    def get_params(self) -> dict:
        flat = np.empty(self.n_params, np.float32)
        check(lib.ign_plan_get_params(self.handle, flat.ctypes.data_as(C.c_void_p)))
        return {name: flat[off:off + int(np.prod(shape))].reshape(shape).copy() for name, shape, off in self.layout}

    def mse_loss(self, pred, labels, dpred, want_loss: bool = True) -> float:
        """Device tensors or addresses: pred/labels/dpred [n] fp32 (n = labels.numel()).  Returns the
        loss; writes dLoss/dpred."""
        out = C.c_double()
        check(lib.ign_mse_loss(self.handle, _ptr(pred), _ptr(labels), labels.numel(), _ptr(dpred),
                               C.byref(out) if want_loss else None))
        return out.value if want_loss else None

    def l2_loss(self) -> float:
        out = C.c_double()
        check(lib.ign_l2_loss(self.handle, C.byref(out)))
        return out.value

    def adam_step(self, grads, m, v, iteration: int, lr: float, beta1=0.9, beta2=0.999, epsilon=1e-7):
        check(lib.ign_adam_step(self.handle, _ptr(grads), _ptr(m), _ptr(v), int(iteration), lr, beta1, beta2, epsilon))
        self.params_version += 1

    def replicas(self, n: int) -> list:
        """``n`` more plans of this model on this device (each its own HIP stream), created once and
        kept; their parameters follow this engine's (SplitBatch re-syncs them when they changed)."""
        while len(self._replicas) < n:
            r = Engine(self.plan, self.device)
            r._synced = -1
            self._replicas.append(r)
        for r in self._replicas[:n]:
            if r._synced != self.params_version:
                flat = np.empty(self.n_params, np.float32)
                check(lib.ign_plan_get_params(self.handle, flat.ctypes.data_as(C.c_void_p)))
                check(lib.ign_plan_set_params(r.handle, flat.ctypes.data_as(C.c_void_p), 0))
                r._synced = self.params_version
        return self._replicas[:n]

    def gather_rows(self, src, idx, dst):
        """dst[i] = src[idx[i]] (device tensors: src [R, C] fp32, idx [n] int32, dst [n, C])."""
        n = idx.numel()
        cols = src.shape[1]
        check(lib.ign_gather_rows(self.handle, C.c_void_p(src.data_ptr()), src.stride(0), C.c_void_p(idx.data_ptr()),
                                  n, cols, C.c_void_p(dst.data_ptr())))

    def close(self):
        for r in getattr(self, "_replicas", []):
            r.close()
        self._replicas = []
        h = getattr(self, "handle", None)
        if h:
            lib.ign_plan_destroy(h)
            self.handle = None

    def __del__(self):
        self.close()


def _ptr(x) -> C.c_void_p:
    """Device pointer of a torch tensor, or a raw integer address."""
    return C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))


def _i64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int64).reshape(-1))


class BatchedGraphs:
    """A batch of graphs as graph-concatenated arrays: key -> (values, per-graph lengths), the
    keys of the input_fn dict (GM:127-158).  ``num_<entity>`` holds one value per graph."""

    def __init__(self, arrays: dict, num_graphs: int):
        self.arrays = arrays
        self.num_graphs = num_graphs

    @classmethod
    def from_dicts(cls, graphs: list) -> "BatchedGraphs":
        keys = {}
        for x in graphs:
            for k in x:
                keys.setdefault(k, None)
        arrays = {}
        for k in keys:
            if not all(k in x for x in graphs):
                continue
            parts = [np.asarray(x[k]).reshape(-1) for x in graphs]
            arrays[k] = (np.concatenate(parts) if parts else np.zeros(0), np.array([len(v) for v in parts], np.int64))
        return cls(arrays, len(graphs))

    def get(self, key):
        if key not in self.arrays:
            raise KeyError("batch has no array %r" % key)
        return self.arrays[key]

    def __contains__(self, key):
        return key in self.arrays


def batch_desc(p: "MPPlan", graphs, halo_rows: dict = None):
    """The ``ign_batch_desc`` of a list of feature dicts or a ``BatchedGraphs`` for plan ``p``:
    (desc, arrays the desc points into, (G, E, num [G, E], edge counts [G, A], halo or None))."""
    bg = graphs if isinstance(graphs, BatchedGraphs) else BatchedGraphs.from_dicts(graphs)
    G = bg.num_graphs
    E = len(p.entities)
    num = np.zeros((G, E), np.int64)
    for e, name in enumerate(p.entities):
        v, _ = bg.get("num_" + name)
        num[:, e] = np.asarray(v, np.int64).reshape(G)
    feats = []
    for e, name in enumerate(p.entities):
        cols = []
        for fname, size in p.features[e]:
            v, lens = bg.get(fname)
            if not np.array_equal(np.asarray(lens, np.int64), num[:, e] * size):
                raise ValueError("feature %s: %s values per graph for %s nodes of size %d"
                                 % (fname, list(lens), list(num[:, e]), size))
            cols.append(np.asarray(v, np.float32).reshape(-1, size))
        feats.append(np.ascontiguousarray(np.concatenate(cols, 1)) if cols else None)
    A = len(p.adj_slots)
    cnt = np.zeros((G, A), np.int64)
    srcs, dsts, seqs = [], [], []
    for a, slot in enumerate(p.adj_slots):
        ks, kd, kq = slot.keys
        (s, ls), (d, ld), (q, lq) = bg.get(ks), bg.get(kd), bg.get(kq)
        if not (np.array_equal(ls, ld) and np.array_equal(ls, lq)):
            raise ValueError("%s/%s/%s have different lengths" % (ks, kd, kq))
        cnt[:, a] = ls
        srcs.append(s), dsts.append(d), seqs.append(q)
    I = len(p.il_slots)
    il_len = np.zeros((G, max(I, 1)), np.int64)
    ils = []
    for i, key in enumerate(p.il_slots):
        v, lens = bg.get(key)
        il_len[:, i] = lens
        ils.append(v)
    # index arrays: int32 as they come when every one is (the native reader's narrow gather,
    # index_bytes = 4: no widening copy here, half the bytes the build reads), else all as int64
    narrow = all(np.asarray(x).dtype == np.int32 for x in srcs + dsts + seqs + ils)
    conv = (lambda x: np.ascontiguousarray(np.asarray(x).reshape(-1))) if narrow else _i64
    srcs, dsts, seqs, ils = ([conv(x) for x in l] for l in (srcs, dsts, seqs, ils))
    fp = C.POINTER(C.c_float)
    lp = C.POINTER(C.c_int64)
    feat_ptrs = (fp * E)(*[f.ctypes.data_as(fp) if f is not None and f.size else fp() for f in feats])
    mk = lambda arrs: (lp * max(len(arrs), 1))(*[C.cast(a.ctypes.data, lp) for a in arrs])
    prm_arrays = []
    for slot in p.adj_slots:
        key = "params_" + slot.adj
        prm_arrays.append(np.ascontiguousarray(np.asarray(bg.get(key)[0], np.float32)) if key in bg else None)
    halo = None
    if halo_rows:
        halo = np.array([int(halo_rows.get(name, 0)) for name in p.entities], np.int64)
    ptrs = (feat_ptrs, mk(srcs), mk(dsts), mk(seqs), mk(ils), (fp * max(A, 1))(*[a.ctypes.data_as(fp) if a is not None
                                                                                 else fp() for a in prm_arrays]))
    desc = _lib.BatchDesc(G, num.ctypes.data_as(lp), ptrs[0], cnt.ctypes.data_as(lp), ptrs[1], ptrs[2], ptrs[3],
                          il_len.ctypes.data_as(lp), ptrs[4], halo.ctypes.data_as(lp) if halo is not None else lp(),
                          ptrs[5], 4 if narrow else 8)
    keep = (num, feats, cnt, srcs, dsts, seqs, il_len, ils, prm_arrays, halo, ptrs)
    return desc, keep, (G, E, num, cnt, halo)


class Batch:
    """A disjoint-union batch of graphs on the device (``ign_batch``).

    ``graphs``: list of feature dicts with the input_fn keys (GM:127-158), features already
    normalised.  Graph-local indices are kept; the engine offsets them per graph."""

    def __init__(self, engine: Engine, graphs, halo_rows: dict = None):
        """``graphs``: a list of feature dicts, or a ``BatchedGraphs`` (graph-concatenated arrays,
        e.g. from the native dataset reader).  ``halo_rows``: {entity: extra rows} for one
        edge-cut partition (see partition.py)."""
        p = engine.plan
        self.engine = engine
        desc, keep, (G, E, num, cnt, halo) = batch_desc(p, graphs, halo_rows)
        self._arrays = keep                 # (may view the caller's buffers) until the engine copied them
        self.halo = [0] * E if halo is None else [int(v) for v in halo]
        h = C.c_void_p()
        check(lib.ign_batch_create(engine.handle, C.byref(desc), C.byref(h)))
        self.handle = h
        _LIVE_BATCHES.add(self)
        info = _lib.BatchInfo()
        check(lib.ign_batch_info(h, C.byref(info)))
        self.num_graphs = info.num_graphs
        self.predictions = info.predictions
        self.output_units = info.output_units
        self.edges_per_forward = info.edges_per_forward
        self.gru_steps_per_forward = info.gru_steps_per_forward
        self.rows = list(info.rows)[:E]
        self.graph_rows = num
        space = p.predict_space     # rows of the predict input space per graph (GM:716-724 splits)
        if space[0] == "entity":
            self.graph_predictions = num[:, space[1]].copy()
        elif space[0] == "graph":
            self.graph_predictions = np.ones(G, np.int64)
        else:
            self.graph_predictions = cnt[:, space[1]].copy()
        self._arrays = None  # the engine copied what it needs
        self._bound = {}

    # ---- stepped forward (edge-cut partitions) -----------------------------------
    def begin(self):
        check(lib.ign_forward_begin(self.engine.handle, self.handle))

    def run_mp(self, mp: int, part: str = "all"):
        check(lib.ign_forward_mp(self.engine.handle, self.handle, mp, _lib.PART[part]))

    def end(self, to_host: bool = True):
        out = np.empty((self.predictions, self.output_units), np.float32) if to_host else None
        check(lib.ign_forward_end(self.engine.handle, self.handle,
                                  out.ctypes.data_as(C.c_void_p) if to_host else None))
        return out

    def mp_split(self, mp: int):
        """(interior, boundary) destination counts of MP ``mp``."""
        a, b = C.c_int64(), C.c_int64()
        check(lib.ign_batch_mp_split(self.handle, mp, C.byref(a), C.byref(b)))
        return a.value, b.value

    def bind_state(self, entity: str, buf0, buf1):
        """Use two caller-owned device buffers (torch tensors) as the entity's state buffers."""
        e = self.engine.plan.entities.index(entity)
        cap = min(buf0.numel(), buf1.numel())
        check(lib.ign_batch_bind_state(self.engine.handle, self.handle, e, C.c_void_p(buf0.data_ptr()),
                                       C.c_void_p(buf1.data_ptr()), cap))
        self._bound[entity] = (buf0, buf1)

    # ---- training -------------------------------------------------------------------------
    def enable_training(self):
        check(lib.ign_batch_enable_training(self.engine.handle, self.handle))

    def forward_train(self, to_host: bool = True):
        out = np.empty((self.predictions, self.output_units), np.float32) if to_host else None
        check(lib.ign_forward_train(self.engine.handle, self.handle,
                                    out.ctypes.data_as(C.c_void_p) if to_host else None))
        return out

    # stepped training step (edge-cut partitions: partition.EdgeCutTraining exchanges between steps)
    def forward_train_begin(self):
        check(lib.ign_forward_train_begin(self.engine.handle, self.handle))

    def forward_train_mp(self):
        check(lib.ign_forward_train_mp(self.engine.handle, self.handle))

    def forward_train_end(self, to_host: bool = True):
        out = np.empty((self.predictions, self.output_units), np.float32) if to_host else None
        check(lib.ign_forward_train_end(self.engine.handle, self.handle,
                                        out.ctypes.data_as(C.c_void_p) if to_host else None))
        return out

    def backward_begin(self, dpred, grads, l2_scale: float = 1.0):
        check(lib.ign_backward_begin(self.engine.handle, self.handle, _ptr(dpred), _ptr(grads), float(l2_scale)))

    def backward_mp(self):
        check(lib.ign_backward_mp(self.engine.handle, self.handle))

    def backward_end(self):
        check(lib.ign_backward_end(self.engine.handle, self.handle))

    def train_buffers(self, entity: str):
        """(state, gradient) device pointers of the entity's current version, [rows + halo][H]."""
        st, gr = C.c_void_p(), C.c_void_p()
        check(lib.ign_batch_train_buffers(self.handle, self.engine.plan.entities.index(entity), C.byref(st),
                                          C.byref(gr)))
        return st.value, gr.value

    def predictions_ptr(self) -> int:
        p = C.c_void_p()
        check(lib.ign_batch_predictions(self.handle, C.byref(p)))
        return p.value

    def backward(self, dpred, grads):
        """dpred, grads: device tensors ([predictions * units], [n_params])."""
        check(lib.ign_backward(self.engine.handle, self.handle, _ptr(dpred), _ptr(grads)))

    def resident_info(self) -> dict:
        """The graph-resident forward of this batch (decided when the batch is built; at its first
        forward under IGN_RESIDENT_EAGER=0): whether it runs, its form and LDS, and the per-launch
        cost model (ign_batch_resident_info)."""
        r = _lib.ResidentInfo()
        if not hasattr(lib, "ign_batch_resident_info"):   # an A/B build of an older tree (IGN_AB_LIB=1)
            return {"active": 0}
        check(lib.ign_batch_resident_info(self.handle, C.byref(r)))
        return {name: getattr(r, name) for name, _ in _lib.ResidentInfo._fields_}

    def state_slot(self, entity: str) -> int:
        s = C.c_int32()
        check(lib.ign_batch_state_slot(self.handle, self.engine.plan.entities.index(entity), C.byref(s)))
        return s.value

    def forward(self, to_host: bool = True):
        eng = self.engine
        if to_host:
            out = np.empty((self.predictions, self.output_units), np.float32)
            check(lib.ign_forward(eng.handle, self.handle, out.ctypes.data_as(C.c_void_p)))
            return out
        check(lib.ign_forward(eng.handle, self.handle, None))
        return None

    def state(self, entity: str) -> np.ndarray:
        p = self.engine.plan
        e = p.entities.index(entity)
        out = np.empty((self.rows[e], p.hidden[e]), np.float32)
        check(lib.ign_batch_state(self.engine.handle, self.handle, e, out.ctypes.data_as(C.c_void_p)))
        return out

    def close(self):
        h = getattr(self, "handle", None)
        if h:
            lib.ign_batch_destroy(h)
            self.handle = None

    def __del__(self):
        self.close()


def split_cuts(n_graphs: int, parts: int) -> list:
    """Boundaries of ``parts`` sub-batches of consecutive graphs (at most one per graph, at least
    one): sub-batch i is graphs [cuts[i], cuts[i + 1]), sizes differing by at most one."""
    if n_graphs < 1:
        raise ValueError("SplitBatch: no graphs")
    parts = max(1, min(int(parts), n_graphs))
    return [n_graphs * i // parts for i in range(parts + 1)]


class SplitBatch:
    """The graphs as ``parts`` sub-batches of consecutive graphs, sub-batch i on the engine's
    replica i (its own plan and HIP stream; replica 0 is the engine itself).  ``forward`` enqueues
    every sub-batch before waiting, so the kernels of different sub-batches co-run: the
    memory-bound sum update of one beside the issue-bound ordered update of another (DESIGN §3b'').
    The predictions are the batch's, in graph order, bitwise those of one ``Batch`` (graphs are
    independent: GM:712-724)."""

    def __init__(self, engine: Engine, graphs, parts: int = 2):
        graphs = list(graphs)
        cuts = split_cuts(len(graphs), parts)
        parts = len(cuts) - 1
        self.engine = engine
        self.engines = [engine] + engine.replicas(parts - 1)
        self.parts = [Batch(e, graphs[cuts[i]:cuts[i + 1]]) for i, e in enumerate(self.engines)]
        self.num_graphs = sum(b.num_graphs for b in self.parts)
        self.predictions = sum(b.predictions for b in self.parts)
        self.output_units = self.parts[0].output_units
        self.edges_per_forward = sum(b.edges_per_forward for b in self.parts)
        self.gru_steps_per_forward = sum(b.gru_steps_per_forward for b in self.parts)
        self.graph_predictions = np.concatenate([b.graph_predictions for b in self.parts])

    def forward(self, to_host: bool = True):
        self.engine.replicas(len(self.parts) - 1)   # re-sync replica parameters if they changed
        for b in self.parts:
            b.forward(to_host=False)
        if not to_host:
            return None
        out = np.empty((self.predictions, self.output_units), np.float32)
        row = 0
        for b in self.parts:
            check(lib.ign_batch_read_predictions(b.engine.handle, b.handle,
                                                 out[row:row + b.predictions].ctypes.data_as(C.c_void_p)))
            row += b.predictions
        return out

    def synchronize(self):
        for e in self.engines:
            e.synchronize()

    def close(self):
        for b in self.parts:
            b.close()

    def __del__(self):
        self.close()


def device_count() -> int:
    n = C.c_int32()
    lib.ign_device_count(C.byref(n))
    return n.value
