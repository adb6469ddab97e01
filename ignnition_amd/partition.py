"""Edge-cut partitioning of one large graph across GPUs, with halo exchange.

The reference runs every graph whole on one device (``model_fn``'s per-graph loop, GM:712-724);
a graph that outgrows one GPU (the 1M-node / 10M-edge synthetic config, BASELINE configs[4])
is split here instead:

* **Partition**: contiguous id ranges per entity (``node_ranges``), owner computes by
  destination. A partition keeps every in-edge of its owned destinations (edge-cut), so each
  destination's messages and their summation order are the same as in the unpartitioned graph.
* **Halo**: the distinct remote source rows a partition reads. They are stored after the owned
  rows in the entity's state buffer, grouped by owner rank, ascending id. The engine gets them
  through ``ign_batch_desc.halo_rows``.
* **Requests**: each partition sends every owner the ids it needs, once at setup, with one
  all-to-all. The reply lists become the owner's send lists. No rank needs the global graph.
* **Exchange**: before an MP reads an entity whose halo is stale, each rank packs its send rows
  with ``ign_gather_rows`` (HIP). One ``all_to_all_single`` (RCCL over xGMI) then delivers them
  straight into the halo rows of the peer's current state buffer. There is no unpack copy.
* **Overlap**: destinations that read no halo row (``IGN_PART_INTERIOR``) run while the exchange
  is in flight. The boundary destinations run after it completes.

Only ``sum`` MPs are partitioned. ``ordered`` / ``interleave`` pad per graph (GM:477-543), so
splitting a graph would change the reference's slot layout; those models shard by graph
(workloads.shard_graph_ids).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .engine import Batch, Engine, MPPlan


def node_ranges(n: int, world: int) -> np.ndarray:
    """Contiguous balanced id ranges: rank r owns [b[r], b[r+1])."""
    return np.array([(n * r) // world for r in range(world + 1)], np.int64)


@dataclass
class HaloPlan:
    entity: str
    n_owned: int
    halo_ids: np.ndarray        # global ids of the halo rows (ascending, hence grouped by owner)
    recv_counts: list           # halo rows received from each rank
    send_rows: np.ndarray       # local owned rows sent, grouped by destination rank (int32)
    send_counts: list

    @property
    def n_halo(self) -> int:
        return int(len(self.halo_ids))


@dataclass
class LocalPart:
    rank: int
    inputs: dict                # input_fn dict of the partition (local ids; halo rows after owned rows)
    ranges: dict                # entity -> node_ranges
    needs: dict                 # entity -> [ids needed from each rank]
    halos: dict = None          # entity -> HaloPlan (after exchange_requests)


def _check_plan(plan: MPPlan):
    for m in plan.mps:
        if m["aggr"] not in ("sum", "convolution"):
            raise ValueError("edge-cut partitioning supports sum and convolution MPs only (ordered/interleave/concat "
                             "pad per graph, GM:477-543; attention normalises over all of a graph's destinations, "
                             "AUX:327-336); shard such batches by graph")


def _overlappable(m) -> bool:
    """Interior destinations can run beside the exchange: a plain sum MP.  A message network reads
    every source row (halo ones included) in its per-edge pass before any destination runs."""
    return m["aggr"] == "sum" and not any(m.get("nets", []))


def local_part(inputs: dict, plan: MPPlan, rank: int, world: int) -> LocalPart:
    """The partition of ``rank`` from a graph's input_fn dict (global ids)."""
    _check_plan(plan)
    ranges = {}
    for name in plan.entities:
        ranges[name] = node_ranges(int(np.asarray(inputs["num_" + name]).reshape(())), world)
    out = {}
    for e, name in enumerate(plan.entities):
        lo, hi = ranges[name][rank], ranges[name][rank + 1]
        out["num_" + name] = np.int64(hi - lo)
        n = int(np.asarray(inputs["num_" + name]).reshape(()))
        for fname, size in plan.features[e]:
            rows = np.asarray(inputs[fname]).reshape(n, size)[lo:hi]
            out[fname] = rows.reshape(-1) if size == 1 else rows
    # remote source ids per source entity
    remote = {name: [] for name in plan.entities}
    kept = []
    for slot in plan.adj_slots:
        ks, kd, kq = slot.keys
        s = np.asarray(inputs[ks], np.int64).reshape(-1)
        d = np.asarray(inputs[kd], np.int64).reshape(-1)
        q = np.asarray(inputs[kq], np.int64).reshape(-1)
        dlo, dhi = ranges[slot.dst][rank], ranges[slot.dst][rank + 1]
        keep = (d >= dlo) & (d < dhi)            # owner computes: every in-edge of an owned destination
        s, d, q = s[keep], d[keep] - dlo, q[keep]
        kp = "params_" + slot.adj                # per-edge parameters (message networks, GEN:156-163)
        if kp in inputs:
            prm = np.asarray(inputs[kp], np.float32)
            out[kp] = prm.reshape(len(keep), -1)[keep]
        slo, shi = ranges[slot.src][rank], ranges[slot.src][rank + 1]
        rem = (s < slo) | (s >= shi)
        remote[slot.src].append(s[rem])
        kept.append((slot, s, d, q, rem))
    halo_ids = {name: np.unique(np.concatenate(remote[name])) if remote[name] else np.zeros(0, np.int64)
                for name in plan.entities}
    for slot, s, d, q, rem in kept:
        ks, kd, kq = slot.keys
        slo, shi = ranges[slot.src][rank], ranges[slot.src][rank + 1]
        ls = s - slo
        ls[rem] = (shi - slo) + np.searchsorted(halo_ids[slot.src], s[rem])
        out[ks], out[kd], out[kq] = ls, d, q
    needs = {}
    for name in plan.entities:
        owner = np.searchsorted(ranges[name], halo_ids[name], side="right") - 1
        needs[name] = [halo_ids[name][owner == p] for p in range(world)]
    part = LocalPart(rank, out, ranges, needs)
    part.halos = {name: HaloPlan(name, int(ranges[name][rank + 1] - ranges[name][rank]), halo_ids[name],
                                 [len(x) for x in needs[name]], None, None) for name in plan.entities}
    return part


def exchange_requests(parts: list, comm) -> None:
    """Setup all-to-all: each owner learns which of its rows every peer reads (fills send lists)."""
    names = list(parts[0].needs)
    for name in names:
        got = comm.alltoall_ids([p.needs[name] for p in parts])
        for p, g in zip(parts, got):
            lo = p.ranges[name][p.rank]
            h = p.halos[name]
            h.send_rows = (np.concatenate(g) - lo).astype(np.int32) if g else np.zeros(0, np.int32)
            h.send_counts = [len(x) for x in g]
            if len(h.send_rows) and (h.send_rows.min() < 0 or h.send_rows.max() >= h.n_owned):
                raise RuntimeError("halo request for a row this rank does not own")


# ---------------------------------------------------------------------------------------------
# Transports.  Both move a list of partitions' packed rows; TorchComm holds exactly one partition
# (one process per GPU), LoopbackComm all of them (tests on one device).

class _Done:
    def wait(self):
        pass


class TorchComm:
    """torch.distributed all-to-all: RCCL ('nccl' backend) over xGMI on GPUs, gloo on CPU."""

    def __init__(self, dist, device=None, group=None, host_staged: bool = False):
        """``host_staged``: device rows go through host memory (gloo rehearsal of the N>1 path
        with several ranks on one GPU, where RCCL refuses duplicate devices)."""
        self.dist, self.device, self.group, self.host_staged = dist, device, group, host_staged
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)

    def alltoall_ids(self, sends: list) -> list:
        import torch
        (send,) = sends
        cnt = torch.tensor([len(x) for x in send], dtype=torch.int64, device=self.device)
        rcnt = torch.empty_like(cnt)
        self.dist.all_to_all_single(rcnt, cnt, group=self.group)
        flat = np.concatenate(send).astype(np.int64) if send else np.zeros(0, np.int64)
        sbuf = torch.from_numpy(flat).to(self.device)
        rc = rcnt.cpu().tolist()
        rbuf = torch.empty(sum(rc), dtype=torch.int64, device=self.device)
        self.dist.all_to_all_single(rbuf, sbuf, rc, cnt.cpu().tolist(), group=self.group)
        r = rbuf.cpu().numpy()
        offs = np.cumsum([0] + rc)
        return [[r[offs[i]:offs[i + 1]] for i in range(self.world)]]

    def exchange(self, sends: list, send_counts: list, recvs: list, recv_counts: list, async_op: bool):
        (send,), (sc,), (recv,), (rc,) = sends, send_counts, recvs, recv_counts
        if self.host_staged:
            hrecv = recv.new_empty(recv.shape, device="cpu")
            self.dist.all_to_all_single(hrecv, send.cpu(), rc, sc, group=self.group)
            recv.copy_(hrecv)
            return _Done()
        w = self.dist.all_to_all_single(recv, send, rc, sc, group=self.group, async_op=async_op)
        return w if async_op else _Done()


class LoopbackComm:
    """All partitions in one process (single-device tests): the all-to-all as copies."""

    def __init__(self, world: int):
        self.rank, self.world = 0, world

    def alltoall_ids(self, sends: list) -> list:
        return [[sends[src][dst] for src in range(self.world)] for dst in range(self.world)]

    def exchange(self, sends, send_counts, recvs, recv_counts, async_op):
        W = self.world
        soff = [np.cumsum([0] + list(c)) for c in send_counts]
        roff = [np.cumsum([0] + list(c)) for c in recv_counts]
        for src in range(W):
            for dst in range(W):
                n = send_counts[src][dst]
                if n != recv_counts[dst][src]:
                    raise RuntimeError("halo count mismatch %d->%d" % (src, dst))
                if n:
                    recvs[dst][roff[dst][src]:roff[dst][src] + n].copy_(sends[src][soff[src][dst]:soff[src][dst] + n])
        return _Done()


# ---------------------------------------------------------------------------------------------
class EdgeCutForward:
    """Forward of a partitioned graph through the stepped C ABI.

    ``parts``: the LocalParts this process runs (one per process with TorchComm).  All of them
    share ``engine`` (one plan per device) and the torch current stream, which the engine is
    bound to so that packing, RCCL and the MP kernels are stream-ordered."""

    def __init__(self, engine: Engine, parts: list, comm, overlap: bool = True):
        import torch
        self.torch = torch
        self.engine, self.parts, self.comm, self.overlap = engine, parts, comm, overlap
        plan = engine.plan
        self.plan = plan
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        self.batches, self.bufs, self.send_idx, self.send_buf = [], [], [], []
        # every rank must call the same collectives: the exchanged entities are those read as a source
        srcs = {s.src for s in plan.adj_slots}
        halo_ents = [n for n in plan.entities if n in srcs] if comm.world > 1 else []
        self.halo_ents = halo_ents
        dev = torch.device("cuda", torch.cuda.current_device())
        for p in parts:
            b = Batch(engine, [p.inputs], halo_rows={n: p.halos[n].n_halo for n in plan.entities})
            bufs, sidx, sbuf = {}, {}, {}
            for n in halo_ents:
                e = plan.entities.index(n)
                H = plan.hidden[e]
                h = p.halos[n]
                cap = (h.n_owned + h.n_halo) * H + 256
                pair = (torch.empty(cap, dtype=torch.float32, device=dev), torch.empty(cap, dtype=torch.float32, device=dev))
                for t in pair:
                    t.zero_()
                b.bind_state(n, *pair)
                bufs[n] = pair
                sidx[n] = torch.from_numpy(np.ascontiguousarray(h.send_rows, np.int32)).to(dev)
                sbuf[n] = torch.empty((len(h.send_rows), H), dtype=torch.float32, device=dev)
            self.batches.append(b)
            self.bufs.append(bufs)
            self.send_idx.append(sidx)
            self.send_buf.append(sbuf)
        self.edges_per_forward = sum(b.edges_per_forward for b in self.batches)
        self.mp_sources = [sorted({plan.entities[s[0]] for s in m["sources"]}) for m in plan.mps]

    def _exchange(self, name, async_op):
        e = self.plan.entities.index(name)
        H = self.plan.hidden[e]
        sends, recvs, sc, rc = [], [], [], []
        for i, p in enumerate(self.parts):
            h = p.halos[name]
            cur = self.bufs[i][name][self.batches[i].state_slot(name)]
            state = cur[:(h.n_owned + h.n_halo) * H].view(h.n_owned + h.n_halo, H)
            if len(h.send_rows):
                self.engine.gather_rows(state, self.send_idx[i][name], self.send_buf[i][name])
            sends.append(self.send_buf[i][name])
            recvs.append(state[h.n_owned:])
            sc.append(h.send_counts)
            rc.append(h.recv_counts)
        return self.comm.exchange(sends, sc, recvs, rc, async_op)

    def forward(self, to_host: bool = True):
        for b in self.batches:
            b.begin()
        stale = set(self.halo_ents)                # halo rows of the initial state come from peers too
        for _ in range(self.plan.iterations):      # GM:406
            for mi, m in enumerate(self.plan.mps):
                need = [n for n in self.mp_sources[mi] if n in stale]
                if need and self.overlap and _overlappable(m):
                    works = [self._exchange(n, True) for n in need]
                    for b in self.batches:
                        b.run_mp(mi, "interior")
                    for w in works:
                        w.wait()
                    for b in self.batches:
                        b.run_mp(mi, "boundary")
                else:
                    for n in need:
                        self._exchange(n, False).wait()
                    for b in self.batches:
                        b.run_mp(mi, "all")
                stale -= set(need)
                dst = self.plan.entities[m["dst"]]
                if dst in self.halo_ents:
                    stale.add(dst)                 # the new buffer's halo rows are two updates old
        return [b.end(to_host) for b in self.batches]

    def close(self):
        for b in self.batches:
            b.close()


# ---------------------------------------------------------------------------------------------
class _DeviceRows:
    """A device buffer the engine owns, seen by torch without a copy (__cuda_array_interface__)."""

    def __init__(self, ptr: int, rows: int, cols: int):
        self.__cuda_array_interface__ = {"shape": (rows, cols), "typestr": "<f4", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


class EdgeCutTraining:
    """One training step (model_fn TRAIN, GM:697-830) on a partitioned graph, through the stepped
    C ABI (ign_forward_train_* / ign_backward_*).

    Forward: every state version keeps owned + halo rows; before an MP reads an entity whose halo
    rows are stale, the owners send them (as EdgeCutForward does, into the version's halo rows).
    Backward: the gradient of a halo row belongs to its owner -- after each MP instance, the halo
    rows of every source entity's current gradient go back to their owners (the reverse all-to-all),
    who add them to their rows (peer by peer: deterministic), and are zeroed.  The loss is the MSE
    over every rank's predictions, the parameter gradients are summed over ranks (each rank's l2
    terms weighted 1/ranks), so one step equals the whole graph's step up to summation order."""

    def __init__(self, engine: Engine, parts: list, comm):
        import torch
        self.torch = torch
        self.engine, self.parts, self.comm = engine, parts, comm
        plan = engine.plan
        self.plan = plan
        for m in plan.mps:
            if m["aggr"] not in ("sum", "convolution"):
                raise ValueError("edge-cut training supports sum and convolution MPs")
        engine.set_stream(torch.cuda.current_stream().cuda_stream)
        srcs = {s.src for s in plan.adj_slots}
        self.halo_ents = [n for n in plan.entities if n in srcs] if comm.world > 1 else []
        self.dev = torch.device("cuda", torch.cuda.current_device())
        self.batches, self.send_idx, self.recv_idx = [], [], []
        for p in parts:
            b = Batch(engine, [p.inputs], halo_rows={n: p.halos[n].n_halo for n in plan.entities})
            b.enable_training()
            self.batches.append(b)
            sidx, ridx = {}, {}
            for n in self.halo_ents:
                h = p.halos[n]
                sidx[n] = torch.from_numpy(np.ascontiguousarray(h.send_rows, np.int64)).to(self.dev)
                offs = np.cumsum([0] + list(h.send_counts))
                ridx[n] = [(int(offs[q]), int(offs[q + 1])) for q in range(len(h.send_counts))]
            self.send_idx.append(sidx)
            self.recv_idx.append(ridx)
        self.mp_sources = [sorted({plan.entities[s[0]] for s in m["sources"]}) for m in plan.mps]
        self.grads = [torch.zeros(engine.n_params, dtype=torch.float32, device=self.dev) for _ in parts]

    def _rows(self, i, name, ptr):
        h = self.parts[i].halos[name]
        H = self.plan.hidden[self.plan.entities.index(name)]
        return self.torch.as_tensor(_DeviceRows(ptr, h.n_owned + h.n_halo, H), device=self.dev)

    def _exchange_states(self, name):
        sends, recvs, sc, rc = [], [], [], []
        for i, p in enumerate(self.parts):
            h = p.halos[name]
            state = self._rows(i, name, self.batches[i].train_buffers(name)[0])
            sends.append(state.index_select(0, self.send_idx[i][name]).contiguous())
            recvs.append(state[h.n_owned:])
            sc.append(h.send_counts)
            rc.append(h.recv_counts)
        self.comm.exchange(sends, sc, recvs, rc, False).wait()

    def _return_gradients(self, name):
        """Halo rows' gradients back to their owners, added there, zeroed here."""
        torch = self.torch
        grads, sends, recvs, sc, rc = [], [], [], [], []
        for i, p in enumerate(self.parts):
            h = p.halos[name]
            g = self._rows(i, name, self.batches[i].train_buffers(name)[1])
            grads.append(g)
            sends.append(g[h.n_owned:].contiguous())
            recvs.append(torch.empty((len(h.send_rows), g.shape[1]), dtype=torch.float32, device=self.dev))
            sc.append(h.recv_counts)      # what this rank received from each peer goes back to it
            rc.append(h.send_counts)
        self.comm.exchange(sends, sc, recvs, rc, False).wait()
        for i, p in enumerate(self.parts):
            h = p.halos[name]
            for q, (a, b) in enumerate(self.recv_idx[i][name]):   # peer by peer: unique rows, fixed order
                if b > a:
                    grads[i].index_add_(0, self.send_idx[i][name][a:b], recvs[i][a:b])
            grads[i][h.n_owned:].zero_()

    def step(self, labels: list, to_host: bool = True):
        """Forward + loss + backward; ``labels``: per partition, its owned predictions' labels.
        Returns (loss over all ranks, summed parameter gradient, per-partition predictions or
        None when not ``to_host``)."""
        torch = self.torch
        plan, M = self.plan, len(self.plan.mps)
        for b in self.batches:
            b.forward_train_begin()
        stale = set(self.halo_ents)
        for _ in range(plan.iterations):                      # GM:406
            for mi, m in enumerate(plan.mps):
                for n in [n for n in self.mp_sources[mi] if n in stale]:
                    self._exchange_states(n)
                    stale.discard(n)
                for b in self.batches:
                    b.forward_train_mp()
                dst = plan.entities[m["dst"]]
                if dst in self.halo_ents:
                    stale.add(dst)
        preds = [b.forward_train_end(to_host=to_host) for b in self.batches]
        ys = self._labels_dev(labels)
        n_local = sum(int(y.numel()) for y in ys)
        n_total = self._sum_scalar(float(n_local))
        loss = 0.0
        dpreds = []
        for b, y in zip(self.batches, ys):
            d = torch.empty_like(y)
            loss += self.engine.mse_loss(b.predictions_ptr(), y, d) * y.numel() / n_total
            dpreds.append(d * (y.numel() / n_total))   # d(mean over every rank) = d(local mean) n_local / N
        loss = self._sum_scalar(loss)
        world = self.comm.world
        for b, d, g in zip(self.batches, dpreds, self.grads):
            b.backward_begin(d, g, 1.0 / world)
        for k in range(plan.iterations * M - 1, -1, -1):      # MP instances in reverse
            for b in self.batches:
                b.backward_mp()
            for n in self.mp_sources[k % M]:
                if n in self.halo_ents:
                    self._return_gradients(n)
        for b in self.batches:
            b.backward_end()
        total = self.grads[0].clone()
        for g in self.grads[1:]:
            total += g
        total = self._sum_tensor(total)
        return loss, total, preds

    def _labels_dev(self, labels):
        """Device label vectors, uploaded once per distinct labels object (a bench repeats them)."""
        key = tuple(id(l) for l in labels)
        if getattr(self, "_lab_key", None) != key:
            self._lab_key, self._lab_src = key, list(labels)   # the references keep the ids unique
            self._lab = [self.torch.from_numpy(np.ascontiguousarray(np.asarray(l, np.float32).reshape(-1))).to(self.dev)
                         for l in labels]
        return self._lab

    def _sum_scalar(self, v: float) -> float:
        if isinstance(self.comm, LoopbackComm):
            return v
        dev = "cpu" if self.comm.host_staged else self.dev
        t = self.torch.tensor([v], dtype=self.torch.float64, device=dev)
        self.comm.dist.all_reduce(t, group=self.comm.group)
        return float(t.item())

    def _sum_tensor(self, g):
        if isinstance(self.comm, LoopbackComm):
            return g
        if self.comm.host_staged:
            h = g.cpu()
            self.comm.dist.all_reduce(h, group=self.comm.group)
            return h.to(g.device)
        self.comm.dist.all_reduce(g, group=self.comm.group)
        return g

    def close(self):
        for b in self.batches:
            b.close()
