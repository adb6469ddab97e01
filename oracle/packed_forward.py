"""ORACLE (test infrastructure only) — second, independent restatement: packed sequences.

Same algorithm as dense_forward.py (ComnetModel.call, GM:384-658) but written the way
the engine executes it: per destination, the list of message *positions* implied by the
dense padding (GM:477-543, AUX:421-440), a masked GRU over positions 0..final_len-1
(AUX:767-796), holes as zero inputs.  Agreement between the two restatements pins the
padding / interleave / masking semantics the engine's step tables encode.  Pure
Python loops: small graphs only.  Used only by tests/.
"""

from __future__ import annotations

import numpy as np

from .dense_forward import DenseOracle, OracleError, gru_cell


class PackedOracle(DenseOracle):
    def _message_passing(self, mp, state, x):
        dt = self.dtype
        dst = mp["destination_entity"]
        num_dst = int(np.asarray(x["num_" + dst]))
        aggr = mp["aggregation"]["type"]
        H_msg = None
        per_dst = [[] for _ in range(num_dst)]      # (position, message vector)
        final_len = np.zeros(num_dst, np.int64)
        slot_off = 0
        flat_idx = None
        if aggr == "interleave":
            flat_idx = np.concatenate([np.asarray(x["indices_" + s["name"] + "_to_" + dst], np.int64)
                                       for s in mp["source_entities"]])
        for src in mp["source_entities"]:
            sname, adj = src["name"], src["adj_vector"]
            src_idx = np.asarray(x["src_" + adj], np.int64)
            dst_idx = np.asarray(x["dst_" + adj], np.int64)
            seq = np.asarray(x["seq_" + sname + "_" + dst], np.int64)
            table = state[sname]
            H_msg = table.shape[1]
            lmax = int(seq.max()) + 1
            for k in range(len(src_idx)):
                pos = slot_off + int(seq[k])
                if flat_idx is not None:
                    pos = int(flat_idx[pos])
                per_dst[int(dst_idx[k])].append((pos, table[int(src_idx[k])].astype(dt)))
                final_len[int(dst_idx[k])] += 1
            slot_off += lmax
        if aggr in ("ordered", "interleave", "concat") and num_dst:
            # the padded sequence has slot_off steps (concat on axis 2: the first source's Lmax);
            # the masked RNN needs max(final_len) == that length (dense_forward.py, AUX:785-795)
            L_pad = slot_off if not (aggr == "concat" and int(mp["aggregation"]["concat_axis"]) == 2) else None
            if L_pad is not None and (final_len.max() < L_pad or final_len.max() > L_pad):
                raise OracleError("final_len width %d vs padded length %d" % (final_len.max(), L_pad))
        cell = self._cell(dst)
        old = state[dst]
        new = np.empty_like(old)
        for d in range(num_dst):
            if aggr == "sum":
                xsum = np.zeros(H_msg, dt)
                for _, v in per_dst[d]:
                    xsum = xsum + v
                new[d] = gru_cell(xsum[None, :], old[d:d + 1], *cell)[0]
            else:
                L = int(final_len[d])
                if L == 0:
                    raise OracleError("destination with no message (gather_nd -1)")
                h = old[d:d + 1]
                for t in range(L):
                    xt = np.zeros(H_msg, dt)
                    for pos, v in per_dst[d]:
                        if pos == t:
                            xt = xt + v
                    h = gru_cell(xt[None, :], h, *cell)
                new[d] = h[0]
        state[dst] = new
