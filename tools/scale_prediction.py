"""Predicted edge-cut numbers of the 1M-node / 10M-edge graph at N = 2, 4, 8.

For each N, every rank's partition of the seeded graph (partition.local_part, the code bench.py's
edge-cut leg runs): owned nodes, in-edges, halo rows and bytes per exchange, the rows it sends, the
largest per-peer message, and the interior share of its destinations (no message from a halo row:
they run during the exchange).  The prediction then prices one exchange on xGMI (each peer pair one
link, ~153 GB/s; the all-to-all's time = the largest per-link message over that rate, plus a fixed
per-collective cost) against the per-MP compute measured at N = 1, scaled by the rank's share of
the in-edges:

    per MP:   t_mp = max(t_exchange, interior share x t_compute) + boundary share x t_compute
    forward:  T x t_mp + readout / N

and a pessimistic line beside it: RCCL at --link-eff of the link rate and --fixed-us per MP for the
halo pack, the extra launches and the host's enqueue (neither is measured: the RCCL leg has never run).

Usage: python tools/scale_prediction.py [--nodes 1000000] [--n1-ms 4.37] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

LINK_GBS = 153.0          # one xGMI link, per direction (MI355X: 7 links per GPU, one per peer at N = 8)
COLLECTIVE_US = 25.0      # fixed cost of one RCCL all_to_all_single (launch + protocol), assumed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--n1-ms", type=float, default=4.37, help="measured N = 1 forward (BENCH_r05 edge_cut_1m)")
    ap.add_argument("--readout-ms", type=float, default=0.25, help="N = 1 readout share of the forward")
    ap.add_argument("--world", type=int, nargs="*", default=[2, 4, 8])
    ap.add_argument("--link-eff", type=float, default=0.6, help="pessimistic: fraction of the link rate RCCL reaches")
    ap.add_argument("--fixed-us", type=float, default=50.0, help="pessimistic: fixed cost per MP (pack, launches)")
    ap.add_argument("--json")
    a = ap.parse_args()
    from ignnition_amd import partition, workloads
    from ignnition_amd.engine import MPPlan
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=a.nodes)
    plan = MPPlan.from_model_info(mi)
    name, H, T = plan.entities[0], plan.hidden[0], plan.iterations
    g = graphs[0]
    total_edges = workloads.edges_per_forward(mi, graphs) // T
    mp_ms_n1 = (a.n1_ms - a.readout_ms) / T
    rows = []
    for world in a.world:
        ranks = []
        for r in range(world):
            part = partition.local_part(g, plan, r, world)
            h = part.halos[name]
            recv = np.asarray(h.recv_counts, np.int64)
            src = np.asarray(part.inputs[plan.adj_slots[0].keys[0]], np.int64)
            dst = np.asarray(part.inputs[plan.adj_slots[0].keys[1]], np.int64)
            n_own = h.n_owned
            remote_dst = np.unique(dst[src >= n_own])
            ranks.append({"owned": n_own, "in_edges": int(len(dst)), "halo_rows": h.n_halo,
                          "recv_by_peer": recv.tolist(), "boundary": int(len(remote_dst))})
        recv_m = np.asarray([x["recv_by_peer"] for x in ranks])          # [i][j]: rows i reads from j
        send_rows = recv_m.sum(axis=0)                                     # rows j sends in all
        link_max = int(recv_m.max()) * H * 4                               # largest per-pair message, bytes
        ex_ms = (link_max / (LINK_GBS * 1e9)) * 1e3 + COLLECTIVE_US * 1e-3
        worst = max(range(world), key=lambda k: ranks[k]["in_edges"])
        share = ranks[worst]["in_edges"] / total_edges
        c_ms = mp_ms_n1 * share
        f_int = 1.0 - ranks[worst]["boundary"] / ranks[worst]["owned"]
        t_mp = max(ex_ms, f_int * c_ms) + (1 - f_int) * c_ms
        t_mp_noov = ex_ms + c_ms
        fwd = T * t_mp + a.readout_ms / world
        ex_p = (link_max / (LINK_GBS * a.link_eff * 1e9)) * 1e3 + COLLECTIVE_US * 1e-3
        fwd_p = T * (max(ex_p, f_int * c_ms) + (1 - f_int) * c_ms + a.fixed_us * 1e-3) + a.readout_ms / world
        rows.append({"n": world, "owned_per_rank": ranks[worst]["owned"],
                     "in_edges_max_rank": ranks[worst]["in_edges"],
                     "halo_rows_max_rank": int(max(x["halo_rows"] for x in ranks)),
                     "halo_mb_per_exchange_max_rank": round(max(x["halo_rows"] for x in ranks) * H * 4 / 1e6, 2),
                     "send_rows_max_rank": int(send_rows.max()),
                     "largest_peer_message_mb": round(link_max / 1e6, 2),
                     "interior_share": round(f_int, 3),
                     "exchange_ms_pred": round(ex_ms, 4), "compute_ms_per_mp_pred": round(c_ms, 4),
                     "ms_per_step_pred": round(fwd, 3), "ms_per_step_pred_no_overlap": round(T * t_mp_noov + a.readout_ms / world, 3),
                     "edges_per_s_pred": round(total_edges * T / (fwd * 1e-3), -7),
                     "exchange_ms_pessimistic": round(ex_p, 4), "ms_per_step_pessimistic": round(fwd_p, 3),
                     "edges_per_s_pessimistic": round(total_edges * T / (fwd_p * 1e-3), -7)})
        print(json.dumps(rows[-1]), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"nodes": a.nodes, "hidden": H, "iterations": T, "link_gbs": LINK_GBS,
                       "collective_us": COLLECTIVE_US, "n1_ms": a.n1_ms, "link_eff_pessimistic": a.link_eff,
                       "fixed_us_pessimistic": a.fixed_us, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
