"""Throughput benchmark: message-passing edges/s, RouteNet synth50 batched (BASELINE.json).

One "step" = one full forward of the engine over one batch (hidden-state init, T=8
iterations of link->path ordered GRU + path->link sum GRU, readout MLP) with every input
already resident in HBM.  edges per step = B x T x sum_mp sum_src |adj|.

Multi-GPU (torchrun): one process per GPU, each rank owns its own batch of 512 graphs
(graph-sharded, weak scaling; the forward has no data-path collective).  Timing: barrier +
device sync on both sides of exactly K steps; the max over ranks is reported.

Extra objects on the JSON line:
  roofline      dominant kernel (most time in the warm-up), on its binding roof:
                algorithmic FLOPs (mfma, peak fp32 MFMA 157.3 TFLOP/s) or bytes (hbm, 8 TB/s)
                per launch / average launch time from HIP events recorded on the engine stream
                around that kernel's launches in the timed region; traffic = HBM bytes per
                launch from the committed rocprofv3 PMC summary (profiles/), or null.
                warmup_kernels: every kernel kind, timed during the warm-up.
  cpu_baseline  the dense-padded oracle (oracle/dense_forward.py, float32 numpy, the TF op
                sequence incl. padded work) on a bounded sample of the same workload, rank 0, N=1,
                one process per CPU this process may use (CPU model and count on the line).
  cpu_baseline_cxx  the second CPU line: the C++/OpenMP float32 restatement
                (oracle/cpu_forward.cpp) on the same sample and CPUs.
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "message-passing edges/sec, RouteNet synth50 batched, 1/2/4/8 MI355X"
PEAK_FP32_MFMA_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0
PEAK_BF16_MFMA_TFLOPS = 2500.0   # dense bf16 (MI355X_MICROARCH.md), the split-bf16 kernels' pipe
CLOCK_GHZ = 2.4                  # MI355X peak engine clock (spec), the issue roof's clock
N_CU = 256
RES_KERNEL = {0: "_Z23resident_forward_kernelILb0ELb1ELb0EEv12ResidentArgs",   # form -> instance (resident.hip)
              1: "_Z23resident_forward_kernelILb1ELb1ELb0EEv12ResidentArgs",
              2: "_Z23resident_forward_kernelILb1ELb0ELb0EEv12ResidentArgs"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--graphs", type=int, default=512, help="graphs per GPU")
    ap.add_argument("--topology", default="synth50")
    ap.add_argument("--model", default="routenet", choices=["routenet", "qsize", "synthetic"],
                    help="synthetic = the 1M-node / 10M-edge graph of BASELINE configs[4] (one graph per rank)")
    ap.add_argument("--nodes", type=int, default=1_000_000, help="synthetic graph size")
    ap.add_argument("--train", action="store_true",
                    help="time the training step (forward keeping activations, MSE, backward, gradient "
                         "all-reduce over ranks, Adam) instead of the forward")
    ap.add_argument("--fresh-batches", action="store_true",
                    help="with --train: time the real train_and_evaluate loop (tar.gz reader -> normalisation -> "
                         "batch build -> step, every step a new shuffled batch of the rank's dataset), with the "
                         "next batches built on a worker thread")
    ap.add_argument("--no-prefetch", action="store_true", help="with --fresh-batches: build each batch inline")
    ap.add_argument("--input-workers", type=int, default=8, help="with --fresh-batches: batch-building threads")
    ap.add_argument("--streams", type=int, default=0,
                    help="forward: the rank's graphs as this many sub-batches, one engine / HIP stream each, "
                         "launched back to back in every step (their kernels co-run); 0 = auto: 4 for graphs "
                         "of fewer than 1000 paths or models of 3+ MPs per iteration (Q-size), else 2")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="skip per-kernel HIP event timing")
    ap.add_argument("--no-edge-cut", action="store_true",
                    help="skip the edge-cut leg (the 1M-node / 10M-edge graph of BASELINE configs[4] split across "
                         "the same ranks, RCCL halo all-to-all per MP; at N=1 the whole graph on one GPU), which "
                         "otherwise runs after the main measurement and is reported under 'edge_cut_1m'")
    ap.add_argument("--edge-cut-nodes", type=int, default=1_000_000, help="edge-cut leg: synthetic graph size")
    ap.add_argument("--edge-cut-steps", type=int, default=0, help="edge-cut leg: timed forwards (0: --steps)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: every rank builds its shard's host inputs and runs the barrier / max-over-ranks "
                         "timing / edge-sum reduction around K empty steps (gloo); rank 0 prints the line with "
                         "value null.  Checks the N-rank plumbing on a CPU-only host")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list) -> int:
    """``bench.py --gpus N`` started as one process (WORLD_SIZE unset): run N ranks of this same
    command under torch.distributed.run, one per GPU of this node, as a CHILD process -- this
    process has not touched the GPU and does not exec -- and return its exit code.  Rank 0's
    JSON line reaches our stdout unchanged (the child inherits it)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver (RCCL)
    sys.stdout.flush()
    return subprocess.call(cmd, env=env)


def load_traffic(kernel_kind, workload):
    path = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as fh:
            d = json.load(fh)
        return d.get(workload, {}).get(kernel_kind, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share():
    """CPUs this process may use: its affinity set, capped by OMP_NUM_THREADS when the launcher
    sets it (the GPU box grants 16 CPUs per GPU and sets it to 16; os.cpu_count() shows the whole
    host there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else max(1, n)


def _cpu_worker(job):
    """One process of the CPU baseline: the dense oracle, one BLAS thread, graph after graph of
    its share until the shared deadline."""
    desc, dims, prm, graphs, t_end = job
    import numpy as np
    from threadpoolctl import threadpool_limits

    from ignnition_amd import workloads
    from ignnition_amd.json_operations import Model_information
    from oracle.dense_forward import DenseOracle
    ora = DenseOracle(desc, dims, prm, dtype=np.float32)
    mi = Model_information(desc, dims)
    done = edges = 0
    per_graph = [workloads.edges_per_forward(mi, [g]) for g in graphs]
    with threadpool_limits(limits=1):
        while time.time() < t_end:     # cycles over its share until the deadline
            k = done % len(graphs)
            ora.forward([graphs[k]])
            edges += per_graph[k]
            done += 1
    return done, edges


def cpu_baseline(desc, dims, prm, graphs, budget_s, what="synth50 graphs"):
    """The dense-padded numpy oracle (the TF op sequence incl. padded rows) on every CPU this
    process may use, one process per CPU with one BLAS thread each, graphs dealt round-robin,
    for ``budget_s`` seconds of wall time.  Forked before the process touches the GPU."""
    import multiprocessing as mproc
    n = _cpu_share()
    graphs = list(graphs)
    while len(graphs) < n:
        graphs = graphs + graphs
    _cpu_worker((desc, dims, prm, graphs[:1], time.time()))   # imports, before the clock starts
    t0 = time.time()
    jobs = [(desc, dims, prm, graphs[k::n], t0 + budget_s) for k in range(n)]
    # close + join, not the context manager's terminate(): SIGTERM to the workers hangs them under
    # rocprofv3 (its preloaded signal handler), and the profile pass runs this same command
    pool = mproc.get_context("fork").Pool(n)
    try:
        res = pool.map(_cpu_worker, jobs)
        pool.close()
    except BaseException:
        pool.terminate()
        raise
    finally:
        pool.join()
    dt = time.time() - t0
    done = sum(r[0] for r in res)
    edges = sum(r[1] for r in res)
    return {"value": edges / dt, "unit": "edges/s", "cores": n, "kind": "port",
            "cpu_model": _cpu_model(), "host_cpus": os.cpu_count(),
            "sample": "%d forwards of %s (full T=8 each; %d distinct) in %.1f s on %d processes x 1 BLAS "
                      "thread, dense-padded numpy float32 oracle (TF op sequence incl. padded rows)"
                      % (done, what, len(set(map(id, graphs))), dt, n)}


def cpu_baseline_cxx(plan, mi, prm, graphs, budget_s, what="synth50 graphs"):
    """SURVEY §8(d)'s second CPU line: the C++/OpenMP float32 restatement (oracle/cpu_forward.cpp,
    packed per destination, no padded work) on the same sample, OpenMP over graphs (or over the
    destinations of one large graph) on every CPU this process may use.  None if it cannot be built."""
    from ignnition_amd import workloads
    try:
        from oracle import cpu_oracle
        cpu_oracle.build()
    except Exception as e:   # no g++ / OpenMP on the host: report why instead of failing the bench
        return {"value": None, "unit": "edges/s", "kind": "port", "error": str(e)[:200]}
    n = _cpu_share()
    graphs = list(graphs)
    per = max(2 * n, 32) if len(graphs) > 1 else 1
    chunks = [graphs[k:k + per] for k in range(0, len(graphs), per)]
    chunk_edges = [workloads.edges_per_forward(mi, c) for c in chunks]
    cpu_oracle.cpu_forward(plan, chunks[0][:1], prm, n)   # load + first touch, before the clock
    t0 = time.time()
    done = edges = k = 0
    while time.time() - t0 < budget_s or done == 0:
        cpu_oracle.cpu_forward(plan, chunks[k % len(chunks)], prm, n)
        edges += chunk_edges[k % len(chunks)]
        done += len(chunks[k % len(chunks)])
        k += 1
    dt = time.time() - t0
    return {"value": edges / dt, "unit": "edges/s", "cores": n, "kind": "port", "cpu_model": _cpu_model(),
            "sample": "%d forwards of %s (full T=8 each) in %.1f s, OpenMP %d threads, C++ float32 restatement "
                      "(oracle/cpu_forward.cpp: packed per destination, no padded work)" % (done, what, dt, n)}


def _reduce(dist, vals, op, device=None):
    """Element-wise MAX or SUM of a list of numbers over the ranks (unchanged without ``dist``)."""
    if dist is None:
        return [float(v) for v in vals]
    import torch
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t.cpu().tolist()


def edge_cut_key(nodes: int) -> str:
    return "edge_cut_1m" if nodes == 1_000_000 else "edge_cut_%dn" % nodes


def edge_cut_parts(args, dist, rank, world):
    """The edge-cut leg's host side: the seeded synthetic graph (every rank generates the same one),
    its plan, and this rank's partition with its halo send lists (one all-to-all of ids)."""
    from ignnition_amd import partition, workloads
    from ignnition_amd.engine import MPPlan
    desc, dims, mi, graphs, _ = workloads.make_synthetic_inputs(n_nodes=args.edge_cut_nodes)
    plan = MPPlan.from_model_info(mi)
    part = None
    if world > 1:
        part = partition.local_part(graphs[0], plan, rank, world)
    return mi, plan, graphs, part


def edge_cut_leg(args, dist, rank, world, device, backend):
    """SURVEY §8(e) / BASELINE configs[4], run in the same ranks after the main measurement: the
    synthetic 1M-node / 10M-edge graph (H=64, T=8, sum + GRU, predict readout) edge-cut across the
    ``world`` ranks.  Contiguous node ranges, owner computes by destination; before every MP the
    halo rows go to their readers with one RCCL ``all_to_all_single`` while the interior
    destinations run (partition.EdgeCutForward).  At N=1 the whole graph runs on one GPU
    (Batch.forward), so the driver's N=1 and N=8 lines time the same work (strong scaling).
    Returns the JSON object of the leg (identical on every rank)."""
    import torch
    from ignnition_amd import partition, workloads
    from ignnition_amd.engine import Batch, Engine
    steps = args.edge_cut_steps or args.steps
    t_build = time.perf_counter()
    mi, plan, graphs, part = edge_cut_parts(args, dist, rank, world)
    name, H, T = plan.entities[0], plan.hidden[0], plan.iterations
    torch.cuda.set_device(device)
    eng = Engine(plan, device)
    eng.set_params(plan.init_params(seed=0, bias_scale=0.05))
    dev = torch.device("cuda", device) if backend == "nccl" else None
    fw = batch = None
    halo = send = 0
    if world > 1:
        if backend == "nccl":
            comm = partition.TorchComm(dist, torch.device("cuda", device))
        else:   # gloo rehearsal (several ranks on one GPU): rows staged through host memory
            comm = partition.TorchComm(dist, None, host_staged=True)
        partition.exchange_requests([part], comm)
        fw = partition.EdgeCutForward(eng, [part], comm)
        step = lambda: fw.forward(to_host=False)
        edges = fw.edges_per_forward
        halo, send = part.halos[name].n_halo, len(part.halos[name].send_rows)
        interior, boundary = fw.batches[0].mp_split(0)
    else:
        batch = Batch(eng, graphs)
        step = lambda: batch.forward(to_host=False)
        edges = batch.edges_per_forward
        interior, boundary = batch.rows[0], 0
    t_build = time.perf_counter() - t_build

    def sync():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize(device)

    def timed(fn, k):
        sync()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        sync()
        return time.perf_counter() - t0

    for _ in range(max(args.warmup, 1)):
        step()
    dt = timed(step, steps)
    res = {"metric": "message-passing edges/sec, synthetic 1M-node / 10M-edge graph (BASELINE configs[4])",
           "unit": "edges/s", "n_ranks": dist.get_world_size() if dist is not None else 1, "steps": steps,
           "warmup": max(args.warmup, 1), "scaling": "strong", "nodes": args.edge_cut_nodes, "hidden": H,
           "iterations": T}
    ex_ms = nov_ms = None
    if fw is not None:
        # the same forward with every exchange completed before its MP starts (no interior overlap)
        fw.overlap = False
        for _ in range(2):
            step()
        nov = timed(step, steps)
        fw.overlap = True
        # one exchange alone (halo pack + all_to_all_single), repeated: what one MP's exchange costs
        reps = 4 * T
        for _ in range(2):
            fw._exchange(name, False).wait()
        ex = timed(lambda: fw._exchange(name, False).wait(), reps)
        dt, nov, ex = _reduce(dist, [dt, nov, ex], "max", dev)
        ex_ms, nov_ms = ex / reps * 1e3, nov / steps * 1e3
    else:
        dt, = _reduce(dist, [dt], "max", dev)
    tot_edges, tot_halo, tot_send, tot_int, tot_bnd = _reduce(dist, [edges, halo, send, interior, boundary], "sum",
                                                              dev)
    max_halo, = _reduce(dist, [halo], "max", dev)
    whole = workloads.edges_per_forward(mi, graphs)
    res.update({"value": tot_edges * steps / dt, "ms_per_step": dt / steps * 1e3,
                "edges_per_step": int(tot_edges), "edges_per_step_whole_graph": int(whole),
                "partition": ("contiguous node ranges over %d ranks, owner computes by destination; halo rows "
                              "exchanged per MP with RCCL all_to_all_single, interior destinations overlapped"
                              % world) if world > 1 else "whole graph on one GPU (no exchange)",
                "halo_rows": {"max_rank": int(max_halo), "total": int(tot_halo)},
                "halo_bytes_per_exchange": {"max_rank": int(max_halo) * H * 4, "total": int(tot_halo) * H * 4},
                "exchanges_per_step": T if world > 1 else 0,
                "exchange_ms_isolated": None if ex_ms is None else round(ex_ms, 4),
                "ms_per_step_no_overlap": None if nov_ms is None else round(nov_ms, 4),
                "interior_destinations": int(tot_int), "boundary_destinations": int(tot_bnd),
                "transport": ("RCCL" if backend == "nccl" else "gloo, host-staged (rehearsal)") if world > 1 else None,
                "edges_match_whole_graph": int(tot_edges) == int(whole),
                "build_s": round(t_build, 3)})
    if fw is not None:
        fw.close()
    if batch is not None:
        batch.close()
    eng.close()
    return res


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:   # the driver's `bench.py --gpus N`: start the N ranks ourselves
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit("bench.py: WORLD_SIZE=%s but --gpus %d; launch with --nproc-per-node equal to --gpus"
                 % (os.environ["WORLD_SIZE"], args.gpus))
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # IGN_DIST_BACKEND=gloo + IGN_BENCH_DEVICE=0 rehearse the N>1 path on a one-GPU box
    backend = "gloo" if args.dry_run else os.environ.get("IGN_DIST_BACKEND", "nccl")
    device = int(os.environ.get("IGN_BENCH_DEVICE", local))
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(device)
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    import numpy as np

    from ignnition_amd import workloads
    from ignnition_amd.engine import Batch, Engine, MPPlan, SplitBatch

    fresh_stats = None   # --fresh-batches: the main thread's wait for the next batch vs the step itself
    engines = []   # every engine of the step (--streams: one per sub-batch)
    subs = []      # --streams: the sub-batches
    batches = []   # the forward's batches (resident_info)

    def barrier_sync(_eng=None):
        for e in engines:
            e.synchronize()
        if dist is not None:
            dist.barrier()
            for e in engines:
                e.synchronize()

    def set_timing(on, kinds=None):
        for e in engines:
            e.set_timing(on, kinds=kinds)

    def stats_all():   # per kind, summed over the engines
        tot = None
        for e in engines:
            st = e.stats()
            if tot is None:
                tot = st
            else:
                for kind, v in st.items():
                    for f, x in v.items():
                        tot[kind][f] += x
        return tot

    synthetic = args.model == "synthetic"
    cleanup = []
    if synthetic:
        # one graph edge-cut across the ranks (strong scaling): every rank generates the same seeded
        # graph, keeps its node range and in-edges, and exchanges halo rows over RCCL (partition.py)
        args.graphs, args.topology = 1, "1m" if args.nodes == 1_000_000 else str(args.nodes)
        desc, dims, mi, graphs, labels = workloads.make_synthetic_inputs(n_nodes=args.nodes)
    else:
        # per-rank shard: graphs [rank*G, (rank+1)*G) -> weak scaling, no forward collective
        ids = workloads.shard_graph_ids(rank, world, args.graphs)
        desc, dims, mi, graphs, labels = workloads.make_batch_inputs(args.model, args.topology, len(ids),
                                                                     first_id=ids[0])
    plan = MPPlan.from_model_info(mi)
    prm = plan.init_params(seed=0, bias_scale=0.05)
    if args.dry_run:
        return dry_run(args, dist, rank, world, mi, graphs, synthetic)
    cpu = cpu_cxx = None
    if world == 1 and not args.no_cpu and not args.train:
        # before anything touches the GPU: the baseline's worker processes are forked
        if synthetic:
            # bounded sample: 25k-node graphs from the same generator (same degree law and locality)
            sd, sdims, _, sg, _ = workloads.make_synthetic_inputs(n_nodes=25_000)
            cpu = cpu_baseline(sd, sdims, prm, sg, args.cpu_seconds, "a 25k-node / 250k-edge synthetic graph")
            cpu_cxx = cpu_baseline_cxx(plan, mi, prm, sg, args.cpu_seconds, "a 25k-node / 250k-edge synthetic graph")
        else:
            cpu = cpu_baseline(desc, dims, prm, graphs, args.cpu_seconds)
            cpu_cxx = cpu_baseline_cxx(plan, mi, prm, graphs, args.cpu_seconds)
    eng = Engine(plan, device if world > 1 else 0)
    eng.set_params(prm)
    engines.append(eng)
    t_build = time.perf_counter()
    halo_rows = 0
    if args.streams <= 0:
        # auto: more, smaller sub-batches where the kernels are short -- small graphs (GEANT2, NSFNET)
        # or, on the batched launches, a step of three or more MPs per iteration (Q-size: 4.15-4.18
        # ms/step with 4 streams against 4.39-4.41 with 2; profiles/r04/streams/).  On the
        # graph-resident forward Q-size takes 2 (3.247 ms against 3.316 with 1 and 3.308 with 4,
        # profiles/r05/streams/), RouteNet synth50 2 (flat from 2 to 4 in round 4)
        sizes = [int(np.asarray(g[k]).reshape(())) for g in graphs[:1] for k in g if k.startswith("num_")]
        batched = os.environ.get("IGN_RESIDENT") == "0"
        args.streams = 4 if (sizes and max(sizes) < 1000) or (batched and len(plan.mps) >= 3) else 2
    if synthetic and world > 1:
        import torch
        from ignnition_amd import partition
        torch.cuda.set_device(device)
        if backend == "nccl":
            comm = partition.TorchComm(dist, torch.device("cuda", device))
        else:   # gloo rehearsal (several ranks on one GPU): rows staged through host memory
            comm = partition.TorchComm(dist, None, host_staged=True)
        part = partition.local_part(graphs[0], plan, rank, world)
        partition.exchange_requests([part], comm)
        halo_rows = part.halos[plan.entities[0]].n_halo
        if args.train:   # one optimizer step of the partitioned graph (halo states / gradients exchanged)
            tr = partition.EdgeCutTraining(eng, [part], comm)
            r = part.ranges[plan.entities[0]]
            lab = np.asarray(labels[0], np.float32).reshape(-1)[r[rank]:r[rank + 1]]
            m_state = torch.zeros(eng.n_params, dtype=torch.float32, device=tr.dev)
            v_state = torch.zeros_like(m_state)
            it_box = [0]

            def step():
                _, g, _ = tr.step([lab], to_host=False)
                eng.adam_step(g, m_state, v_state, it_box[0], 1e-3)
                it_box[0] += 1
            edges = tr.batches[0].edges_per_forward
            gru_steps = tr.batches[0].gru_steps_per_forward
            cleanup.append(tr.close)
        else:
            fw = partition.EdgeCutForward(eng, [part], comm)
            step = lambda: fw.forward(to_host=False)
            edges = fw.edges_per_forward
            gru_steps = fw.batches[0].gru_steps_per_forward
    elif args.train and args.fresh_batches:
        # the real input pipeline: write the rank's graphs as a tar.gz dataset in the reference
        # layout, then every step reads a new shuffled batch through the native reader
        import tempfile

        import torch
        from ignnition_amd import generate_model as gm
        from ignnition_amd import synthetic as synth_data   # (the name `synthetic` is the --model flag here)
        from ignnition_amd.training import Trainer
        torch.cuda.set_device(device if world > 1 else 0)
        tmp = tempfile.mkdtemp(prefix="ign_bench_")
        synth_data.write_tar_dataset(synth_data.dataset(args.topology, len(ids), first_id=ids[0]), os.path.join(tmp, "train"))
        gm.register_user_functions(workloads.USER_FUNCTIONS)
        gm.set_model_info(mi)
        trainer = Trainer(mi, params=prm, device=device if world > 1 else 0, dist=dist)
        eng = trainer.engine
        engines[:] = [eng]
        probe = Batch(eng, graphs)
        edges, gru_steps = probe.edges_per_forward, probe.gru_steps_per_forward
        probe.close()
        source = gm.NativeInput(os.path.join(tmp, "train"), shuffle=True, batch_size=len(ids), seed=1)
        if args.no_prefetch:
            batches = (trainer.prepare(*source.load(i)) for i in source.ids())
        else:
            batches = trainer.prefetch(source.ids(), depth=args.input_workers + 1, workers=args.input_workers,
                                       load=source.load)

        pipe_t = {"wait_s": 0.0, "step_s": 0.0, "steps": 0, "waits": []}

        def step():   # train_and_evaluate's loop (FO:108-166): next batch from the pipeline, one step
            t0 = time.perf_counter()
            nb = next(batches)
            t1 = time.perf_counter()
            # as framework_operations.train_and_evaluate: the loss reaches the host on logged steps only
            trainer.train_prepared(*nb, want_loss=pipe_t["steps"] % 10 == 0)
            pipe_t["wait_s"] += t1 - t0
            pipe_t["waits"].append(t1 - t0)
            pipe_t["step_s"] += time.perf_counter() - t1
            pipe_t["steps"] += 1
        pipe_t["trainer"] = trainer
        fresh_stats = pipe_t
        if not args.no_prefetch:
            cleanup.append(batches.close)
    elif args.streams > 1 and not args.train and len(graphs) > 1:
        # the rank's batch as K sub-batches of consecutive graphs on K plans / HIP streams
        # (engine.SplitBatch): the memory-bound sum update of one co-runs with the issue-bound
        # ordered update of another.  The same graphs and work per step as one batch.
        sb = SplitBatch(eng, graphs, args.streams)
        engines[:] = sb.engines
        subs += sb.parts
        step = lambda: sb.forward(to_host=False)
        edges = sb.edges_per_forward
        gru_steps = sb.gru_steps_per_forward
        batches += sb.parts
    else:
        batch = Batch(eng, graphs)
        batches.append(batch)
        step = lambda: batch.forward(to_host=False)
        edges = batch.edges_per_forward
        gru_steps = batch.gru_steps_per_forward
        if args.train:
            import torch
            torch.cuda.set_device(device if world > 1 else 0)
            eng.set_stream(torch.cuda.current_stream().cuda_stream)
            batch.enable_training()
            y = torch.from_numpy(np.concatenate([np.asarray(l, np.float32).reshape(-1) for l in labels])).cuda()
            dpred = torch.empty_like(y)
            grads = torch.zeros(eng.n_params, dtype=torch.float32, device=y.device)
            m_state, v_state = torch.zeros_like(grads), torch.zeros_like(grads)
            it_box = [0]

            def step():   # model_fn TRAIN (GM:712-818): one optimizer step on the rank's batch
                batch.forward_train(to_host=False)
                eng.mse_loss(batch.predictions_ptr(), y, dpred, want_loss=False)
                batch.backward(dpred, grads)
                if dist is not None:
                    dist.all_reduce(grads)
                eng.adam_step(grads, m_state, v_state, it_box[0], 1e-3)
                it_box[0] += 1
    t_build = time.perf_counter() - t_build

    # Warm-up with every launch timed (per-kind breakdown, picks the dominant kernel); the timed
    # region then records HIP event pairs around the dominant kernel's launches only, since each
    # pair adds a few microseconds of queue time (all ~35 launches per step: ~5 %).
    set_timing(not args.no_timing)
    for _ in range(max(args.warmup, 1)):
        step()
    barrier_sync()
    warm = stats_all()
    dom = max(("seq_gru", "sum_gru", "readout", "mp_resident"), key=lambda k: warm[k]["ms"])
    set_timing(not args.no_timing, kinds=[dom])
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier_sync()
    dt = time.perf_counter() - t0
    stats = stats_all()
    isolated = isolated_all = None
    if len(subs) > 1 and not args.no_timing and not args.train:
        # isolated leg, after the timed region: sub-batch 0 alone on the chip, its dominant kernel's
        # and the readout's launches timed (in the timed region the sub-batches' kernels co-run, so
        # there a launch's duration is its share of a chip it does not have to itself)
        set_timing(False)
        kinds = [dom] + (["readout"] if dom != "readout" else [])
        engines[0].set_timing(True, kinds=kinds)
        for _ in range(3):
            subs[0].forward(to_host=False)
        engines[0].synchronize()
        isolated_all = engines[0].stats()
        isolated = isolated_all[dom]
    for fn in cleanup:
        fn()
    dev = None
    if dist is not None and backend == "nccl":
        import torch
        dev = torch.device("cuda", device)
    dt, total_edges_step = workloads.reduce_step_stats(dist, dt, edges, dev)
    total_edges = total_edges_step * args.steps
    value = total_edges / dt
    edge_cut = None
    if not (synthetic or args.train or args.no_edge_cut):
        # BASELINE configs[4] in the same ranks: the 1M-node graph edge-cut over
        # RCCL at N>1, whole on one GPU at N=1; the main line's value stays the RouteNet metric
        edge_cut = edge_cut_leg(args, dist, rank, world, device if world > 1 else 0, backend)

    if rank != 0:
        dist.destroy_process_group()
        return

    def pipe(v):
        if v["ms"] <= 0 or (v["mfma_bf16"] <= 0 and v["mfma_f32"] <= 0):
            return None
        bf = v["mfma_bf16"] >= v["mfma_f32"]
        tf = (v["mfma_bf16"] if bf else v["mfma_f32"]) / (v["ms"] / 1e3) / 1e12
        peak = PEAK_BF16_MFMA_TFLOPS if bf else PEAK_FP32_MFMA_TFLOPS
        return {"dtype": "bf16|f16" if bf else "f32", "achieved_tflops": round(tf, 2), "peak_tflops": peak,
                "frac": round(tf / peak, 4)}

    workload = "%s_%s_x%d%s" % (args.model, args.topology, args.graphs,
                                ("_train_fresh" + ("" if args.no_prefetch else "_prefetch")) if args.fresh_batches
                                else "_train" if args.train else "")
    roof = None
    if not args.no_timing and not args.train and stats[dom]["ms"] > 0:
        s = stats[dom]
        launches = max(s["launches"], 1)
        avg_s = s["ms"] / launches / 1e3
        flops_launch = s["flops"] / launches
        bytes_launch = s["bytes"] / launches
        # the binding roof: whichever of bytes/BW and flops/peak is larger
        hbm_bound = bytes_launch / (PEAK_HBM_GBS * 1e9) > flops_launch / (PEAK_FP32_MFMA_TFLOPS * 1e12)
        if hbm_bound:
            achieved, peak, unit = bytes_launch / avg_s / 1e9, PEAK_HBM_GBS, "GB/s"
        else:
            achieved, peak, unit = flops_launch / avg_s / 1e12, PEAK_FP32_MFMA_TFLOPS, "TFLOP/s"
        roof = {"bound": "hbm" if hbm_bound else "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": peak,
                "unit": unit, "frac": round(achieved / peak, 4),
                "traffic": load_traffic(dom, workload),
                "alg_bytes_per_launch": bytes_launch, "alg_flops_per_launch": flops_launch,
                "avg_launch_ms": round(s["ms"] / launches, 4),
                "hbm_frac_alg": round(bytes_launch / avg_s / 1e9 / PEAK_HBM_GBS, 4),
                "mfma_frac_alg": round(flops_launch / avg_s / 1e12 / PEAK_FP32_MFMA_TFLOPS, 4),
                "timed_launches": s["launches"],
                "streams": len(engines),
                # the matrix pipe the kernel actually runs on: FLOPs its MFMAs execute (bf16 piece
                # products on the split-bf16 kernels) per launch time, against that pipe's dense peak
                "mfma_pipe": pipe(s),
                "warmup_kernels": {k: {"launches": v["launches"], "ms_total": round(v["ms"], 3),
                                       "tflops": round(v["flops"] / max(v["ms"], 1e-9) / 1e9, 2),
                                       "alg_gbs": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1),
                                       "mfma_pipe": pipe(v)}
                                   for k, v in warm.items() if v["launches"]}}
    seq_v = int(os.environ.get("IGN_SEQ_VARIANT", "6"))
    seq_v = seq_v if seq_v in (2, 4) else 6          # the engine's mapping (engine.cpp)
    ro_v = int(os.environ.get("IGN_READOUT_VARIANT", "4"))
    ro_v = ro_v if ro_v in (1, 2, 5) else 4
    sum_v = int(os.environ.get("IGN_SUM_VARIANT", "8"))
    BF = "split-bf16: exact 3-piece bf16 operands, %d products, fp32 accumulate"
    H16 = ("split-fp16: power-of-two-scaled 2-piece fp16 operands (RNE, 2^-22 relative), %d products, "
           "fp32 accumulate")
    seq_c = {2: "f32 MFMA", 4: BF % 6, 6: H16 % 3}
    ro_c = {1: "f32 MFMA", 2: BF % 6, 4: "both layers " + H16 % 3 + ", 16x16x32",
            5: "both layers " + H16 % 3 + ", 32x32x16"}
    contraction = {"ordered_update_hU": seq_c.get(seq_v, "f32 MFMA") if plan.hidden[0] in (32, 64) else "f32 MFMA",
                   "readout": ro_c.get(ro_v, BF % 6),
                   # sum variants 8 (default) / 7: split-fp16 / split-bf16 x.W and h.U at DIN = H = 64,
                   # split-bf16 at 32
                   "sum_update": (H16 % 3 if plan.hidden[0] == 64 and sum_v == 8 else BF % 6)
                   if plan.hidden[0] in (32, 64) and sum_v in (7, 8) else "f32 MFMA",
                   "projection": "f32 MFMA"}
    contraction["mp_resident"] = "ordered update %s; sum update %s" % (contraction["ordered_update_hU"],
                                                                     contraction["sum_update"])
    if roof is not None and isolated and isolated["launches"]:
        il = isolated["launches"]
        iavg = isolated["ms"] / il / 1e3
        iach = (isolated["bytes"] / il / iavg / 1e9) if roof["unit"] == "GB/s" else (isolated["flops"] / il / iavg / 1e12)
        roof["note"] = ("timed region: %d sub-batches on %d streams, so each launch of the kernel shares the chip "
                        "with the other sub-batches' kernels; 'isolated' is the same kernel alone" % (len(subs), len(subs)))
        roof["isolated"] = {"what": "sub-batch 0 (%d graphs) alone on the chip, after the timed region"
                                    % subs[0].num_graphs,
                            "launches": il, "avg_launch_ms": round(iavg * 1e3, 4),
                            "alg_flops_per_launch": isolated["flops"] / il, "alg_bytes_per_launch": isolated["bytes"] / il,
                            "achieved": round(iach, 3), "frac": round(iach / roof["peak"], 4),
                            "mfma_pipe": pipe(isolated)}
    if roof is not None and dom == "mp_resident":
        roof.update(resident_roof(batches, roof, isolated))
    if roof is not None and isolated_all is not None:
        roof.update(step_account(isolated_all, dom, len(subs), dt / args.steps * 1e3, pipe))
    if roof is not None:
        roof["contraction"] = contraction[{"seq_gru": "ordered_update_hU", "readout": "readout",
                                           "mp_resident": "mp_resident"}.get(dom, "sum_update")]
    line = {
        "metric": METRIC, "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if synthetic else "weak",
        "vs_baseline": None, "dtype": "fp32",
        "data": ("synthetic: %d-node graph, in-degree Poisson(10) capped at 30, 90%% of sources within +-4096 ids, "
                 "PCG64 seed 20261015, random-init weights" % args.nodes) if synthetic else
                ("synthetic: random %s-size topologies (networkx gnm, shortest-path routing, PCG64 seed "
                 "20261015+graph_id), migrate.py sample layout, random-init weights" % args.topology),
        "config": {"workload": workload, "model": args.model, "graphs_per_gpu": args.graphs,
                   "global_batch": args.graphs * (1 if synthetic else world), "hidden": plan.hidden[0], "iterations": plan.iterations,
                   "edges_per_step_per_gpu": edges, "gru_steps_per_forward": gru_steps,
                   "parallelism": ("edge-cut over %d ranks, RCCL halo all-to-all per iteration (rank 0 halo rows: %d)"
                                   % (world, halo_rows)) if synthetic else
                                  "graph-sharded (%d ranks), no collective in the forward" % world,
                   "batch_build_s": round(t_build, 3), "contraction": contraction, "streams": len(engines),
                   "samples_per_s": round(args.graphs * world * args.steps / dt, 1)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_cxx": cpu_cxx,
    }
    if edge_cut is not None:
        line[edge_cut_key(args.edge_cut_nodes)] = edge_cut
    if fresh_stats and fresh_stats["steps"]:
        n = fresh_stats["steps"]   # warm-up included
        timed = fresh_stats["waits"][-args.steps:]   # the timed steps only (the warm-up fills the pipeline)
        line["input_pipeline"] = {"workers": 0 if args.no_prefetch else args.input_workers,
                                  "ms_waiting_for_batch": round(1e3 * sum(timed) / max(len(timed), 1), 2),
                                  "ms_waiting_for_batch_incl_warmup": round(1e3 * fresh_stats["wait_s"] / n, 2),
                                  "ms_in_step": round(1e3 * fresh_stats["step_s"] / n, 2), "steps": n,
                                  "host_cpus_granted": int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None}
        sp = getattr(fresh_stats.get("trainer"), "step_prof", None)
        if sp and sp["steps"]:   # IGN_STEP_PROF=1: the step's host phases (ms per step)
            line["input_pipeline"]["step_phases_ms"] = {k: round(1e3 * v / sp["steps"], 2) for k, v in sp.items()
                                                        if k != "steps"}
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def step_account(iso, dom, parts, ms_step, pipe):
    """the step's kernels timed alone (sub-batch 0 on an idle chip, after the timed
    region) against the measured step: the readout's launch time and its 16-bit pipe fraction, and
    the sum of every sub-batch's isolated dominant + readout launches beside ms_per_step (the
    difference is what co-running the sub-batches hides, or loses)."""
    out = {}
    ro = iso.get("readout")
    per = {}
    for k in (dom, "readout"):
        v = iso.get(k)
        if v and v["launches"]:
            per[k] = v["ms"] / v["launches"]
    if ro and ro["launches"]:
        out["readout_isolated"] = {"avg_launch_ms": round(per["readout"], 4), "launches": ro["launches"],
                                   "mfma_pipe": pipe(ro),
                                   "what": "sub-batch 0's readout (fused Dense 256 -> 256 -> 1) alone on the chip"}
    if per:
        total = parts * sum(per.values())
        out["step_account"] = {"what": "every sub-batch's isolated launches summed, against ms_per_step",
                               "sub_batches": parts,
                               "per_sub_batch_ms": {k: round(v, 4) for k, v in per.items()},
                               "sum_isolated_ms": round(total, 4), "ms_per_step": round(ms_step, 4),
                               "co_run_gain_ms": round(total - ms_step, 4)}
    return out


def resident_roof(batches, roof, isolated):
    """The graph-resident forward's per-launch cost model (ign_batch_resident_info) and its issue
    roof: phase A's tile-steps x the cycles one tile-step's instructions hold a SIMD's vector issue
    (tools/isa_mix.py over the built kernel: VALU 2, packed f32 4, transcendental 8, an MFMA's hold 8
    cycles; MI355X_MICROARCH.md constants table), over the launch's SIMDs at the 2.4 GHz clock.  Phase
    B (the message sums, the GRU step of the union rows, the projection) is not in it: the roof is a
    floor for phase A's share of the launch (68 % of the cycles in round 4's stamps)."""
    infos = [b.resident_info() for b in batches]
    infos = [i for i in infos if i["active"]]
    if not infos:
        return {}
    n = len(infos)
    avg = {k: sum(i[k] for i in infos) / n for k in ("tile_steps", "union_tiles", "seg_rows", "messages",
                                                     "bytes_compulsory", "bytes_roundtrip", "bytes_stage", "lds_bytes")}
    out = {"resident": {"form": {0: "all states in LDS", 1: "path states in HBM/L2",
                                 2: "path states and sum CSR in HBM/L2"}[infos[0]["form"]],
                        "launches_per_step": n, "lds_bytes": int(avg["lds_bytes"]),
                        "workgroups_per_launch": infos[0].get("workgroups"),
                        "graphs_per_workgroup": infos[0].get("graphs_per_workgroup"),
                        "tile_steps_per_launch": avg["tile_steps"], "union_tiles_per_iteration": avg["union_tiles"],
                        "segmented_rows": avg["seg_rows"], "sum_messages_per_iteration": avg["messages"]},
           # alg bytes = B_stage over the launch's T x MPs (the line's alg_bytes_per_launch);
           # the compulsory bytes (inputs once, final states once) and the design's L2 round trips beside it
           "bytes_per_launch": {"b_stage": avg["bytes_stage"], "compulsory": avg["bytes_compulsory"],
                                "roundtrip_l2": avg["bytes_roundtrip"]}}
    path = os.path.join(REPO, "ignnition_amd", "isa_mix.json")
    if not os.path.exists(path):
        return out
    with open(path) as f:
        mix = json.load(f)["kernels"].get(RES_KERNEL[infos[0]["form"]])
    if not mix:
        return out
    wgs = max(i.get("workgroups") or 0 for i in infos) or max(b.num_graphs for b in batches)
    simds = 4 * min(wgs, N_CU)
    issue_ms = avg["tile_steps"] * mix["cycles_per_tile_step"] / (simds * CLOCK_GHZ * 1e9) * 1e3
    iso_ms = isolated["ms"] / isolated["launches"] if isolated and isolated["launches"] else None
    out["issue"] = {"what": "phase A's VALU/MFMA issue floor: tile_steps x cycles_per_tile_step / (SIMDs x clock)",
                    "cycles_per_tile_step": mix["cycles_per_tile_step"],
                    "tile_step_mix": {k: mix[k] for k in ("valu", "valu_pk", "trans", "mfma16", "lds", "vmem", "salu")},
                    "simds": simds, "clock_ghz": CLOCK_GHZ, "issue_floor_ms": round(issue_ms, 4),
                    "frac": round(issue_ms / roof["avg_launch_ms"], 4),
                    "frac_isolated": round(issue_ms / iso_ms, 4) if iso_ms else None}
    return out


def dry_run(args, dist, rank, world, mi, graphs, synthetic):
    """--dry-run: the rank plumbing of a real run without a GPU (the shard of each rank, the
    barrier + MAX-over-ranks time, the SUM of edges), so a CPU host can check that `--gpus N`
    yields one line from N ranks."""
    from ignnition_amd import workloads
    if synthetic:
        edges = workloads.edges_per_forward(mi, graphs) // world   # the rank's in-edge share
    else:
        edges = workloads.edges_per_forward(mi, graphs)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt, total = workloads.reduce_step_stats(dist, dt, edges)
    edge_cut = None
    if not (synthetic or args.train or args.no_edge_cut):
        # the edge-cut leg's host side: every rank's partition of the seeded graph and the setup
        # all-to-all of halo requests (gloo); the partitions' edges must add up to the graph's
        from ignnition_amd import partition
        emi, eplan, egraphs, part = edge_cut_parts(args, dist, rank, world)
        name = eplan.entities[0]
        halo = send = 0
        recv_c, send_c = [0] * world, [0] * world   # rows this rank receives from / sends to each rank
        if part is not None:
            partition.exchange_requests([part], partition.TorchComm(dist, None))
            halo, send = part.halos[name].n_halo, len(part.halos[name].send_rows)
            recv_c, send_c = list(part.halos[name].recv_counts), list(part.halos[name].send_counts)
            e_local = workloads.edges_per_forward(emi, [part.inputs])
        else:
            e_local = workloads.edges_per_forward(emi, egraphs)
        tot_e, tot_halo, tot_send = _reduce(dist, [e_local, halo, send], "sum")
        # per rank pair: recv[i][j] (rows rank i reads from j) must equal send[j][i] (rows j sends i)
        recv_m = [[0] * world for _ in range(world)]
        send_m = [[0] * world for _ in range(world)]
        recv_m[rank], send_m[rank] = recv_c, send_c
        flat = _reduce(dist, [v for row in recv_m for v in row] + [v for row in send_m for v in row], "sum")
        recv_m = [[int(flat[i * world + j]) for j in range(world)] for i in range(world)]
        send_m = [[int(flat[world * world + i * world + j]) for j in range(world)] for i in range(world)]
        whole = workloads.edges_per_forward(emi, egraphs)
        edge_cut = {"value": None, "unit": "edges/s", "n_ranks": world, "nodes": args.edge_cut_nodes,
                    "edges_per_step": int(tot_e), "edges_per_step_whole_graph": int(whole),
                    "edges_match_whole_graph": int(tot_e) == int(whole),
                    "halo_rows": {"total": int(tot_halo)}, "send_rows_total": int(tot_send),
                    "halo_recv_by_pair": recv_m, "halo_send_by_pair": send_m,
                    "halo_symmetric": all(recv_m[i][j] == send_m[j][i] for i in range(world) for j in range(world)),
                    "dry_run": True}
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
                          "scaling": "strong" if synthetic else "weak", "vs_baseline": None, "dtype": "fp32",
                          "data": "dry run (no GPU)",
                          "config": {"workload": "%s_%s_x%d" % (args.model, args.topology, args.graphs),
                                     "edges_per_step_total": total, "dry_run": True},
                          **({edge_cut_key(args.edge_cut_nodes): edge_cut} if edge_cut else {})}))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
