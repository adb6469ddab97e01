#!/bin/bash
# N=2 rehearsal on one GPU: both ranks on device 0, gloo with host-staged halo rows (the driver's
# 8-GPU node runs the RCCL leg).  Synthetic edge-cut graph, then the driver's default line: the
# graph-sharded RouteNet batch on the resident forward with the 1M-node edge-cut leg (edge_cut_1m).
mkdir -p gpurun_out
export IGN_DIST_BACKEND=gloo IGN_BENCH_DEVICE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --model synthetic --gpus 2 --steps 3 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/n2_syn.log 2>&1 || { echo "n2 synthetic failed"; tail -30 gpurun_out/n2_syn.log; exit 1; }
grep '"metric"' gpurun_out/n2_syn.log | tail -1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --edge-cut-steps 3 > gpurun_out/n2_rn.log 2>&1 || { echo "n2 routenet failed"; tail -30 gpurun_out/n2_rn.log; exit 1; }
grep '"metric"' gpurun_out/n2_rn.log | tail -1
