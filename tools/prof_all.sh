#!/bin/bash
# Round-end measurement set on the GPU box: bench lines for every config + rocprofv3 trace and
# PMC passes for the headline (RouteNet 512 x synth50) and the 1M-node synthetic graph.
# Usage: bash tools/prof_all.sh <tag>   (outputs under gpurun_out/)
set -e
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
timeout -k 10 300 python bench.py --model synthetic > gpurun_out/bench_synthetic.log 2>&1
timeout -k 10 300 python bench.py --model qsize --no-cpu > gpurun_out/bench_qsize.log 2>&1
timeout -k 10 300 python bench.py --topology geant2 --no-cpu > gpurun_out/bench_geant2.log 2>&1
bash profiles/collect.sh $TAG
TRACE_ARGS="--model synthetic" BENCH_ARGS="--model synthetic --steps 2 --warmup 1 --no-cpu" bash profiles/collect.sh ${TAG}_syn
