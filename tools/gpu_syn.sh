#!/bin/bash
# GPU tests, then the synthetic 1M/10M profile (trace + PMC passes) and its bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
BENCH_ARGS="--model synthetic --steps 3 --warmup 1 --no-cpu" TRACE_ARGS="--model synthetic" bash profiles/collect.sh syn || exit 1
timeout -k 10 300 python bench.py --model synthetic > gpurun_out/bench_synthetic.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_synthetic.log; exit 1; }
tail -1 gpurun_out/bench_synthetic.log
