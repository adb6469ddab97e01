set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
timeout -k 10 300 python bench.py --model synthetic > gpurun_out/bench_synthetic.log 2>&1
bash profiles/collect.sh r01d
TRACE_ARGS="--model synthetic" BENCH_ARGS="--model synthetic --steps 2 --warmup 1 --no-cpu" bash profiles/collect.sh r01d_syn
