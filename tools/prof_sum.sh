set -e
for v in 3 4; do
IGN_SUM_VARIANT=$v BENCH_ARGS="--model synthetic --steps 2 --warmup 1 --no-cpu" bash profiles/collect.sh syn_v$v
done
