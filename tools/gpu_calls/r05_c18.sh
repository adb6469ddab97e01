# training step with the resident SAVE forward: kernel trace + PMC passes (per-kernel breakdown, traffic)
set -o pipefail
TRACE_ARGS="--train --steps 5 --warmup 2 --no-cpu --no-edge-cut" BENCH_ARGS="--train --steps 3 --warmup 1 --no-cpu --no-edge-cut" \
  bash profiles/collect.sh r05_train || exit 1
