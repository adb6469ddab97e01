# round 4, call 34: kernel trace + PMC passes of Q-size x512 with the default (now four) sub-batch
# streams, so traffic.json's per-launch bytes match the bench line's launches
set -o pipefail
BENCH_ARGS="--model qsize --steps 3 --warmup 1 --no-cpu --no-edge-cut" TRACE_ARGS="--model qsize --no-edge-cut" \
  bash profiles/collect.sh r04_qsize_4streams
