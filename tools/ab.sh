#!/bin/bash
# A/B of engine variants on the GPU box.  Parity suite first (default and candidate env), then
# the bench once per CONFIG ("name:ENV=VAL,ENV=VAL"); stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_ab.log; exit 1; }
tail -1 gpurun_out/pt_ab.log
if [ -n "$PT_ENV" ]; then
  env $(echo $PT_ENV | tr ',' ' ') timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ab2.log 2>&1 || { echo "pytest ($PT_ENV) failed"; tail -30 gpurun_out/pt_ab2.log; exit 1; }
  tail -1 gpurun_out/pt_ab2.log
fi
for cfg in ${CONFIGS:-"base:IGN_SEQ_VARIANT=2"}; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > gpurun_out/ab_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/ab_$name.log; exit 1; }
  python tools/show_bench.py gpurun_out/ab_$name.log
done
