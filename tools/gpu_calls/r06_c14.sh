# round 6 call 14: fresh-batch training, A/B interleaved on one box (40 timed steps each): the
# native reader's gather pool on (16) / off (0) at 8 workers, then 10 and 12 workers with the pool
set -o pipefail
mkdir -p gpurun_out/c14
run() {  # name, env...
  local n=$1; shift
  env "$@" IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py --train --fresh-batches --steps 40 --input-workers ${W:-8} > gpurun_out/c14/$n.json 2> gpurun_out/c14/$n.err || return 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c14/$n.json) $(grep -o '"close": [0-9.]*' gpurun_out/c14/$n.json)"
}
run a1 IGN_GATHER_POOL=16 && run b1 IGN_GATHER_POOL=0 && run a2 IGN_GATHER_POOL=16 && run b2 IGN_GATHER_POOL=0 && \
W=10 run w10 IGN_GATHER_POOL=16 && W=12 run w12 IGN_GATHER_POOL=16 && \
timeout -k 10 300 python3 bench.py --train --steps 40 > gpurun_out/c14/train.json 2> gpurun_out/c14/train.err && \
echo "train $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c14/train.json)"
