# round 6 call 13: the native reader's recycled gather buffers: host stages with 1 and 8 builder
# threads, then fresh-batch training (8 workers) with the pool (default) and without (IGN_GATHER_POOL=0)
set -o pipefail
mkdir -p gpurun_out/c13
REPS=4 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c13/host1.txt 2>&1 || exit 1
tail -1 gpurun_out/c13/host1.txt
REPS=4 THREADS=8 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c13/host8.txt 2>&1 || exit 1
tail -1 gpurun_out/c13/host8.txt
for pool in 16 0; do
  IGN_GATHER_POOL=$pool IGN_STEP_PROF=1 timeout -k 10 400 python3 bench.py --train --fresh-batches > gpurun_out/c13/fresh_pool$pool.json 2> gpurun_out/c13/fresh_pool$pool.err || exit 1
  echo "pool $pool $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c13/fresh_pool$pool.json) $(grep -o '"input_pipeline": {[^}]*' gpurun_out/c13/fresh_pool$pool.json)"
done
IGN_STEP_PROF=1 timeout -k 10 400 python3 bench.py --train --fresh-batches --steps 60 > gpurun_out/c13/fresh_60.json 2> gpurun_out/c13/fresh_60.err || exit 1
echo "60 steps $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c13/fresh_60.json)"
timeout -k 10 300 python3 bench.py --train > gpurun_out/c13/train.json 2> gpurun_out/c13/train.err || exit 1
echo "train $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c13/train.json)"
