# fresh-batch training: the device block cache cap (a released batch's blocks trimmed with hipFree under the pool lock)
set -o pipefail
mkdir -p gpurun_out/c30
for gb in 16 64 128; do
  IGN_POOL_CACHE_GB=$gb IGN_STEP_PROF=1 IGN_BUILD_PROF=1 timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 15 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c30/fresh_$gb.json 2> gpurun_out/c30/fresh_$gb.err || exit 1
done
