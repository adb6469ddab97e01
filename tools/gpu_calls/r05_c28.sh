# fresh-batch training: what batch close waits for (host block cache cap, glibc mmap threshold)
set -o pipefail
mkdir -p gpurun_out/c28
i=0
for cfg in "IGN_HOST_CACHE_GB=4" "IGN_HOST_CACHE_GB=32" "MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736" "IGN_HOST_CACHE_GB=32 MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736"; do
  i=$((i+1))
  env $cfg IGN_STEP_PROF=1 IGN_BUILD_PROF=1 timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 15 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c28/fresh_$i.json 2> gpurun_out/c28/fresh_$i.err || exit 1
done
