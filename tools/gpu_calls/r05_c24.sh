# builder contention: glibc mmap threshold (large temporaries from the heap instead of mmap/munmap per batch)
set -o pipefail
mkdir -p gpurun_out/c24
run() {  # tag, env...
  local tag=$1; shift
  env "$@" IGN_BUILD_PROF=1 REPS=3 timeout -k 10 300 python -u tools/host_pipeline_profile.py > gpurun_out/c24/host_$tag.txt 2>&1 || return 1
}
run base_t8 THREADS=8 &&
run mmap_t8 THREADS=8 MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 &&
run mmap_t1 THREADS=1 MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 &&
run mmap_t4 THREADS=4 MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 || exit 1
MALLOC_MMAP_THRESHOLD_=4294967296 MALLOC_TRIM_THRESHOLD_=68719476736 timeout -k 10 400 python -u bench.py --train --fresh-batches --steps 20 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c24/fresh_mmap.json 2> gpurun_out/c24/fresh_mmap.err || exit 1
