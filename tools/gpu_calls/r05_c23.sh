# builder contention: host blocks (cache cap) x resident tables in the builder; fresh-batch training
set -o pipefail
mkdir -p gpurun_out/c23
run() {  # tag, env...
  local tag=$1; shift
  env "$@" IGN_BUILD_PROF=1 REPS=3 timeout -k 10 300 python -u tools/host_pipeline_profile.py > gpurun_out/c23/host_$tag.txt 2>&1 || return 1
}
run e1c4_t1 THREADS=1 IGN_RESIDENT_EAGER=1 IGN_HOST_CACHE_GB=4 &&
run e1c4_t8 THREADS=8 IGN_RESIDENT_EAGER=1 IGN_HOST_CACHE_GB=4 &&
run e1c32_t8 THREADS=8 IGN_RESIDENT_EAGER=1 IGN_HOST_CACHE_GB=32 &&
run e0c4_t8 THREADS=8 IGN_RESIDENT_EAGER=0 IGN_HOST_CACHE_GB=4 || exit 1
for cfg in "IGN_RESIDENT_EAGER=0 IGN_HOST_CACHE_GB=4" "IGN_RESIDENT_EAGER=1 IGN_HOST_CACHE_GB=32"; do
  tag=$(echo $cfg | tr -dc '0-9')
  env $cfg timeout -k 10 400 python -u bench.py --train --fresh-batches --steps 20 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c23/fresh_$tag.json 2> gpurun_out/c23/fresh_$tag.err || exit 1
done
