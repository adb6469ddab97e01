# fresh-batch training: where the main thread's step time goes (IGN_STEP_PROF), builders 8 vs 6, and inline
set -o pipefail
mkdir -p gpurun_out/c27
for args in "--input-workers 8" "--input-workers 6" "--no-prefetch"; do
  tag=$(echo $args | tr -dc 'a-z0-9')
  IGN_STEP_PROF=1 timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 15 --warmup 3 --no-cpu --no-edge-cut $args \
    > gpurun_out/c27/fresh_$tag.json 2> gpurun_out/c27/fresh_$tag.err || exit 1
done
timeout -k 10 300 python -u bench.py --train --steps 15 --warmup 3 --no-cpu --no-edge-cut > gpurun_out/c27/train.json 2> gpurun_out/c27/train.err || exit 1
