# the fresh-batch training input pipeline: where the step's time goes, by builder count
set -o pipefail
mkdir -p gpurun_out/c15
for w in 8 16 4; do
  timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 12 --warmup 3 --input-workers $w --no-edge-cut > gpurun_out/c15/fresh_w$w.json 2> gpurun_out/c15/fresh_w$w.err || exit 1
done
timeout -k 10 300 python -u bench.py --train --steps 10 --warmup 2 --no-edge-cut > gpurun_out/c15/resident.json 2> gpurun_out/c15/resident.err || exit 1
