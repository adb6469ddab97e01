# training-step kernel traces with the transposed ga on and off
set -o pipefail
export TMPDIR=/tmp
for v in 1 0; do
  rm -rf gpurun_out/prof_train_t$v && mkdir -p gpurun_out/prof_train_t$v
  IGN_BWD_TSLOT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_t$v -o train --output-format csv -- \
    python3 bench.py --train --steps 2 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/prof_train_t$v.log 2>&1 || exit 1
done
