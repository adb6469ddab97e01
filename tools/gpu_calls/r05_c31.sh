# fresh-batch training with the new pool cap default and trims outside the lock; training and parity tests
set -o pipefail
mkdir -p gpurun_out/c31
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_parity.py \
  > gpurun_out/c31/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  IGN_STEP_PROF=1 timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 20 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c31/fresh_$rep.json 2> gpurun_out/c31/fresh_$rep.err || exit 1
done
timeout -k 10 300 python -u bench.py --train --steps 20 --warmup 3 --no-cpu --no-edge-cut > gpurun_out/c31/train.json 2> gpurun_out/c31/train.err || exit 1
