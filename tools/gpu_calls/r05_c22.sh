# resident tables built by the batch builder: parity, host-stage profile, fresh-batch training
set -o pipefail
mkdir -p gpurun_out/c22
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_parity.py \
  > gpurun_out/c22/pytest.log 2>&1 || exit 1
for th in 1 8; do
  IGN_BUILD_PROF=1 THREADS=$th REPS=3 timeout -k 10 300 python -u tools/host_pipeline_profile.py \
    > gpurun_out/c22/host_t${th}.txt 2>&1 || exit 1
done
timeout -k 10 400 python -u bench.py --train --fresh-batches --steps 20 --warmup 3 --no-cpu --no-edge-cut \
  > gpurun_out/c22/fresh.json 2> gpurun_out/c22/fresh.err || exit 1
timeout -k 10 400 python -u bench.py --train --steps 20 --warmup 3 --no-cpu --no-edge-cut \
  > gpurun_out/c22/train.json 2> gpurun_out/c22/train.err || exit 1
