# deferred builder uploads: parity, host-stage profile (1 / 8 builders, defer on / off), fresh-batch training
set -o pipefail
mkdir -p gpurun_out/c21
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py tests/test_gpu_parity.py \
  > gpurun_out/c21/pytest.log 2>&1 || exit 1
for d in 1 0; do
  for th in 1 8; do
    IGN_UPLOAD_DEFER=$d IGN_BUILD_PROF=1 THREADS=$th REPS=3 timeout -k 10 300 python -u tools/host_pipeline_profile.py \
      > gpurun_out/c21/host_d${d}_t${th}.txt 2>&1 || exit 1
  done
done
for d in 1 0; do
  IGN_UPLOAD_DEFER=$d timeout -k 10 400 python -u bench.py --train --fresh-batches --steps 20 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c21/fresh_d$d.json 2> gpurun_out/c21/fresh_d$d.err || exit 1
done
