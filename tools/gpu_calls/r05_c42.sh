# new round-5 GPU tests: builder switches, deferred weight-gradient reduction
set -o pipefail
mkdir -p gpurun_out/c42
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_training.py \
  -k "switches or deferred or resident_training" > gpurun_out/c42/pytest.log 2>&1 || exit 1
