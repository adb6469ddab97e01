# sum backward with dW / dU formed in the kernel (IGN_SUM_BWD_FUSE): training tests and the A/B
set -o pipefail
mkdir -p gpurun_out/c47
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c47/pytest.log 2>&1 || exit 1
bash tools/ab_env.sh IGN_SUM_BWD_FUSE "1 0" 2 --train --steps 10 --warmup 3 > gpurun_out/c47/ab.txt 2>&1 || exit 1
