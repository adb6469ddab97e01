# per-instance weight gradients reduced once per backward (IGN_DEFER_WGRAD): training parity and the A/B
set -o pipefail
mkdir -p gpurun_out/c39
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c39/pytest.log 2>&1 || exit 1
bash tools/ab_env.sh IGN_DEFER_WGRAD "1 0" 2 --train --steps 10 --warmup 3 > gpurun_out/c39/ab.txt 2>&1 || exit 1
