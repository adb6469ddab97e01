# the fused ordered backward's partials also reduced once per backward: training tests and the A/B (IGN_DEFER_WGRAD)
set -o pipefail
mkdir -p gpurun_out/c46
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c46/pytest.log 2>&1 || exit 1
bash tools/ab_env.sh IGN_DEFER_WGRAD "1 0" 2 --train --steps 10 --warmup 3 > gpurun_out/c46/ab.txt 2>&1 || exit 1
