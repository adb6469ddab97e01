# resident SAVE without the final hs row: parity (also under pool poison) and the --train A/B against the previous build
set -o pipefail
mkdir -p gpurun_out/c32
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c32/pytest.log 2>&1 || exit 1
IGN_POOL_POISON=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py -k "resident or autograd" > gpurun_out/c32/pytest_poison.log 2>&1 || exit 1
bash tools/ab_lib.sh "fix cur" 2 --train --steps 10 --warmup 3 > gpurun_out/c32/ab.txt 2>&1 || exit 1
