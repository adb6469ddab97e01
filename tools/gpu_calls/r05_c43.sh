# resident SAVE forward without the first hs row (the backward reads step 0's state from the version):
# new GPU tests, training parity under pool poison, and the --train A/B
set -o pipefail
mkdir -p gpurun_out/c43
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c43/pytest.log 2>&1 || exit 1
IGN_POOL_POISON=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py -k "resident or autograd or deferred" > gpurun_out/c43/pytest_poison.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "switches" > gpurun_out/c43/pytest_switches.log 2>&1 || exit 1
bash tools/ab_lib.sh "prev cur2" 2 --train --steps 10 --warmup 3 > gpurun_out/c43/ab.txt 2>&1 || exit 1
