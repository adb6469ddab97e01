# resident training forward also saves the ordered MP's tables (backward skips build_table): tests + A/B
set -o pipefail
mkdir -p gpurun_out/c49
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c49/pytest.log 2>&1 || exit 1
IGN_POOL_POISON=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py -k "resident" > gpurun_out/c49/pytest_poison.log 2>&1 || exit 1
bash tools/ab_env.sh IGN_RESIDENT_SAVE_TABLE "1 0" 2 --train --steps 10 --warmup 3 > gpurun_out/c49/ab.txt 2>&1 || exit 1
