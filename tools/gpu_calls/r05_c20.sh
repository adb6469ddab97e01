# store-wait fixes (unconditional ga / hs stores, global address space for the SAVE pointers): parity + train A/B
set -o pipefail
mkdir -p gpurun_out/c20
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_training.py \
  > gpurun_out/c20/pytest_training.log 2>&1 || exit 1
bash tools/ab_lib.sh "base fix" 2 --train --steps 10 --warmup 3 > gpurun_out/c20/ab.txt 2>&1 || exit 1
