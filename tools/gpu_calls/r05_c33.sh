# N = 1 weight-gradient kernel (tsgemv): training parity and the --train A/B
set -o pipefail
mkdir -p gpurun_out/c33
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c33/pytest.log 2>&1 || exit 1
bash tools/ab_lib.sh "cur gemv" 2 --train --steps 10 --warmup 3 > gpurun_out/c33/ab.txt 2>&1 || exit 1
