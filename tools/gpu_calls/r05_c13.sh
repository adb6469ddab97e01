# transposed ga: bitwise test, then the training step A/B (IGN_BWD_TSLOT 1 / 0)
set -o pipefail
mkdir -p gpurun_out/c13
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -v --timeout 200 --timeout-method thread -k "transposed or consumes or gradients_match" > gpurun_out/c13/test.log 2>&1 || { echo tests failed; exit 1; }
bash tools/ab_env.sh IGN_BWD_TSLOT "1 0" 2 --train --steps 10 > gpurun_out/c13/ab.txt 2>&1 || exit 1
