# dW2 contraction with XCD-paired column groups: parity (bitwise the same partials) and the --train A/B
set -o pipefail
mkdir -p gpurun_out/c34
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_training.py > gpurun_out/c34/pytest.log 2>&1 || exit 1
bash tools/ab_lib.sh "gemv xcd" 2 --train --steps 10 --warmup 3 > gpurun_out/c34/ab.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c34/trace -o t --output-format csv -- python3 bench.py --train --steps 4 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/c34/trace.log 2>&1 || exit 1
