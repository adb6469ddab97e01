set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t27.log 2>&1
