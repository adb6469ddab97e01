set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/final/tests.log 2>&1 || { tail -30 gpurun_out/final/tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/final/train.json 2>&1 || exit 1
