set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/gpu_tests.log 2>&1 || { tail -30 gpurun_out/full/gpu_tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/full/bench.log 2>&1
