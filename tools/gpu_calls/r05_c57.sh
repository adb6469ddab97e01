# csr_gather_add: 8 columns per thread for wide rows vs 4: training A/B, tests, trace
set -o pipefail
mkdir -p gpurun_out/c57
tools/ab_lib.sh "v1 v2" 3 --train --steps 10 --warmup 3 > gpurun_out/c57/ab.txt 2>&1 || { cat gpurun_out/c57/ab.txt; exit 1; }
cat gpurun_out/c57/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c57/tests.txt 2>&1 || { tail -30 gpurun_out/c57/tests.txt; exit 1; }
tail -3 gpurun_out/c57/tests.txt
bash tools/gpu_calls/r05_c53.sh > gpurun_out/c57/trace.txt 2>&1 || exit 1; grep csr_gather gpurun_out/c57/trace.txt | tail -4
