# csr_gather_add: two interleaved elements per thread for <= 32 columns vs one: training A/B, tests, trace
set -o pipefail
mkdir -p gpurun_out/c55
tools/ab_lib.sh "r1 r2" 3 --train --steps 10 --warmup 3 > gpurun_out/c55/ab.txt 2>&1 || { cat gpurun_out/c55/ab.txt; exit 1; }
cat gpurun_out/c55/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c55/tests.txt 2>&1 || { tail -30 gpurun_out/c55/tests.txt; exit 1; }
tail -3 gpurun_out/c55/tests.txt
bash tools/gpu_calls/r05_c53.sh > gpurun_out/c55/trace.txt 2>&1 || exit 1; grep csr_gather gpurun_out/c55/trace.txt | tail -4
