# readout first-layer input gradient on dense_bf (K = 256 -> M = 32) vs row_gemm_t: training A/B,
# then the training tests on the new default
set -o pipefail
mkdir -p gpurun_out/c52
tools/ab_lib.sh "m128 m32" 3 --train --steps 10 --warmup 3 > gpurun_out/c52/ab.txt 2>&1 || { cat gpurun_out/c52/ab.txt; exit 1; }
cat gpurun_out/c52/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c52/tests.txt 2>&1 || { tail -30 gpurun_out/c52/tests.txt; exit 1; }
tail -3 gpurun_out/c52/tests.txt
