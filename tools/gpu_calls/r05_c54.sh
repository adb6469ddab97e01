# csr_gather_add: the < 8 tail as one batch vs the serial tail: training A/B, then the training tests
set -o pipefail
mkdir -p gpurun_out/c54
tools/ab_lib.sh "gserial gbatch" 3 --train --steps 10 --warmup 3 > gpurun_out/c54/ab.txt 2>&1 || { cat gpurun_out/c54/ab.txt; exit 1; }
cat gpurun_out/c54/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c54/tests.txt 2>&1 || { tail -30 gpurun_out/c54/tests.txt; exit 1; }
tail -3 gpurun_out/c54/tests.txt
bash tools/gpu_calls/r05_c53.sh > gpurun_out/c54/trace.txt 2>&1 || exit 1; grep csr_gather gpurun_out/c54/trace.txt | tail -4
