# round 4, call 35: the message-sum items dealt in a snake (odd rounds backwards) against the plain
# strided order (lib_fused23 from call 33): resident parity, then the headline, interleaved
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident" > gpurun_out/c35_tests.log 2>&1 || { tail -30 gpurun_out/c35_tests.log; exit 1; }
tail -1 gpurun_out/c35_tests.log
bash tools/ab_lib.sh "snake fused23" 3
