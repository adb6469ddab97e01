# round 4, call 30: the global-path resident form with its step codes in LDS (default) against
# read from global memory (-DIGN_RES_PG_GLOBAL_CODES): parity, then the headline, interleaved
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident" > gpurun_out/c30_tests.log 2>&1 || { tail -30 gpurun_out/c30_tests.log; exit 1; }
tail -1 gpurun_out/c30_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep smoke
bash tools/ab_lib.sh "lcodes gcodes" 3
