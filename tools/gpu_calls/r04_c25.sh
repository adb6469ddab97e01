# round 4, call 25: the resident forward with the path states in global memory (synth50-size graphs):
# parity tests, then the headline and GEANT2 with IGN_RESIDENT_PG=1 / 0
set -o pipefail
O=gpurun_out/c25
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_env.sh IGN_RESIDENT_PG "1 0" 2
