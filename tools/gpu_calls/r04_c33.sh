# round 4, call 33: the resident forward's GRU step and projection fused per link tile (one wave
# per tile, where the link tiles fit one round) against the separate B2 / B3 passes
# (-DIGN_RES_B23_SPLIT): parity, then the headline and GEANT2, interleaved
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident" > gpurun_out/c33_tests.log 2>&1 || { tail -30 gpurun_out/c33_tests.log; exit 1; }
tail -1 gpurun_out/c33_tests.log
bash tools/ab_lib.sh "fused23 split23" 3 && bash tools/ab_lib.sh "fused23 split23" 2 --topology geant2
