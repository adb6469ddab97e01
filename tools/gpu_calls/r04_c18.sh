# round 4, call 18: the output-layer gradient rows formed by dense_h16_t and written in place over
# a2 (no row_outer_t, no on-the-fly B in tsgemm): training tests, then IGN_FUSE_OUTER_BWD 1 / 0;
# then the library built with -fno-slp-vectorize against the default (headline, GEANT2)
set -o pipefail
O=gpurun_out/c18
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_training.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_env.sh IGN_FUSE_OUTER_BWD "1 0" 2 --train --steps 10 --warmup 3 &&
  bash tools/ab_lib.sh "base noslp" 3 && bash tools/ab_lib.sh "base noslp" 2 --topology geant2
