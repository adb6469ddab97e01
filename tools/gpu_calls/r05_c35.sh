# full GPU suite on the round-5 tree (deferred builder copies, eager resident tables, pool cap, training forward resident)
set -o pipefail
mkdir -p gpurun_out/c35
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c35/pytest_gpu.log 2>&1 || exit 1
bash tools/ab_lib.sh "base2 g16" 2 --train --steps 10 --warmup 3 > gpurun_out/c35/ab_g16.txt 2>&1 || exit 1   # (g16: sixteen ga rows in flight, slower; reverted)
