# ordered-backward ablations on the training step: no dU contraction / no ga stores (timing only)
set -o pipefail
bash tools/ab_lib.sh "base nodu noga" 2 --train --steps 10 --warmup 3 > gpurun_out/c19_ab.txt 2>&1 || exit 1
