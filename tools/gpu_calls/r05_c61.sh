# seq_gru_bwd: non-temporal loads of the saved state rows vs plain: training A/B
set -o pipefail
mkdir -p gpurun_out/c61
tools/ab_lib.sh "base hsnt" 3 --train --steps 10 --warmup 3 > gpurun_out/c61/ab.txt 2>&1 || { cat gpurun_out/c61/ab.txt; exit 1; }
cat gpurun_out/c61/ab.txt
