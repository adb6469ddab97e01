# csr_gather_add: non-temporal row loads for the wide (ga) gather vs plain: training A/B
set -o pipefail
mkdir -p gpurun_out/c59
tools/ab_lib.sh "base gnt" 3 --train --steps 10 --warmup 3 > gpurun_out/c59/ab.txt 2>&1 || { cat gpurun_out/c59/ab.txt; exit 1; }
cat gpurun_out/c59/ab.txt
