set -o pipefail
mkdir -p gpurun_out/ab14
bash tools/ab_lib.sh "dma nodma" 3 --streams 1 > gpurun_out/ab14/s1.log 2>&1
