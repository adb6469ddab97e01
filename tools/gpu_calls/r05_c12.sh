# is the readout bound by streaming W2 through LDS?  one stream (the readout alone after the MP loop),
# default vs every chunk reusing chunk 0 (no DMA; timing only)
set -o pipefail
bash tools/ab_lib.sh "base nodma" 2 --streams 1 > gpurun_out/c12_ab.txt 2>&1 || exit 1
