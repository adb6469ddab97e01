# training readout backward (dense_bf, K = 256, split-fp16): one 16-row tile per wave (110 VGPRs, 2 blocks per CU) vs two
set -o pipefail
mkdir -p gpurun_out/c37
bash tools/ab_lib.sh "base2 rt1" 2 --train --steps 10 --warmup 3 > gpurun_out/c37/ab.txt 2>&1 || exit 1
