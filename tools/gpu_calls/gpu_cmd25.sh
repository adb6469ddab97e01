set -o pipefail
mkdir -p gpurun_out/ab25
timeout -k 10 400 python tools/ab_bitwise.py pers nopers > gpurun_out/ab25/bitwise.log 2>&1 || exit 1
bash tools/ab_lib.sh "pers nopers" 3 > gpurun_out/ab25/s2.log 2>&1 || exit 1
bash tools/ab_lib.sh "pers nopers" 2 --streams 1 > gpurun_out/ab25/s1.log 2>&1
