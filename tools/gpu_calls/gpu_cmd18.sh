set -o pipefail
mkdir -p gpurun_out/ab18
timeout -k 10 400 python tools/ab_bitwise.py w4 w5 w6 w8 > gpurun_out/ab18/bitwise.log 2>&1 || exit 1
bash tools/ab_lib.sh "w4 w5 w6 w8" 2 --streams 1 > gpurun_out/ab18/s1.log 2>&1 || exit 1
bash tools/ab_lib.sh "w4 w5 w6 w8" 2 > gpurun_out/ab18/s2.log 2>&1
