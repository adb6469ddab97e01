set -o pipefail
mkdir -p gpurun_out/ab22
timeout -k 10 400 python tools/ab_bitwise.py sb ss > gpurun_out/ab22/bitwise.log 2>&1 || exit 1
bash tools/ab_lib.sh "sb ss" 3 > gpurun_out/ab22/s2.log 2>&1 || exit 1
bash tools/ab_lib.sh "sb ss" 2 --streams 1 > gpurun_out/ab22/s1.log 2>&1 || exit 1
bash tools/ab_lib.sh "sb ss" 2 --model qsize > gpurun_out/ab22/q.log 2>&1
