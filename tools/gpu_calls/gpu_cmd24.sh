set -o pipefail
mkdir -p gpurun_out/ab24
timeout -k 10 400 python tools/ab_bitwise.py p0 p1 > gpurun_out/ab24/bitwise.log 2>&1 || exit 1
bash tools/ab_lib.sh "p0 p1" 3 > gpurun_out/ab24/s2.log 2>&1 || exit 1
bash tools/ab_lib.sh "p0 p1" 2 --streams 1 > gpurun_out/ab24/s1.log 2>&1
