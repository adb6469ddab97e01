set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 400 python tools/ab_bitwise.py w4r2 w8r1 w4r1 > gpurun_out/ab/bitwise_rt.log 2>&1 || exit 1
bash tools/ab_lib.sh "w4r2 w8r1 w4r1" 2 --streams 1 > gpurun_out/ab/rt_s1.log 2>&1 || exit 1
bash tools/ab_lib.sh "w4r2 w8r1 w4r1" 2 > gpurun_out/ab/rt_s2.log 2>&1
