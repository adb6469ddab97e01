set -o pipefail
mkdir -p gpurun_out/ab11
bash tools/ab_lib.sh "sl0 sl1 sl2 sl4" 2 --streams 1 > gpurun_out/ab11/s1.log 2>&1 || exit 1
bash tools/ab_lib.sh "sl0 sl1 sl2 sl4" 2 > gpurun_out/ab11/s2.log 2>&1
