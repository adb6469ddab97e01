set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python tools/ab_bitwise.py base epi > gpurun_out/ab/bitwise_epi.log 2>&1 || exit 1
bash tools/ab_lib.sh "base epi" 3 --streams 1 > gpurun_out/ab/epi_s1.log 2>&1 || exit 1
bash tools/ab_lib.sh "base epi" 2 > gpurun_out/ab/epi_s2.log 2>&1
