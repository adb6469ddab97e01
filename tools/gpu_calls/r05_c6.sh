# same-box A/B of the round-4 and round-5 libraries (headline, GEANT2), then one-stream isolated kernel times
set -o pipefail
bash tools/ab_lib.sh "r4 r5" 3 > gpurun_out/ab_r4r5.txt 2>&1 || exit 1
bash tools/ab_lib.sh "r4 r5" 2 --topology geant2 >> gpurun_out/ab_r4r5.txt 2>&1 || exit 1
mkdir -p gpurun_out/c6
timeout -k 10 300 python -u bench.py --no-cpu --no-edge-cut --streams 1 > gpurun_out/c6/s1.json 2> gpurun_out/c6/s1.err || exit 1
