# gates staged across the lane's elements (more independent transcendentals in flight): stamps + A/B
set -o pipefail
mkdir -p gpurun_out/c11
MODEL=routenet TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_stagedst.so \
  timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/c11/stagedst.json 2> gpurun_out/c11/stagedst.err || exit 1
bash tools/ab_lib.sh "base staged" 3 > gpurun_out/c11/ab.txt 2>&1 || exit 1
