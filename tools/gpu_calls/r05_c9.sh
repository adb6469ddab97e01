# 8-wave resident workgroups (2 waves per SIMD, 161 VGPRs) against the 16-wave default: stamps + bench A/B
set -o pipefail
mkdir -p gpurun_out/c9
RES_WAVES=8 MODEL=routenet TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_w8stamp.so \
  timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/c9/w8stamp.json 2> gpurun_out/c9/w8stamp.err || exit 1
bash tools/ab_lib.sh "base w8" 2 > gpurun_out/c9/ab.txt 2>&1 || exit 1
