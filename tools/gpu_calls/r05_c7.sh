# phase stamps (synth50 RouteNet x256, Q-size synth50 x256) and the A/B of static priority / no SLP
set -o pipefail
mkdir -p gpurun_out/c7
for m in routenet qsize; do
  MODEL=$m TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so \
    timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/c7/stamps_$m.json 2> gpurun_out/c7/stamps_$m.err || exit 1
done
bash tools/ab_lib.sh "base prio noslp" 3 > gpurun_out/c7/ab.txt 2>&1 || exit 1
