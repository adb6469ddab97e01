# phase-A ablations under stamps (synth50 RouteNet x256): full, no gate math, no MFMAs
set -o pipefail
mkdir -p gpurun_out/c8
for v in rstamp ablgate ablmfma; do
  MODEL=routenet TOPO=synth50 GRAPHS=256 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$v.so \
    timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/c8/$v.json 2> gpurun_out/c8/$v.err || exit 1
done
