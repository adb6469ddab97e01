# round 6 call 30: the resident forward's phase stamps on the final tree (diagnostic library built
# with -DIGN_RES_STAMP): RouteNet synth50 x256 and GEANT2 x256, one stream
set -o pipefail
mkdir -p gpurun_out/c30
for spec in "routenet_synth50_x256|TOPO=synth50" "routenet_geant2_x256|TOPO=geant2"; do
  n=${spec%%|*}; e=${spec#*|}
  env $e IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 300 python3 tools/probes/res_stamps.py > gpurun_out/c30/$n.json 2> gpurun_out/c30/$n.err || { tail -5 gpurun_out/c30/$n.err; exit 1; }
  tail -c 600 gpurun_out/c30/$n.json; echo
done
