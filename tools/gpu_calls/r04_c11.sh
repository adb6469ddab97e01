# round 4, call 11: resident-forward phase stamps (diagnostic build -DIGN_RES_STAMP), GEANT2 x256 and NSFNET x256
set -o pipefail
O=gpurun_out/c11
mkdir -p $O
for topo in geant2 nsfnet; do
  TOPO=$topo IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > $O/$topo.json 2> $O/$topo.err || { tail -20 $O/$topo.err; exit 1; }
  cat $O/$topo.json
done
