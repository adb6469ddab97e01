# round 4, call 13: resident-forward phase stamps after the phase-B rewrite (GEANT2 / NSFNET x256)
set -o pipefail
O=gpurun_out/c13
mkdir -p $O
for topo in geant2 nsfnet; do
  TOPO=$topo IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > $O/stamps-$topo.json 2> $O/stamps-$topo.err || { tail -20 $O/stamps-$topo.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/stamps-$topo.json')); print('$topo', d['cycles_per_graph_mean'], d['share_all_waves']); print([round(x) for x in d['A_work_per_wave']]); print([round(x) for x in d['B_work_per_wave']]); print(d['per_wave_mean_cycles'])"
done
