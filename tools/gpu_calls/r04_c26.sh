# round 4, call 26: phase stamps of the resident forward's global-path form (synth50 x256) and of
# the all-LDS form (GEANT2 x256)
set -o pipefail
for topo in synth50 geant2; do
  TOPO=$topo IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > gpurun_out/stamps-$topo.json 2> gpurun_out/stamps-$topo.err || { tail -20 gpurun_out/stamps-$topo.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/stamps-$topo.json')); print('$topo', d['cycles_per_graph_mean'], {k: round(v) for k, v in d['per_wave_mean_cycles'].items()}); print([round(x) for x in d['A_work_per_wave']]); print([round(x) for x in d['B_work_per_wave']]); print(d['A_tiles_per_wave'][:4], d['B_tiles_per_wave'][:4])"
done
