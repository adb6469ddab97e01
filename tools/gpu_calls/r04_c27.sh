# round 4, call 27: global-path resident form with the sum CSR in LDS and sixteen path rows in
# flight in the message sums: parity, headline A/B against the batched launches, stamps
set -o pipefail
O=gpurun_out/c27
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/ab_env.sh IGN_RESIDENT_PG "1 0" 2 &&
TOPO=synth50 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rstamp.so timeout -k 10 200 python -u tools/probes/res_stamps.py > $O/stamps-synth50.json 2> $O/stamps.err &&
python3 -c "import json; d=json.load(open('$O/stamps-synth50.json')); print('synth50', d['cycles_per_graph_mean'], {k: round(v) for k, v in d['per_wave_mean_cycles'].items()}); print('B1', round(d['B1_cycles_per_wave_mean']), 'B1+B2', round(d['B1_B2_cycles_per_wave_mean']))"
