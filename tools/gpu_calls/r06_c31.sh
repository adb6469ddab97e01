# round 6 call 31: the resident forward's B2 by column half for workgroups of <= 8 union-row tiles
# (GEANT2, NSFNET, Q-size's small graphs; its own kernel instantiation): the resident parity tests,
# then GEANT2 / NSFNET / Q-size GEANT2 x512 with IGN_RES_B2_SPLIT 1 / 0 interleaved, and the headline
set -o pipefail
mkdir -p gpurun_out/c31
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "resident or graph_groups or int32" > gpurun_out/c31/pytest.log 2>&1 || { tail -30 gpurun_out/c31/pytest.log; exit 1; }
tail -1 gpurun_out/c31/pytest.log
for w in "geant2|--topology geant2" "nsfnet|--topology nsfnet" "qgeant2|--model qsize --topology geant2"; do
  n=${w%%|*}; a=${w#*|}
  for sp in 1 0 1 0; do
    IGN_RES_B2_SPLIT=$sp timeout -k 10 200 python3 bench.py $a --no-cpu --no-edge-cut > gpurun_out/c31/$n-$sp.json 2> gpurun_out/c31/$n-$sp.err || exit 1
    echo "$n split=$sp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c31/$n-$sp.json)"
  done
done
timeout -k 10 200 python3 bench.py --no-cpu --no-edge-cut > gpurun_out/c31/default.json 2> gpurun_out/c31/default.err || exit 1
echo "default $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c31/default.json)"
