# round 6 call 7: new parity cases (IGN_RES_GROUP graph groups, Q-size under IGN_SUM_WINDOW=0 and the
# IEEE yardstick), then GEANT2 / NSFNET x512 with K graphs per resident workgroup x sub-batch streams
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c07
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "graph_groups or edge_cases or resident_forward_is or segmented_sum_rule" > gpurun_out/c07/pytest.log 2>&1 || { tail -40 gpurun_out/c07/pytest.log; exit 1; }
tail -1 gpurun_out/c07/pytest.log
grep -h "IEEE float32 yardstick" gpurun_out/c07/pytest.log | head -5
for topo in geant2 nsfnet; do
  for k in 1 2 3; do
    for s in 1 2 4; do
      IGN_RES_GROUP=$k timeout -k 10 120 python3 bench.py --no-cpu --no-edge-cut --topology $topo --streams $s --steps 20 > gpurun_out/c07/${topo}_k${k}_s${s}.json 2>&1 || exit 1
      echo "$topo K=$k streams=$s $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c07/${topo}_k${k}_s${s}.json)"
    done
  done
done
