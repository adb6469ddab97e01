# round 6 call 26: the bench sweep on the final tree (every workload's line) and smoke()
set -o pipefail
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_c26.log 2>&1 || { tail -20 gpurun_out/smoke_c26.log; exit 1; }
tail -2 gpurun_out/smoke_c26.log
rm -rf gpurun_out/sweep
timeout -k 10 1000 bash tools/bench_sweep.sh || exit 1
for n in default synthetic qsize geant2 train train_fresh; do
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sweep/$n.json | head -1)"
done
