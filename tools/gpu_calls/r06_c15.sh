# round 6 call 15: the whole GPU suite and smoke on the current tree (gather pool, two-pass OOM trim
# outside the pool lock, device cache cap a quarter of free memory), then fresh-batch training at 8
# and 12 workers with IGN_BUILD_PROF=1 (out-of-memory trims are reported)
set -o pipefail
mkdir -p gpurun_out/c15
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c15/pytest.log 2>&1 || { tail -30 gpurun_out/c15/pytest.log; exit 1; }
tail -1 gpurun_out/c15/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c15/smoke.log 2>&1 || { tail -20 gpurun_out/c15/smoke.log; exit 1; }
tail -2 gpurun_out/c15/smoke.log
for w in 8 12; do
  IGN_BUILD_PROF=1 IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py --train --fresh-batches --steps 40 --input-workers $w > gpurun_out/c15/w$w.json 2> gpurun_out/c15/w$w.err || exit 1
  echo "w$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c15/w$w.json) $(grep -o '"close": [0-9.]*' gpurun_out/c15/w$w.json) oom-trims $(grep -c 'ign-pool' gpurun_out/c15/w$w.err)"
done
