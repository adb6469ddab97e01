# round 6 call 12: the resident tables built by a counting sort and two threads per builder: the
# resident parity tests, then fresh-batch training with 8 builders at IGN_BUILD_THREADS 1 / 2 / 4
set -o pipefail
mkdir -p gpurun_out/c12
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "resident or graph_groups or pooled or fused_readout" > gpurun_out/c12/pytest.log 2>&1 || { tail -40 gpurun_out/c12/pytest.log; exit 1; }
tail -1 gpurun_out/c12/pytest.log
for t in 2 1 4; do
  IGN_BUILD_THREADS=$t IGN_BUILD_PROF=1 IGN_STEP_PROF=1 timeout -k 10 400 python3 bench.py --train --fresh-batches > gpurun_out/c12/bt$t.json 2> gpurun_out/c12/bt$t.err || exit 1
  echo "threads $t $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c12/bt$t.json) $(grep -o '"ms_waiting_for_batch": [0-9.]*' gpurun_out/c12/bt$t.json)"
  grep "batch sections" gpurun_out/c12/bt$t.err | awk '{for(i=1;i<=NF;i++){if($i=="mp0")a+=$(i+1); if($i=="mp1+readout")b+=$(i+1); if($i=="tables")c+=$(i+1)}; n++} END{print "  n",n,"mp0",a/n,"mp1+ro",b/n,"resident",c/n}'
done
timeout -k 10 300 python3 bench.py --train > gpurun_out/c12/train.json 2> gpurun_out/c12/train.err || exit 1
echo "train $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c12/train.json)"
