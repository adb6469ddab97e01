set -o pipefail
mkdir -p gpurun_out/c4
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --timeout 200 --timeout-method thread -k "lane_walk_only" > gpurun_out/c4/test.log 2>&1 || echo "test failed"
for spec in "default|--no-cpu" "qsize|--model qsize --no-edge-cut --no-cpu" "geant2|--topology geant2 --no-edge-cut --no-cpu" "qsize_batched|--model qsize --no-edge-cut --no-cpu"; do
  name=${spec%%|*}; args=${spec#*|}
  if [ $name = qsize_batched ]; then export IGN_RESIDENT=0; fi
  timeout -k 10 300 python -u bench.py $args > gpurun_out/c4/$name.json 2> gpurun_out/c4/$name.err || { echo "$name failed"; exit 1; }
  echo "$name done"
done
