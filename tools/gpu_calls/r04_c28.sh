# round 4, call 28: the resident tables built at the first ign_forward instead of at batch
# creation (training batches no longer pay for them): resident parity tests, the fresh-batch
# training line, the headline
set -o pipefail
O=gpurun_out/c28
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "resident or hip_graph" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for spec in "train_fresh|--train --fresh-batches" "default|--no-cpu"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python -u bench.py $args > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('$O/$name.json') if l.startswith('{')][-1]); print('$name', round(d['ms_per_step'],4), d['config'].get('batch_build_s'))"
done
