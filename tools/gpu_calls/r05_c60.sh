# final tree with the non-temporal ga gather: smoke(), full GPU suite, default / train / fresh lines
set -o pipefail
mkdir -p gpurun_out/c60
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c60/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c60/pytest_gpu.log 2>&1 || exit 1
for spec in "default|" "train|--train" "train_fresh|--train --fresh-batches"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/c60/$name.json 2> gpurun_out/c60/$name.err || exit 1
done
