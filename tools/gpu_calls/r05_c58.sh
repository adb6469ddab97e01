# final round-5 tree after the training changes: smoke(), full GPU suite, bench sweep, training-step trace
set -o pipefail
mkdir -p gpurun_out/c58
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c58/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c58/pytest_gpu.log 2>&1 || exit 1
bash tools/bench_sweep.sh > gpurun_out/c58/sweep_log.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c58/trace -o t --output-format csv -- \
  python3 bench.py --train --steps 5 --warmup 2 --no-cpu --no-edge-cut > gpurun_out/c58/trace.log 2>&1 || exit 1
