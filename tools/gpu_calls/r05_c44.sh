# final round-5 checks: smoke(), full GPU suite, bench sweep, training-step trace
set -o pipefail
mkdir -p gpurun_out/c44
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/c44/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c44/pytest_gpu.log 2>&1 || exit 1
bash tools/bench_sweep.sh > gpurun_out/c44/sweep_log.txt 2>&1 || exit 1
