# round 6 call 9: the tree as committed + bench step account: smoke, the full GPU suite, the default bench line
set -o pipefail
mkdir -p gpurun_out/c09
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c09/smoke.log 2>&1 || { tail -20 gpurun_out/c09/smoke.log; exit 1; }
tail -2 gpurun_out/c09/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/c09/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/c09/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/c09/pytest_gpu.log
timeout -k 10 400 python -u bench.py > gpurun_out/c09/default.json 2> gpurun_out/c09/default.err || exit 1
python3 tools/show_bench.py gpurun_out/c09/default.json 2>/dev/null | head -20 || true
