# round 6 call 32: the GPU suite and smoke() on the final tree (after the reverted probes)
set -o pipefail
mkdir -p gpurun_out/c32
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c32/pytest.log 2>&1 || { tail -30 gpurun_out/c32/pytest.log; exit 1; }
tail -1 gpurun_out/c32/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c32/smoke.log 2>&1 || { tail -20 gpurun_out/c32/smoke.log; exit 1; }
tail -2 gpurun_out/c32/smoke.log
