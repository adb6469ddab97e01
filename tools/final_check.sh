#!/bin/bash
# Round-end check: full GPU tests, smoke, the default bench line and the other configs' lines.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
timeout -k 10 300 python bench.py --model qsize > gpurun_out/bench_qsize.log 2>&1 || { echo "bench qsize failed"; tail -20 gpurun_out/bench_qsize.log; exit 1; }
timeout -k 10 300 python bench.py --topology geant2 > gpurun_out/bench_geant2.log 2>&1 || { echo "bench geant2 failed"; tail -20 gpurun_out/bench_geant2.log; exit 1; }
for f in default qsize geant2; do tail -1 gpurun_out/bench_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$f', round(d['ms_per_step'],3), '%.3g' % d['value'], r['kernel'], r['frac'], d['cpu_baseline']['value'])"; done
