#!/bin/bash
# windowed-sum parity tests, then Q-size x512 with the auto rule (default) vs forced off / on
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "windowed or qsize or Q_size" > gpurun_out/pt_win.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pt_win.log; exit 1; }
grep -E "passed|failed" gpurun_out/pt_win.log | tail -2
for cfg in "IGN_SUM_WINDOW=-1" "IGN_SUM_WINDOW=0" "IGN_SUM_WINDOW=1"; do
  env $cfg timeout -k 10 200 python bench.py --model qsize --steps 10 --warmup 2 --no-cpu --no-edge-cut > gpurun_out/bq.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/bq.log; exit 1; }
  tail -1 gpurun_out/bq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; w=r['warmup_kernels']; print('$cfg', round(d['ms_per_step'],3), {k: round(v['ms_total']/2,3) for k,v in w.items()})"
done
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-edge-cut > gpurun_out/br.log 2>&1 && tail -1 gpurun_out/br.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('routenet default', round(d['ms_per_step'],3))"
