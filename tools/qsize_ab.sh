#!/bin/bash
# Q-size synth50 x512: sum-update layouts (default / split gather + GRU / windowed) side by side.
mkdir -p gpurun_out
for cfg in "default" "IGN_SUM_SPLIT=1" "IGN_SUM_WINDOW=1"; do
  envs=""; [ "$cfg" != default ] && envs="$cfg"
  env $envs timeout -k 10 200 python bench.py --model qsize --steps 10 --warmup 2 --no-cpu > gpurun_out/bq.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/bq.log; exit 1; }
  tail -1 gpurun_out/bq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; w=r['warmup_kernels']; print('$cfg', round(d['ms_per_step'],3), {k: round(v['ms_total']/2,3) for k,v in w.items()})"
done
