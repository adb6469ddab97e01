#!/bin/bash
# RouteNet synth50 x512: ordered-update variants side by side (seq_gru ms per launch from the warm-up timing)
mkdir -p gpurun_out
for cfg in "IGN_SEQ_VARIANT=4" "IGN_SEQ_VARIANT=6" "IGN_SEQ_VARIANT=4 IGN_XCD_REMAP=1" "IGN_SEQ_VARIANT=4"; do
  env $cfg timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bs.log 2>&1 || { echo "bench $cfg failed"; tail -20 gpurun_out/bs.log; exit 1; }
  tail -1 gpurun_out/bs.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$cfg', round(d['ms_per_step'],3), r['kernel'], r['avg_launch_ms'])"
done
