# round 6 call 11: fresh-batch training with the loss on logged steps only (no per-step host wait):
# 8 / 10 / 12 builders, the GIL switch interval at Python's 5 ms and at 0.5 ms; the resident-batch step beside
set -o pipefail
mkdir -p gpurun_out/c11
timeout -k 10 300 python3 bench.py --train > gpurun_out/c11/train.json 2> gpurun_out/c11/train.err || exit 1
echo "train $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c11/train.json)"
for cfg in "w8|8|" "w8g05|8|0.5" "w10|10|" "w12|12|" "w12g05|12|0.5"; do
  n=$(echo $cfg | cut -d'|' -f1); w=$(echo $cfg | cut -d'|' -f2); g=$(echo $cfg | cut -d'|' -f3)
  IGN_BUILD_PROF=1 IGN_STEP_PROF=1 IGN_GIL_SWITCH_MS=$g timeout -k 10 400 python3 bench.py --train --fresh-batches --input-workers $w \
    > gpurun_out/c11/$n.json 2> gpurun_out/c11/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c11/$n.json) $(grep -o '"input_pipeline": {[^}]*}[^}]*}' gpurun_out/c11/$n.json)"
done
