# round 6 call 23: batch-builder threads pinned to CPU pairs of one NUMA node (IGN_PIN_BUILDERS,
# default on) vs free to migrate: fresh-batch training interleaved on one box, and the resident step
set -o pipefail
mkdir -p gpurun_out/c23
for n in pin1 free1 pin2 free2 train; do
  a="--train --fresh-batches --steps 40"; e="IGN_PIN_BUILDERS=1"
  case $n in free*) e="IGN_PIN_BUILDERS=0";; train) a="--train --steps 40";; esac
  env $e IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py $a > gpurun_out/c23/$n.json 2> gpurun_out/c23/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c23/$n.json)"
done
REPS=3 THREADS=8 PIN=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c23/host8_pin.txt 2>&1 || exit 1
tail -1 gpurun_out/c23/host8_pin.txt
