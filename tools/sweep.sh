# usage: SWEEP="A=1,B=2 A=2,B=3" [BENCH="--model synthetic ..."] bash tools/sweep.sh
set -e
mkdir -p gpurun_out/sweep
BENCH=${BENCH:-"--model synthetic --steps 5 --warmup 1 --no-cpu"}
for combo in $SWEEP; do
  envs=$(echo $combo | tr ',' ' ')
  env $envs timeout -k 10 200 python bench.py $BENCH > gpurun_out/sweep/$combo.log 2>&1
done
