# fresh-batch training, same box: resident tables in the builder (EAGER) x resident training forward (RT)
set -o pipefail
mkdir -p gpurun_out/c26
TIMEFORMAT='cpu: %R real %U user %S sys'
for rep in 1 2; do
  for cfg in "IGN_RESIDENT_EAGER=0 IGN_RESIDENT_TRAIN=0" "IGN_RESIDENT_EAGER=1 IGN_RESIDENT_TRAIN=1" "IGN_RESIDENT_EAGER=0 IGN_RESIDENT_TRAIN=1" "IGN_RESIDENT_EAGER=1 IGN_RESIDENT_TRAIN=0"; do
    tag=$(echo $cfg | tr -dc '0-9')_$rep
    { time env $cfg timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 15 --warmup 3 --no-cpu --no-edge-cut \
      > gpurun_out/c26/fresh_$tag.json 2> gpurun_out/c26/fresh_$tag.err ; } 2> gpurun_out/c26/time_$tag.txt || exit 1
  done
done
