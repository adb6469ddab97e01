set -e
mkdir -p gpurun_out
for o in 0 1 2; do for x in 0 1; do
IGN_SUM_ORDER=$o IGN_XCD_REMAP=$x timeout -k 10 200 python bench.py --model synthetic --steps 5 --warmup 1 --no-cpu > gpurun_out/sw_$o$x.log 2>&1
done; done
