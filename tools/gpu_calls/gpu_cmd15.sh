set -o pipefail
mkdir -p gpurun_out/ab15
for r in 1 2; do
  timeout -k 10 400 python bench.py --train --fresh-batches --steps 10 > gpurun_out/ab15/def-$r.json 2>&1 || exit 1
  IGN_HOST_CACHE_GB=16 IGN_POOL_CACHE_GB=64 timeout -k 10 400 python bench.py --train --fresh-batches --steps 10 > gpurun_out/ab15/big-$r.json 2>&1 || exit 1
done
nproc > gpurun_out/ab15/nproc.txt; uptime >> gpurun_out/ab15/nproc.txt
for r in 1 2; do
  for n in rbase runroll; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab15/$n-$r.json 2>&1 || exit 1
  done
done
