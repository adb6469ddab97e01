set -o pipefail
mkdir -p gpurun_out/ab21
for r in 1 2; do
  IGN_PERSIST_CAP=2 timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab21/il-c2-$r.log 2>&1 || exit 1
  IGN_PERSIST_CAP=3 timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab21/il-c3-$r.log 2>&1 || exit 1
  IGN_PERSIST_CAP=1 timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab21/il-c1-$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-interleave > gpurun_out/ab21/ni-$r.log 2>&1 || exit 1
done
