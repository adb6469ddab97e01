set -o pipefail
mkdir -p gpurun_out/ab12
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab12/t-$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-timing > gpurun_out/ab12/nt-$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --streams 1 --no-timing > gpurun_out/ab12/nt1-$r.log 2>&1 || exit 1
done
