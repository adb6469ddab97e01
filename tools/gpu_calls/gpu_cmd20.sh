set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab20
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab20/t.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu > gpurun_out/ab20/il-$r.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --no-cpu --no-interleave > gpurun_out/ab20/ni-$r.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab20/trace -o trace --output-format csv -- python3 bench.py --no-cpu > gpurun_out/ab20/trace.log 2>&1
