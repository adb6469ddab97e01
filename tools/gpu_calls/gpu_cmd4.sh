set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/b4-st-$r.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-stagger > gpurun_out/b4-ns-$r.log 2>&1 || exit 1
done
mkdir -p gpurun_out/prof4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4/trace -o trace --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof4/trace.log 2>&1
