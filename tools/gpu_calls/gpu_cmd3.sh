set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/bench3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --streams 1 > gpurun_out/bench3_s1.log 2>&1 || exit 1
mkdir -p gpurun_out/prof3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3/trace -o trace --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof3/trace.log 2>&1
