set -e
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_training.py -x -q > gpurun_out/pytest_train.log 2>&1
rm -rf gpurun_out/prof_train && mkdir -p gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu --no-edge-cut ${BENCH_EXTRA:-} > gpurun_out/prof_train.log 2>&1
