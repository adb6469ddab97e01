#!/bin/bash
# training parity tests, then the default training step line
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_train.log; exit 1; }
tail -1 gpurun_out/pytest_train.log
timeout -k 10 200 python bench.py --train --steps 10 --warmup 2 --no-cpu > gpurun_out/btrain.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/btrain.log; exit 1; }
tail -1 gpurun_out/btrain.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train', d['ms_per_step'])"
