#!/bin/bash
# Training tests, then the training step with the f32 / split-bf16 gate recompute in seq_gru_bwd.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_train.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_train.log; exit 1; }
tail -2 gpurun_out/pytest_train.log
for v in 0 1; do
  IGN_BWD_BF=$v timeout -k 10 200 python bench.py --train --steps 10 --warmup 2 --no-cpu > gpurun_out/bbwd_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/bbwd_$v.log; exit 1; }
  tail -1 gpurun_out/bbwd_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bwd_bf=$v', d['ms_per_step'])"
done
bash tools/train_prof.sh || exit 1
python tools/train_breakdown.py gpurun_out/prof_train 3 | head -6
