# resident SAVE training forward: parity against the per-MP training launches, then the --train A/B
set -o pipefail
mkdir -p gpurun_out/c17
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_training.py \
  -k "resident or autograd or consumes or reduces" > gpurun_out/c17/pytest.log 2>&1 || exit 1
for v in 1 0 1 0; do
  IGN_RESIDENT_TRAIN=$v timeout -k 10 300 python -u bench.py --train --steps 20 --warmup 5 --no-cpu \
    > gpurun_out/c17/train_$v.json 2> gpurun_out/c17/train_$v.err || exit 1
  tail -1 gpurun_out/c17/train_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'])"
done
