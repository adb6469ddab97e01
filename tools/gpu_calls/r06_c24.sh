# round 6 call 24: the training step's kernel breakdown on the final tree (rocprofv3 kernel trace of
# bench.py --train) for profiles/r06/routenet_synth50_x512_train/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c24
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c24/train -o train --output-format csv -- \
  python3 bench.py --train --steps 10 --warmup 3 > gpurun_out/c24/train.json 2> gpurun_out/c24/train.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/c24/train.json
