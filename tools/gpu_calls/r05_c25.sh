# fresh-batch training step: kernel trace (which kernels grow on fresh batches), and the non-resident training forward
set -o pipefail
mkdir -p gpurun_out/c25
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
IGN_RESIDENT_TRAIN=0 timeout -k 10 400 python -u bench.py --train --fresh-batches --steps 12 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c25/fresh_rt0.json 2> gpurun_out/c25/fresh_rt0.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c25/trace -o fresh --output-format csv -- \
  python3 bench.py --train --fresh-batches --steps 8 --warmup 2 --no-cpu --no-edge-cut > gpurun_out/c25/trace.log 2>&1 || exit 1
