# fresh-batch training: batch destroy's phases inside the library vs the Python close around it
set -o pipefail
mkdir -p gpurun_out/c29
IGN_STEP_PROF=1 IGN_BUILD_PROF=1 timeout -k 10 300 python -u bench.py --train --fresh-batches --steps 15 --warmup 3 --no-cpu --no-edge-cut \
    > gpurun_out/c29/fresh.json 2> gpurun_out/c29/fresh.err || exit 1
