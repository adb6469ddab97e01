# round 6 call 2: kernel traces of the headline at 1 and 2 sub-batch streams (resident / readout durations)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c02
for s in 1 2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c02/s$s -o s$s --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --streams $s --steps 10 --warmup 3 > gpurun_out/c02/s$s.json 2> gpurun_out/c02/s$s.err || exit 1
done
