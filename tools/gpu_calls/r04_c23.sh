# round 4, call 23: kernel trace + PMC passes of GEANT2 x512 on the resident forward (profiles/collect.sh),
# then the training step's kernel trace (tools/train_prof.sh without its test pass)
set -o pipefail
BENCH_ARGS="--topology geant2 --steps 3 --warmup 1 --no-cpu --no-edge-cut" TRACE_ARGS="--topology geant2 --no-edge-cut" \
  bash profiles/collect.sh r04_geant2_resident &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
rm -rf gpurun_out/prof_train && mkdir -p gpurun_out/prof_train &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/prof_train.log 2>&1 &&
python3 tools/train_breakdown.py gpurun_out/prof_train > gpurun_out/train_breakdown.txt 2>&1; head -24 gpurun_out/train_breakdown.txt
