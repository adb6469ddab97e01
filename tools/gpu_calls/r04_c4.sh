# round 4, call 4: PMC + trace profiles of Q-size and GEANT2 x512 with the round-4 defaults (segmented
# node sum, 4 GEANT2 sub-batches); training-step kernel trace; bench sweep of every workload
set -o pipefail
O=gpurun_out/c4
mkdir -p $O
export TMPDIR=/tmp
BENCH_ARGS="--model qsize --no-cpu --no-edge-cut --steps 3 --warmup 1" TRACE_ARGS="--model qsize --no-cpu --no-edge-cut" \
  bash profiles/collect.sh r04_qsize_final || exit 1
BENCH_ARGS="--topology geant2 --no-cpu --no-edge-cut --steps 3 --warmup 1" TRACE_ARGS="--topology geant2 --no-cpu --no-edge-cut" \
  bash profiles/collect.sh r04_geant2_final || exit 1
rm -rf gpurun_out/prof_train && mkdir -p gpurun_out/prof_train
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o train --output-format csv -- \
  python3 bench.py --train --steps 3 --warmup 1 --no-cpu --no-edge-cut > gpurun_out/prof_train.log 2>&1 || { tail -20 gpurun_out/prof_train.log; exit 1; }
python3 tools/train_breakdown.py gpurun_out/prof_train 4 > $O/train_breakdown.txt && cat $O/train_breakdown.txt
mkdir -p gpurun_out/sweep
for spec in "qsize|--model qsize --no-edge-cut" "geant2|--topology geant2 --no-edge-cut" "synthetic|--model synthetic" \
            "train|--train --no-cpu"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 300 python -u bench.py $args > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || {
    echo "$name failed"; tail -20 gpurun_out/sweep/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sweep/$name.json').read().splitlines()[-1]); print('$name', round(d['ms_per_step'],4), '%.4g' % d['value'])"
done
