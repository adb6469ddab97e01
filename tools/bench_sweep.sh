#!/bin/bash
# One bench line per workload (GPU box, repo root): gpurun_out/sweep/<name>.json
set -o pipefail
mkdir -p gpurun_out/sweep
for spec in "default|" "synthetic|--model synthetic" "qsize|--model qsize --no-edge-cut" "geant2|--topology geant2 --no-edge-cut" \
            "train|--train" "train_fresh|--train --fresh-batches"; do
  name=${spec%%|*}; args=${spec#*|}
  timeout -k 10 400 python -u bench.py $args > gpurun_out/sweep/$name.json 2> gpurun_out/sweep/$name.err || {
    echo "$name failed"; exit 1; }
  echo "$name done"
done
