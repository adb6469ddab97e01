# round 6 call 10: the fresh-batch training pipeline on the round-6 tree: resident-batch step, fresh-batch
# step with the step's host phases (IGN_STEP_PROF) and the builders' scopes (IGN_BUILD_PROF), the host
# stages alone with 1 and 8 builder threads
set -o pipefail
mkdir -p gpurun_out/c10
timeout -k 10 300 python3 bench.py --train > gpurun_out/c10/train.json 2> gpurun_out/c10/train.err || exit 1
IGN_STEP_PROF=1 IGN_BUILD_PROF=1 timeout -k 10 400 python3 bench.py --train --fresh-batches > gpurun_out/c10/fresh.json 2> gpurun_out/c10/fresh.err || exit 1
THREADS=1 REPS=3 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c10/host1.txt 2>&1 || exit 1
THREADS=8 REPS=2 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c10/host8.txt 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/c10/train.json gpurun_out/c10/fresh.json
grep -o '"input_pipeline": {[^}]*}[^}]*}' gpurun_out/c10/fresh.json
tail -1 gpurun_out/c10/host1.txt; tail -1 gpurun_out/c10/host8.txt
