# round 6 call 21: the host block cache reusing blocks up to two size classes up: the GPU suite, the
# builders' host sections, then fresh-batch training A/B'd against the resident step on one box
set -o pipefail
mkdir -p gpurun_out/c21
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c21/pytest.log 2>&1 || { tail -30 gpurun_out/c21/pytest.log; exit 1; }
tail -1 gpurun_out/c21/pytest.log
IGN_BUILD_PROF_FINE=1 REPS=4 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c21/host1.txt 2> gpurun_out/c21/host1.err || exit 1
tail -1 gpurun_out/c21/host1.txt
grep "fine sections" gpurun_out/c21/host1.err | tail -2
REPS=3 THREADS=8 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c21/host8.txt 2> gpurun_out/c21/host8.err || exit 1
tail -1 gpurun_out/c21/host8.txt
for n in fresh1 train fresh2; do
  a="--train --steps 40"; case $n in fresh*) a="--train --fresh-batches --steps 40";; esac
  IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py $a > gpurun_out/c21/$n.json 2> gpurun_out/c21/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c21/$n.json)"
done
