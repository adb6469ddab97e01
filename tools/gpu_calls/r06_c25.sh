# round 6 call 25: the training tables' transposed CSRs on the GPU (train_csr.hip): training tests
# (bitwise against the host build), the GPU suite, the builders' host sections, then fresh-batch
# training against the resident step on one box
set -o pipefail
mkdir -p gpurun_out/c25
timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c25/train_tests.log 2>&1 || { tail -30 gpurun_out/c25/train_tests.log; exit 1; }
tail -1 gpurun_out/c25/train_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/c25/pytest.log 2>&1 || { tail -30 gpurun_out/c25/pytest.log; exit 1; }
tail -1 gpurun_out/c25/pytest.log
IGN_BUILD_PROF_FINE=1 REPS=4 THREADS=1 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c25/host1.txt 2> gpurun_out/c25/host1.err || exit 1
tail -1 gpurun_out/c25/host1.txt; grep "fine sections" gpurun_out/c25/host1.err | tail -2
REPS=3 THREADS=8 timeout -k 10 300 python3 tools/host_pipeline_profile.py > gpurun_out/c25/host8.txt 2> gpurun_out/c25/host8.err || exit 1
tail -1 gpurun_out/c25/host8.txt
for n in fresh1 train fresh2 hostcsr; do
  a="--train --fresh-batches --steps 40"; e="IGN_TRAIN_CSR_GPU=1"
  case $n in train) a="--train --steps 40";; hostcsr) e="IGN_TRAIN_CSR_GPU=0";; esac
  env $e IGN_STEP_PROF=1 timeout -k 10 300 python3 bench.py $a > gpurun_out/c25/$n.json 2> gpurun_out/c25/$n.err || exit 1
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c25/$n.json)"
done
