set -o pipefail
mkdir -p gpurun_out/ab16
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab16/train_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in fbase fold; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab16/$n-$r.json 2>&1 || exit 1
  done
done
