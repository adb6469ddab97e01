set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab30
for n in base late wide; do
  IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab30/$n -o $n --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu > gpurun_out/ab30/$n.log 2>&1 || exit 1
done
for r in 1 2; do
  for n in base late wide; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab30/t-$n-$r.json 2>&1 || exit 1
  done
done
for n in late wide; do
  IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab30/train_tests_$n.log 2>&1 || exit 1
done
