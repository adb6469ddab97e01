set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/full gpurun_out/ab34
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full/gpu_tests.log 2>&1 || { tail -30 gpurun_out/full/gpu_tests.log; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/full/bench.log 2>&1 || exit 1
timeout -k 10 300 python tools/ab_bitwise.py tl db --train > gpurun_out/ab34/bitwise_train.log 2>&1 || exit 1
for n in tl db; do
  IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab34/$n -o $n --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu > gpurun_out/ab34/$n.log 2>&1 || exit 1
done
for r in 1 2; do
  for n in tl db; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab34/t-$n-$r.json 2>&1 || exit 1
  done
done
timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab34/t-default.json 2>&1 || exit 1
IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_db.so timeout -k 10 600 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab34/train_tests_db.log 2>&1 || exit 1
