set -o pipefail
mkdir -p gpurun_out/ab5
for r in 1 2; do
  for n in s3 s4 s4b3; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab5/$n-$r.json 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab5/$n-$r.json; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab5/$n-$r.json') if l.startswith('{')][-1]); print('$n', d['ms_per_step'])"
  done
done
IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_s4.so timeout -k 10 300 python -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab5/train_tests_s4.log 2>&1 || exit 1
IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_s4b3.so timeout -k 10 300 python -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab5/train_tests_s4b3.log 2>&1 || exit 1
IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_s4.so timeout -k 10 300 python tools/probes/train_two_stream.py 10 > gpurun_out/ab5/two_stream.log 2>&1
