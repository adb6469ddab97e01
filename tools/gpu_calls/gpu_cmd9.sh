set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab9
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_edge_cut.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab9/train_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in tbase tnew; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab9/$n-$r.json 2>&1 || { echo "$n failed"; exit 1; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/ab9/$n-$r.json') if l.startswith('{')][-1]); print('$n', d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab9/prof_train -o train --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu > gpurun_out/ab9/prof_train.log 2>&1
