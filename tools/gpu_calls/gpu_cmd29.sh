set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab29
for n in sv nt; do
  IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab29/$n -o $n --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu > gpurun_out/ab29/$n.log 2>&1 || exit 1
done
for r in 1 2; do
  for n in sv nt; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab29/t-$n-$r.json 2>&1 || exit 1
  done
done
