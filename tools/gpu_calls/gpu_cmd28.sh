set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/ab28
for n in sv nosv; do
  IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab28/$n -o $n --output-format csv -- python3 bench.py --train --steps 2 --warmup 1 --no-cpu > gpurun_out/ab28/$n.log 2>&1 || exit 1
done
