set -o pipefail
mkdir -p gpurun_out/ab17
for r in 1 2; do
  for n in g4 g8 g16; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab17/$n-$r.json 2>&1 || exit 1
  done
done
