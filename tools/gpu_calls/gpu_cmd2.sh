set -o pipefail
mkdir -p gpurun_out/ab2
for r in 1 2; do
  for s in 1 2 3 4; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_rw4.so timeout -k 10 200 python bench.py --no-cpu --streams $s > gpurun_out/ab2/rw4-s$s-$r.json 2>&1 || exit 1
  done
  timeout -k 10 200 python bench.py --no-cpu --streams 2 > gpurun_out/ab2/rw8-s2-$r.json 2>&1 || exit 1
done
