set -o pipefail
mkdir -p gpurun_out/ab23
timeout -k 10 400 python tools/ab_bitwise.py slp noslp > gpurun_out/ab23/bitwise.log 2>&1 || exit 1
bash tools/ab_lib.sh "slp noslp" 3 > gpurun_out/ab23/s2.log 2>&1 || exit 1
bash tools/ab_lib.sh "slp noslp" 2 --streams 1 > gpurun_out/ab23/s1.log 2>&1 || exit 1
for r in 1 2; do
  for n in slp noslp; do
    IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 200 python bench.py --no-cpu --train --steps 10 > gpurun_out/ab23/t-$n-$r.json 2>&1 || exit 1
  done
done
