# round 6 call 29: csr_gather_add with 16 rows per batch in flight instead of 8 (IGN_GATHER_BATCH,
# A/B libraries, the same additions in the same order): gradients bitwise, then the training step
# and the gather's kernel time, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c29
timeout -k 10 300 python3 tools/ab_bitwise.py gb8 gb16 --train > gpurun_out/c29/bitwise.txt 2>&1 || { cat gpurun_out/c29/bitwise.txt; exit 1; }
tail -2 gpurun_out/c29/bitwise.txt
for n in gb8 gb16 gb8 gb16; do
  k=$n$(ls gpurun_out/c29 | grep -c "^$n")
  IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_$n.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c29/$k -o $k --output-format csv -- \
    python3 bench.py --train --steps 20 --warmup 3 > gpurun_out/c29/$k.json 2> gpurun_out/c29/$k.err || exit 1
  echo "$k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c29/$k.json) $(grep -h 'csr_gather_add_kernel<1, true' gpurun_out/c29/$k/${k}_kernel_stats.csv | cut -d, -f4 | tr '\n' ' ')"
done
