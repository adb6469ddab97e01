# round 6 call 6: where readout_h32 (4 waves, 3-slot ring) spends its time -- timing-only ablations
# (wrong results): no W2 DMA, no layer-2 activation, no layer-1 activation; readout_h16 without DMA
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c06
for cfg in "v5|IGN_READOUT_VARIANT=5" "v4|IGN_READOUT_VARIANT=4" "nodma|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_nodma.so" \
           "noepi|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_noepi.so" "nol1v|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_nol1v.so" \
           "h16nodma|IGN_READOUT_VARIANT=4 IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_h16nodma.so"; do
  n=${cfg%%|*}; e=${cfg#*|}
  env $e timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c06/$n -o $n --output-format csv -- \
    python3 bench.py --no-cpu --no-edge-cut --streams 1 --steps 10 --warmup 3 > gpurun_out/c06/$n.json 2> gpurun_out/c06/$n.err || exit 1
  echo "$n $(grep -h 'readout_h' gpurun_out/c06/$n/*kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
