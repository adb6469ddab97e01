# round 6 call 8: where seq_gru_bwd (the ordered backward, 5.5 ms of the 16.2 ms training step) spends
# its time -- timing-only ablations (wrong gradients): no per-step row loads, no gate recompute
# transcendentals, no ga stores, no dU contraction; kernel trace of the training bench for each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c08
for cfg in "base|IGN_X=0" "noload|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_bnoload.so" \
           "nogate|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_bnogate.so" \
           "noga|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_bnoga.so" \
           "nodu|IGN_AB_LIB=1 IGN_LIB_PATH=$PWD/ignnition_amd/ab/lib_bnodu.so"; do
  n=${cfg%%|*}; e=${cfg#*|}
  env $e timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/c08/$n -o $n --output-format csv -- \
    python3 bench.py --train --steps 5 --warmup 2 > gpurun_out/c08/$n.json 2> gpurun_out/c08/$n.err || exit 1
  echo "$n $(grep -h 'seq_gru_bwd' gpurun_out/c08/$n/*kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done
