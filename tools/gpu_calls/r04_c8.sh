# round 4, call 8: the pipelined readout (layer 1 of the next row group inside layer 2's chunks):
# bitwise against the phase-by-phase kernel (nopipe), then A/B of waves x row tiles
# (reverted: pipe81 bitwise equal but 0.737 against 0.598 ms per launch on one stream; DESIGN.md round-4 notes)
set -o pipefail
O=gpurun_out/c8
mkdir -p $O
export TMPDIR=/tmp
for n in pipe81 pipe41 pipe42; do
  timeout -k 10 300 python -u tools/ab_bitwise.py nopipe $n > $O/bitwise_$n.log 2>&1 || { tail -20 $O/bitwise_$n.log; exit 1; }
  tail -1 $O/bitwise_$n.log
done
timeout -k 10 300 python -u tools/ab_bitwise.py nopipe pipe81 --model qsize > $O/bitwise_qs.log 2>&1 || { tail -20 $O/bitwise_qs.log; exit 1; }
tail -1 $O/bitwise_qs.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "hidden or readout or split" \
  > $O/test_parity.log 2>&1 || { tail -30 $O/test_parity.log; exit 1; }
tail -1 $O/test_parity.log
bash tools/ab_lib.sh "nopipe pipe81 pipe41 pipe42" 2 --steps 20 > $O/ab_pipe.log 2>&1 || { tail -20 $O/ab_pipe.log; exit 1; }
cat $O/ab_pipe.log
bash tools/ab_lib.sh "nopipe pipe81 pipe41 pipe42" 1 --steps 20 --streams 1 > $O/ab_pipe_s1.log 2>&1 || { tail -20 $O/ab_pipe_s1.log; exit 1; }
cat $O/ab_pipe_s1.log
