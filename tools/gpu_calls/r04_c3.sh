# round 4, call 3: the ordered update's next-tile state prefetch (LDS-DMA, hpf = default tree) against
# the previous tile prologue (nohpf = -DIGN_SEQ_NO_HPF): bitwise check, parity tests, A/B
# (reverted: bitwise equal, 1-2 % slower per launch; DESIGN.md round-4 notes)
set -o pipefail
O=gpurun_out/c3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_bitwise.py nohpf hpf > $O/bitwise_rn.log 2>&1 || { tail -20 $O/bitwise_rn.log; exit 1; }
tail -3 $O/bitwise_rn.log
timeout -k 10 300 python -u tools/ab_bitwise.py nohpf hpf --model qsize > $O/bitwise_qs.log 2>&1 || { tail -20 $O/bitwise_qs.log; exit 1; }
tail -3 $O/bitwise_qs.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread \
  > $O/test_parity.log 2>&1 || { tail -30 $O/test_parity.log; exit 1; }
tail -2 $O/test_parity.log
bash tools/ab_lib.sh "hpf nohpf" 3 --steps 20 > $O/ab_hpf.log 2>&1 || { tail -20 $O/ab_hpf.log; exit 1; }
cat $O/ab_hpf.log
bash tools/ab_lib.sh "hpf nohpf" 2 --steps 20 --streams 1 > $O/ab_hpf_s1.log 2>&1 || { tail -20 $O/ab_hpf_s1.log; exit 1; }
cat $O/ab_hpf_s1.log
